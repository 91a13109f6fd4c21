"""Multi-GPU sharding of the hot path (one process per GPU, torch.distributed over RCCL).

Transactions shard by index with no data-path collective: each rank verifies its own contiguous
range and keeps its verdicts / senders.  The only exchange is the block tx root:
Merkle<H, width> (Merkle.h:170-208) groups every level from index 0, so when rank r's leaf range
starts at a multiple of width^L, its level-L nodes are exactly the reference tree's level-L nodes for
that range.  Each rank computes its frontier on its own GPU, ONE all-gather moves the frontiers
(count-prefixed, fixed-size buffers, a few KB), and every rank finishes the top levels -- so the
root is bit-identical to the single-device / reference root for any leaf count.
"""
import math

import torch
import torch.distributed as dist


def choose_levels(n, world, width, target_frontier=64):
    """Levels computed per shard: the largest L with world * target_frontier * width^L <= n
    (so the gathered frontier stays small but every rank still has whole width^L blocks), and the
    global level-L count >= 2 (the reference tree must have more than L levels)."""
    L = 0
    while True:
        blk = width ** (L + 1)
        if world * target_frontier * blk > n or math.ceil(n / blk) < 2:
            break
        L += 1
    return L


def shard_plan(n, world, width, levels):
    """Contiguous leaf ranges [lo, hi) per rank; every lo is a multiple of width^levels."""
    blk = width ** levels
    per = math.ceil(n / (world * blk)) * blk
    return [(min(r * per, n), min((r + 1) * per, n)) for r in range(world)]


def sharded_merkle_root(frontier_fn, root_fn, n, width, levels, rank, world, dev, group=None):
    """Root of the reference tree over n leaves sharded across `world` ranks.

    frontier_fn(lo, hi) -> uint8 tensor [ceil((hi-lo)/width^levels), 32] on `dev`: this rank's
        level-`levels` nodes (computed on its GPU; for levels == 0 the leaves themselves).
    root_fn(frontier [m, 32]) -> uint8 tensor [32]: Merkle<H, width> root of the frontier.
    """
    plan = shard_plan(n, world, width, levels)
    blk = width ** levels
    lo, hi = plan[rank]
    cap = math.ceil((plan[0][1] - plan[0][0]) / blk) if plan[0][1] > plan[0][0] else 1
    buf = torch.zeros((cap + 1, 32), dtype=torch.uint8, device=dev)  # row 0: count record
    if hi > lo:
        f = frontier_fn(lo, hi)
        m = f.shape[0]
        buf[1:1 + m] = f
    else:
        m = 0
    buf[0, :4] = torch.tensor(list(int(m).to_bytes(4, "big")), dtype=torch.uint8, device=dev)
    gathered = torch.empty((world, cap + 1, 32), dtype=torch.uint8, device=dev)
    if world > 1:
        dist.all_gather_into_tensor(gathered.view(-1), buf.view(-1), group=group)
    else:
        gathered[0] = buf
    parts = []
    for r in range(world):
        cnt = int.from_bytes(bytes(gathered[r, 0, :4].cpu().tolist()), "big")
        if cnt:
            parts.append(gathered[r, 1:1 + cnt])
    frontier = torch.cat(parts, 0).contiguous()
    return root_fn(frontier)


def gpu_frontier_fn(hasher, width, levels, leaves):
    """frontier_fn over a device-resident global leaf tensor (rank-local rows are used)."""
    from . import device

    def fn(lo, hi):
        part = leaves[lo:hi].contiguous()
        if levels == 0:
            return part
        m = math.ceil((hi - lo) / width ** levels)
        work = torch.empty((2 * math.ceil((hi - lo) / width), 32), dtype=torch.uint8, device=leaves.device)
        out = torch.empty((m, 32), dtype=torch.uint8, device=leaves.device)
        device.merkle_frontier(hasher, width, part, levels, work, out)
        return out

    return fn


def gpu_root_fn(hasher, width):
    from . import device

    def fn(frontier):
        m = frontier.shape[0]
        tree = torch.empty((max(device.merkle_size(m, width), 1), 32), dtype=torch.uint8, device=frontier.device)
        root = torch.empty(32, dtype=torch.uint8, device=frontier.device)
        device.merkle_root(hasher, width, frontier, tree, root)
        return root

    return fn


class ShardedTxRoot:
    """The multi-GPU tx root as a preallocated, host-sync-free step (used by bench.py's C4 workload).

    Every rank knows the shard plan, hence every rank's frontier size, so the exchange needs no count
    records and no device->host read: the rank's level-L nodes are written straight into its fixed-size
    send buffer, ONE all_gather_into_tensor (RCCL over xGMI on the GPU box, gloo in the CPU tests) moves
    them, an index_select compacts the concatenated frontier on the device, and the top levels run on
    the device (bcosgpu_merkle_root_dev).  `frontier_fn(local_leaves, levels, out)` and
    `root_fn(frontier, root_out)` are injectable so the same exchange logic runs on CPU under gloo.
    """

    def __init__(self, n, world, rank, width, dev, frontier_fn, root_fn, levels=None, group=None):
        self.n, self.world, self.rank, self.width, self.group = n, world, rank, width, group
        self.levels = choose_levels(n, world, width) if levels is None else levels
        self.plan = shard_plan(n, world, width, self.levels)
        blk = width ** self.levels
        self.counts = [math.ceil((hi - lo) / blk) if hi > lo else 0 for lo, hi in self.plan]
        self.cap = max(max(self.counts), 1)
        self.send = torch.zeros((self.cap, 32), dtype=torch.uint8, device=dev)
        self.recv = torch.zeros((world * self.cap, 32), dtype=torch.uint8, device=dev)
        idx = [r * self.cap + j for r, c in enumerate(self.counts) for j in range(c)]
        self.index = torch.tensor(idx, dtype=torch.int64, device=dev)
        self.frontier = torch.empty((len(idx), 32), dtype=torch.uint8, device=dev)
        self.root = torch.empty(32, dtype=torch.uint8, device=dev)
        self.frontier_fn, self.root_fn = frontier_fn, root_fn

    @property
    def local_range(self):
        return self.plan[self.rank]

    def __call__(self, local_leaves):
        """local_leaves: this rank's rows [lo, hi) of the leaf vector -> the global root (device tensor)."""
        m = self.counts[self.rank]
        if m:
            if self.levels == 0:
                self.send[:m].copy_(local_leaves)
            else:
                self.frontier_fn(local_leaves, self.levels, self.send[:m])
        if self.world > 1:
            dist.all_gather_into_tensor(self.recv, self.send, group=self.group)
        else:
            self.recv.copy_(self.send)
        torch.index_select(self.recv, 0, self.index, out=self.frontier)
        self.root_fn(self.frontier, self.root)
        return self.root


def gpu_sharded_tx_root(n, world, rank, hasher, width, dev, group=None):
    """ShardedTxRoot over libbcosgpu.so: frontier and top levels on the GPU."""
    from . import device

    shard = shard_plan(n, world, width, choose_levels(n, world, width))[rank]
    m = max(shard[1] - shard[0], 1)
    # the shard's whole tree in one call (bcosgpu_merkle_root_dev: the one-launch / subtree + climb
    # kernels), whose level `levels - 1` is the frontier -- the shard starts on a width^levels boundary, so
    # its first `levels` levels are exactly the reference tree's nodes over its range; the per-level
    # frontier launches (bcosgpu_merkle_frontier_dev) took ~0.3 ms of C4's 12.8 ms step
    shard_tree = torch.empty((max(device.merkle_size(m, width), 1), 32), dtype=torch.uint8, device=dev)
    shard_root = torch.empty(32, dtype=torch.uint8, device=dev)
    work = torch.empty((max(2 * math.ceil(m / width), 1), 32), dtype=torch.uint8, device=dev)
    tree = {}

    def frontier_fn(leaves, levels, out):
        k = leaves.shape[0]
        pos, c, prev = 0, k, k
        for lv in range(levels):  # entry index of level `levels - 1`'s count record in the shard's tree
            prev, c = c, -(-c // width)
            if lv < levels - 1:
                pos += c + 1
        if prev <= 1:  # the shard's tree ends below level `levels - 1` (a small last shard, whose nodes
            # the reference still hashes one child at a time): the per-level path
            device.merkle_frontier(hasher, width, leaves, levels, work, out)
            return
        device.merkle_root(hasher, width, leaves, shard_tree, shard_root)
        out.copy_(shard_tree[pos + 1:pos + 1 + c])

    def root_fn(frontier, root):
        m = frontier.shape[0]
        if m not in tree:
            tree[m] = torch.empty((max(device.merkle_size(m, width), 1), 32), dtype=torch.uint8, device=dev)
        device.merkle_root(hasher, width, frontier, tree[m], root)

    return ShardedTxRoot(n, world, rank, width, dev, frontier_fn, root_fn, group=group)
