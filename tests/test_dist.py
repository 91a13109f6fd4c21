"""Multi-rank path on CPU: world_size 2 (and 3) over gloo, 127.0.0.1 rendezvous.

The collective code of bcos_gpu.parallel (shard plan, count-prefixed frontier all-gather, top-level
completion) runs exactly as on the GPUs; only the per-shard level computation is the oracle here
(the GPU level kernels are covered by tests/test_gpu_hash.py and test_dist_gpu below).  The sharded
root must equal the single-process reference-tree root for every size, including sizes that leave
ranks empty or with partial blocks.
"""
import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_levels(o, hasher, width, leaves, levels):
    cur = leaves
    for _ in range(levels):
        n = cur.shape[0]
        m = math.ceil(n / width)
        off = np.minimum(np.arange(m + 1, dtype=np.uint64) * np.uint64(32 * width), np.uint64(32 * n))
        cur = o.hash_packed(hasher, cur.reshape(-1), off)
    return cur


def _worker(rank, world, port, cases, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "fisco-bcos_amd"))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from bcos_gpu import parallel
    from oracle import oracle as o
    out = []
    for (hasher, width, n, seed) in cases:
        leaves = np.random.default_rng(seed).integers(0, 256, size=(n, 32), dtype=np.uint8)
        L = parallel.choose_levels(n, world, width, target_frontier=4)

        def frontier_fn(lo, hi):
            return torch.from_numpy(_oracle_levels(o, hasher, width, leaves[lo:hi], L).copy())

        def root_fn(frontier):
            return torch.from_numpy(np.frombuffer(o.merkle(hasher, width, frontier.numpy()), dtype=np.uint8).copy())

        r = parallel.sharded_merkle_root(frontier_fn, root_fn, n, width, L, rank, world, "cpu")
        out.append((L, bytes(r.tolist())))
    if rank == 0:
        q.put(out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_tx_root_gloo(oracle, world):
    cases = [(0, 2, 1000, 1), (1, 2, 4097, 2), (0, 16, 100_000, 3), (1, 16, 1000, 4), (0, 2, 5, 5),
             (1, 2, 65536, 6), (0, 4, 777, 7)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cases, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for (hasher, width, n, seed), (L, got) in zip(cases, res):
        leaves = np.random.default_rng(seed).integers(0, 256, size=(n, 32), dtype=np.uint8)
        assert got == oracle.merkle(hasher, width, leaves), (hasher, width, n, L)
    assert any(L > 0 for L, _ in res)


def test_shard_plan_alignment():
    from bcos_gpu import parallel
    for n in (1, 2, 17, 1000, 4097, 1_000_000):
        for world in (1, 2, 4, 8):
            for width in (2, 16):
                L = parallel.choose_levels(n, world, width)
                plan = parallel.shard_plan(n, world, width, L)
                assert plan[0][0] == 0 and plan[-1][1] == n
                for (lo, hi), (lo2, _) in zip(plan, plan[1:]):
                    assert hi == lo2 and lo % (width ** L) == 0
                if L:
                    assert math.ceil(n / width ** L) >= 2


@pytest.mark.gpu
def test_sharded_root_gpu_single_process(gpu, oracle):
    """The GPU frontier/root functions with world = 1 and simulated ranks (one process, one GPU)."""
    from bcos_gpu import device, parallel
    for hasher, width, n in ((0, 2, 1_000_000), (1, 16, 100_000), (0, 2, 20_000)):
        leaves_h = np.random.default_rng(n).integers(0, 256, size=(n, 32), dtype=np.uint8)
        leaves = torch.from_numpy(leaves_h).cuda()
        for world in (2, 8):
            L = parallel.choose_levels(n, world, width)
            plan = parallel.shard_plan(n, world, width, L)
            ff = parallel.gpu_frontier_fn(hasher, width, L, leaves)
            fr = torch.cat([ff(lo, hi) for lo, hi in plan if hi > lo], 0)
            root = parallel.gpu_root_fn(hasher, width)(fr.contiguous())
            torch.cuda.synchronize()
            assert bytes(root.cpu().tolist()) == oracle.merkle(hasher, width, leaves_h, nthreads=16)


def _worker_sync_free(rank, world, port, cases, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "fisco-bcos_amd"))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from bcos_gpu import parallel
    from oracle import oracle as o
    out = []
    for (hasher, width, n, seed) in cases:
        leaves = np.random.default_rng(seed).integers(0, 256, size=(n, 32), dtype=np.uint8)

        def frontier_fn(local, levels, dst):
            dst.copy_(torch.from_numpy(_oracle_levels(o, hasher, width, local.numpy(), levels).copy()))

        def root_fn(frontier, dst):
            dst.copy_(torch.from_numpy(np.frombuffer(o.merkle(hasher, width, frontier.numpy()), dtype=np.uint8).copy()))

        st = parallel.ShardedTxRoot(n, world, rank, width, "cpu", frontier_fn, root_fn)
        lo, hi = st.local_range
        r = st(torch.from_numpy(leaves[lo:hi].copy()))
        r2 = st(torch.from_numpy(leaves[lo:hi].copy()))  # buffers are reused across steps
        out.append((st.levels, bytes(r.tolist()), bytes(r2.tolist())))
    if rank == 0:
        q.put(out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_tx_root_sync_free_gloo(oracle, world):
    """bench.py C4's exchange (parallel.ShardedTxRoot: fixed-size frontiers, one all-gather, on-device
    compaction) equals the single-process root, including ranks with empty shards."""
    cases = [(0, 2, 100_000, 11), (1, 2, 3, 12), (0, 16, 70_000, 13), (1, 2, 1, 14), (0, 2, 131_072, 15)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_sync_free, args=(r, world, port, cases, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for (hasher, width, n, seed), (L, got, got2) in zip(cases, res):
        leaves = np.random.default_rng(seed).integers(0, 256, size=(n, 32), dtype=np.uint8)
        assert got == got2 == oracle.merkle(hasher, width, leaves), (hasher, width, n, L)
    assert any(L > 0 for L, _, _ in res)


@pytest.mark.gpu
def test_sharded_tx_root_gpu_frontier_ranks(gpu, oracle):
    """gpu_sharded_tx_root's frontier (the shard's whole tree through bcosgpu_merkle_root_dev, then its
    level L - 1) for every rank of world 2 / 8, simulated in one process: the gathered frontiers give the
    oracle root; and a shard whose tree ends below level L - 1 takes the per-level path with the same
    nodes as bcosgpu_merkle_frontier_dev."""
    from bcos_gpu import device, parallel
    for hasher, width, n in ((0, 2, 1_000_003), (1, 2, 300_001), (0, 16, 400_000)):
        leaves_h = np.random.default_rng(n + 7).integers(0, 256, size=(n, 32), dtype=np.uint8)
        leaves = torch.from_numpy(leaves_h).cuda()
        for world in (2, 8):
            fronts = []
            for rank in range(world):
                st = parallel.gpu_sharded_tx_root(n, world, rank, hasher, width, "cuda")
                lo, hi = st.local_range
                m = st.counts[rank]
                if m:
                    out = torch.empty((m, 32), dtype=torch.uint8, device="cuda")
                    st.frontier_fn(leaves[lo:hi], st.levels, out)
                    fronts.append(out)
            fr = torch.cat(fronts, 0).contiguous()
            root = parallel.gpu_root_fn(hasher, width)(fr)
            torch.cuda.synchronize()
            assert bytes(root.cpu().tolist()) == oracle.merkle(hasher, width, leaves_h, nthreads=16), (n, world)
    st = parallel.gpu_sharded_tx_root(64, 1, 0, 0, 2, "cuda")
    for k, levels in ((1, 3), (3, 4), (5, 2), (4, 2)):
        small = leaves[:k]
        m = -(-k // 2 ** levels)
        got = torch.empty((m, 32), dtype=torch.uint8, device="cuda")
        st.frontier_fn(small, levels, got)
        want = torch.empty((m, 32), dtype=torch.uint8, device="cuda")
        work = torch.empty((max(2 * -(-k // 2), 1), 32), dtype=torch.uint8, device="cuda")
        device.merkle_frontier(0, 2, small, levels, work, want)
        torch.cuda.synchronize()
        assert torch.equal(got, want), (k, levels)


@pytest.mark.gpu
def test_sharded_tx_root_gpu_world1(gpu, oracle):
    """gpu_sharded_tx_root (bench C4's step) on one GPU equals the oracle root."""
    from bcos_gpu import parallel
    for hasher, width, n in ((0, 2, 1_000_000), (1, 2, 20_001)):
        leaves_h = np.random.default_rng(n + 1).integers(0, 256, size=(n, 32), dtype=np.uint8)
        st = parallel.gpu_sharded_tx_root(n, 1, 0, hasher, width, "cuda")
        lo, hi = st.local_range
        r = st(torch.from_numpy(leaves_h[lo:hi].copy()).cuda())
        torch.cuda.synchronize()
        assert bytes(r.cpu().tolist()) == oracle.merkle(hasher, width, leaves_h, nthreads=16)
