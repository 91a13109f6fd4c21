#!/usr/bin/env python3
"""bench.py -- BASELINE.json's metric on MI355X: "secp256k1 recover & SM2 verify sigs/sec at 1/8 GPUs;
Merkle root GB/s".  One JSON line (rank 0).

`value` (the headline, BASELINE.json configs[1], "C2"): per GPU a batch of 10,000 synthetic
secp256k1-signed transactions resident in HBM; one step = one pass of the hot path over the batch:
Keccak256 tx hash of each preimage (TarsHashable.h:16-41) + ECDSA public-key recovery
(Secp256k1Crypto.cpp:79-93) + sender = right160(Keccak256(pub)) (Transaction.h:68-82), i.e.
bcosgpu_tx_verify_batch_dev.  Multi-GPU: one process per GPU, each verifies its own shard (weak
scaling, no data-path collective); value = txs of all ranks / max-over-ranks wall time.  Exactly
--steps steps are timed; the warm-up runs at least --warmup steps AND --warm-seconds of back-to-back
launches so the clock has settled under load before the timed region starts.

Sub-legs in the same line (`legs`), each timed for >= --leg-seconds of back-to-back steps:
  c2sm2  C2's size on the guomi suite: 10k SM2/SM3 txs per GPU (the SM2 pair kernel; weak scaling).
  c3  configs[2]: 1M SM2/SM3 txs per GPU: SM3 tx hash + SM2 verify + sender (weak scaling).
  c4  configs[3]: 1M secp256k1 txs in TOTAL sharded over the ranks + the block tx root (width-2
      Keccak Merkle, BlockImpl.h:111-154): per-rank frontier, ONE RCCL all-gather, top levels on
      every rank (strong scaling).
  c5  configs[4] (with --legs ...,c5): PBFT block-verify replay, 64 blocks x 20k txs sharded by block:
      recover + each block's tx root (strong scaling).
Each leg carries its roofline (the tx_verify kernel, HIP events on its launch stream; integer-MAC
bound) and its HBM traffic from the committed rocprofv3 PMC pass of the same workload (profiles/).

`merkle` (rank 0, N = 1): configs[0] (merkleBench, width-16 root over 100k 32-byte leaves) and 1M /
16M-leaf roots, Keccak256 and SM3, widths 2 and 16, device-resident, with the ALU roofline.

`cpu_baseline` (rank 0, N = 1): the same work on the host's cores over bounded samples -- the OpenSSL
1.1.1 libcrypto EC stand-in (oracle/standin_openssl.c) and the oracle's portable C
restatement, secp256k1 and SM2 -- plus the Merkle CPU restatement with per-level threads.

--gpus N without torchrun spawns the N ranks itself (torch.distributed.run, 127.0.0.1) before
touching the GPU; under torchrun WORLD_SIZE must equal --gpus.
"""
import argparse
import hashlib
import json
import math
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "fisco-bcos_amd"))
sys.path.insert(0, ROOT)

# Algorithmic work per unit: 1 F = one 256-bit modular multiplication = 136 32x32->64
# multiply-accumulates (8-limb CIOS); secp256k1 recover 3,240 F, SM2 verify 3,210 F (non-GLV counts).
MAC_PER_F = 136
F_SECP_RECOVER = 3240
F_SM2_VERIFY = 3210
# Field multiplications the kernels actually execute per unit (counted from their schedules,
# DESIGN.md §9; the safegcd inversions are ALU work outside the F count): GLV recover with the
# 16-bit comb / the 8-bit comb for u1 G; SM2 radix-16 Booth with the 16-bit / 8-bit comb for s G.
F_SECP_EXEC_WIDE = 2255
F_SECP_EXEC_COMB8 = 2431
F_SM2_EXEC = 3092
F_SM2_EXEC_COMB8 = 3268
# the SM2 lane-trio kernel's low-window split (ecc_pair.hip kSm2TrioSplit, BCOSGPU_SM2_SPLIT=0 turns it
# off): the high chain's tail doublings (4 per moved window, 8 F each) and the one extra complete
# addition (16 F) are executed work the split adds for its shorter critical path
SM2_TRIO_SPLIT = 0 if os.environ.get("BCOSGPU_SM2_SPLIT") == "0" else 44
F_SM2_TRIO_EXTRA = 4 * 8 * SM2_TRIO_SPLIT + 16 if SM2_TRIO_SPLIT else 0
# kernel (name without template arguments; the one-lane kernel by suite) -> (F with the 16-bit comb
# tables present, F on the 8-bit tables): which comb each kernel's launcher hands it (ecc_coop.hip
# launch_verify_small_secp: the trio kernel takes the wide tables, the pair / split kernels the 8-bit
# ones; ecc_pair.hip launch_verify_small_sm2: the SM2 pair kernels the 8-bit R'-domain table;
# ecc_txv.hip launch_verify: the one-lane kernels the wide ones; the SM2 trio kernel the wide R'-domain
# table since round 4)
KERNEL_F_EXEC = {
    "tx_verify_trio26_kernel": (F_SECP_EXEC_WIDE, F_SECP_EXEC_COMB8),
    "tx_verify_coop26_kernel": (F_SECP_EXEC_COMB8, F_SECP_EXEC_COMB8),
    "tx_verify_coop_kernel": (F_SECP_EXEC_COMB8, F_SECP_EXEC_COMB8),
    "tx_verify_split_kernel": (F_SECP_EXEC_COMB8, F_SECP_EXEC_COMB8),
    "tx_verify_kernel/0": (F_SECP_EXEC_WIDE, F_SECP_EXEC_COMB8),
    "tx_verify_sm2_trio26_kernel": (F_SM2_EXEC + F_SM2_TRIO_EXTRA, F_SM2_EXEC_COMB8 + F_SM2_TRIO_EXTRA),
    "tx_verify_sm2_pair26_kernel": (F_SM2_EXEC_COMB8, F_SM2_EXEC_COMB8),
    "tx_verify_sm2_pair_kernel": (F_SM2_EXEC_COMB8, F_SM2_EXEC_COMB8),
    "tx_verify_kernel/1": (F_SM2_EXEC, F_SM2_EXEC_COMB8),
}


def kernel_f_exec(kname, wide_tables=None):
    """Executed F per unit of the launched kernel `kname` (as _kernel_name returns it)."""
    base = kname.split("<")[0]
    if base == "tx_verify_kernel":
        base += "/" + kname.split("<")[1].split(",")[0]
    if wide_tables is None:
        wide_tables = os.environ.get("BCOSGPU_TABLES") != "small"
    wide, comb8 = KERNEL_F_EXEC[base]
    return wide if wide_tables else comb8
# measured gfx950 lane-op peaks (fisco-bcos_amd/tools/intbench.hip on MI355X, profiles/r01_intbench.json)
PEAK_MAC_PER_S = 3.0785e13      # v_mad_u64_u32
PEAK_ALU_PER_S = 3.7497e13      # full-rate 32-bit VALU (v_alignbit_b32)
# SURVEY §8d ALU ops per permutation / compression
KECCAK_F_OPS = 6240
SM3_C_OPS = 2100
PMC_GLOB = "r06_pmc_{}.json"
# per-leg PMC summary of the Merkle and hash legs (tools/leg_run.py under rocprofv3, tools/leg_prof.py)
LEG_PMC = "r06_pmc_legs.json"
KERNEL_SRC = ["fisco-bcos_amd/csrc/ecc_device.h", "fisco-bcos_amd/csrc/ecc_tables.hip", "fisco-bcos_amd/csrc/ecc_sig.hip",
              "fisco-bcos_amd/csrc/ecc_txv.hip", "fisco-bcos_amd/csrc/ecc_coop.hip", "fisco-bcos_amd/csrc/ecc_pair.hip",
              "fisco-bcos_amd/csrc/fe_asm.h", "fisco-bcos_amd/csrc/fe.h",
              "fisco-bcos_amd/csrc/ec.h", "fisco-bcos_amd/csrc/hash_device.h", "fisco-bcos_amd/csrc/modinv.h",
              "fisco-bcos_amd/csrc/fe26.h", "fisco-bcos_amd/csrc/ec26.h", "fisco-bcos_amd/csrc/recover26.h",
              "fisco-bcos_amd/csrc/fp26.h", "fisco-bcos_amd/csrc/ecp26.h", "fisco-bcos_amd/csrc/verify_sm2_26.h",
              "fisco-bcos_amd/csrc/ec26_trio.h", "fisco-bcos_amd/csrc/ecp26_trio.h", "fisco-bcos_amd/csrc/ecc_row.hip",
              "fisco-bcos_amd/csrc/fe_row.h", "fisco-bcos_amd/csrc/ec_row.h", "fisco-bcos_amd/csrc/hash_kernels.hip",
              "fisco-bcos_amd/csrc/sm3_x.h"]

WORKLOADS = {
    "c2": dict(suite=0, n=10_000, scaling="weak",
               name="C2: 10k synthetic secp256k1 txs / GPU: Keccak256 tx hash + ECDSA recover + sender"),
    "c2sm2": dict(suite=1, n=10_000, scaling="weak",
                  name="C2-SM2: 10k synthetic SM2/SM3 txs / GPU (C2's size, guomi suite): SM3 tx hash + SM2 verify "
                       "+ sender"),
    "c3": dict(suite=1, n=1_000_000, scaling="weak",
               name="C3: 1M synthetic SM2/SM3 txs / GPU: SM3 tx hash + SM2 verify + sender"),
    "c4": dict(suite=0, n=1_000_000, scaling="strong",
               name="C4: 1M synthetic secp256k1 txs sharded over the GPUs: tx hash + recover + sender "
                    "+ width-2 Keccak tx root (per-GPU frontier, RCCL all-gather)"),
    "c5": dict(suite=0, n=64 * 20_000, blocks=64, scaling="strong",
               name="C5: PBFT block-verify replay, 64 blocks x 20k secp256k1 txs sharded by block: "
                    "recover + per-block width-2 Keccak tx root"),
}


def kernel_source_sha():
    h = hashlib.sha256()
    for p in KERNEL_SRC:
        with open(os.path.join(ROOT, p), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


ROW_LAT, ROW_LAT_N = 0.38, 0.18  # ecc_txv.hip kRowLat, kRowLatN
ROW_LAT_SM2, ROW_LAT_N_SM2 = 0.43, 0.14  # kRowLatSM2, kRowLatNSM2
ROW_RESIDENT_SM2 = 4  # kRowResidentSM2


def _auto_kernel(suite, n, cus, small_ok=True, row_ok=True):
    """Mirror of ecc_txv.hip auto_kernel (rounds x latency): 3 row (secp256k1 recovery), 2 trio, 1 pair,
    0 one-lane at occupancy 1, -2 one-lane at occupancy 2 (whose tail round of <= one wave per SIMD has
    its own latency)."""
    lat = (4.315, 2.399, 1.678, 1.0) if suite == 1 else (4.475, 2.643, 1.279, 1.0)
    occ2_tail = 2.452 if suite == 1 else 2.556
    per = (512 * cus, 256 * cus, 64 * cus, 40 * cus)
    code = (-2, 0, 1, 2)
    best, cost = 0, float("inf")
    for k in (3, 2, 1, 0) if small_ok else (1, 0):
        c = -(-n // per[k]) * lat[k]
        if k == 0:
            tail = n % per[0]
            c = (n // per[0]) * lat[0] + (0 if tail == 0 else occ2_tail if tail <= per[1] else lat[0])
        if c < cost:
            best, cost = code[k], c
    r1, rn = (ROW_LAT_SM2, ROW_LAT_N_SM2) if suite == 1 else (ROW_LAT, ROW_LAT_N)
    m = -(-n // cus)
    res = ROW_RESIDENT_SM2 if suite == 1 else m
    rounds = -(-m // res)
    if row_ok and small_ok and rounds * r1 + (m - rounds) * rn < cost:
        best = 3
    return best


def _kernel_name(suite, n):
    """Which tx-verify kernel the library launches for this batch (mirrors launch_verify and its
    policy: BCOSGPU_TXV_* and BCOSGPU_K1_F26, read once by the library)."""
    import torch
    f26 = os.environ.get("BCOSGPU_K1_F26", "1") != "0"
    split = os.environ.get("BCOSGPU_TXV_SPLIT")
    small = (split == "1") if split in ("0", "1") else n <= (1 << 15)
    coop = {"0": 0, "1": 1, "3": 3}.get(os.environ.get("BCOSGPU_TXV_COOP", "2"), 2)
    occ = os.environ.get("BCOSGPU_TXV_OCC")
    occ = int(occ) if occ in ("1", "2") else 0
    if split not in ("0", "1") and coop == 2 and f26:
        cus = torch.cuda.get_device_properties(0).multi_processor_count if torch.cuda.is_available() else 256
        k = _auto_kernel(suite, n, cus, n <= (1 << 16), os.environ.get("BCOSGPU_TXV_ROW", "1") != "0")
        small = k > 0
        if small:
            coop = k
        elif not occ:
            occ = 2 if k == -2 else 1
    if not occ:
        occ = 2 if n >= (1 << 17) else 1
    if suite == 0 and small:
        if coop == 3 and f26:
            return "recover_row_kernel<TxIO>"
        if not coop:
            return "tx_verify_split_kernel"
        if coop == 2 and f26:
            return "tx_verify_trio26_kernel<TxIO>"
        return "tx_verify_coop26_kernel<TxIO>" if f26 else "tx_verify_coop_kernel"
    if suite == 1 and small and coop:
        if coop == 3 and f26:
            return "sm2_verify_row_kernel<TxIO>"
        if f26:
            return ("tx_verify_sm2_trio26_kernel<TxIO,%d>" % SM2_TRIO_SPLIT if coop >= 2
                    else "tx_verify_sm2_pair26_kernel<TxIO>")
        return "tx_verify_sm2_pair_kernel"
    return "tx_verify_kernel<%d,%d,%s,TxIO>" % (suite, occ, "true" if f26 else "false")


def _norm(name):
    return name.replace("void ", "").replace("bcosgpu::", "").replace(" ", "").split("(")[0]


def _traffic(workload, kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes of this workload
    (tools/prof_summary.py; FETCH_SIZE doubled per MI355X_MICROARCH.md's gfx950 correction), and
    whether they were taken on the kernel sources of this tree."""
    path = os.path.join(ROOT, "profiles", PMC_GLOB.format(workload))
    try:
        with open(path) as f:
            pmc = json.load(f)
    except (OSError, ValueError):
        return None, None, None
    for name, c in pmc.get("kernels", {}).items():
        if _norm(name) == _norm(kernel) and "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            same = pmc.get("kernel_source_sha") == kernel_source_sha()
            return (2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0, os.path.relpath(path, ROOT), same
    return None, None, None


def _valu_issue(workload, kernel):
    """VALU issue fraction of `kernel` from the same PMC file: wave64 VALU instructions per SIMD x 4
    cycles (a SIMD16 issues one wave64 VALU op per 4 cycles) over the dispatch's cycles per XCD
    (GRBM_GUI_ACTIVE is summed over the 8 XCDs).  Near 1 = the kernel is issue-bound, and only fewer
    instructions make it faster."""
    path = os.path.join(ROOT, "profiles", PMC_GLOB.format(workload))
    try:
        with open(path) as f:
            pmc = json.load(f)
    except (OSError, ValueError):
        return None
    for name, c in pmc.get("kernels", {}).items():
        if _norm(name) == _norm(kernel) and c.get("SQ_INSTS_VALU") and c.get("GRBM_GUI_ACTIVE") and c.get("SQ_WAVES"):
            simds = 1024.0
            cycles = c["GRBM_GUI_ACTIVE"] / 8.0
            return {"frac": c["SQ_INSTS_VALU"] * 4.0 / simds / cycles,
                    "valu_per_wave": c["SQ_INSTS_VALU"] / c["SQ_WAVES"],
                    "waves": c["SQ_WAVES"], "source": os.path.relpath(path, ROOT),
                    "note": "VALU instructions x 4 cycles / 1,024 SIMDs / dispatch cycles per XCD; a lone "
                            "wave per SIMD (latency kernels) cannot reach 1"}
    return None


def _block_plan(nblocks, world, rank):
    per = math.ceil(nblocks / world)
    return min(rank * per, nblocks), min((rank + 1) * per, nblocks)


def launcher_selftest_plans(ctx, dist):
    """The multi-rank plumbing of the GPU run, on the CPU (gloo): every rank derives its C4 shard exactly as
    run_leg does (parallel.choose_levels / shard_plan: width^L-aligned tx ranges of configs[3]'s 1M txs) and
    its C5 block range (_block_plan over configs[4]'s 64 blocks), builds its level-L frontier over stand-in
    leaves (leaf i = blake2b-256 of i; a stand-in hash, this checks the plan and the gather, not Keccak --
    blake2b also builds the levels), and the frontiers go through parallel.sharded_merkle_root's
    count-prefixed all-gather as on RCCL; rank 0 reports every rank's ranges, the gathered root, the
    device list the one-process device-set legs would take and the per-GPU kernel choice at C4."""
    import hashlib as hl
    import torch
    from bcos_gpu import parallel
    world, rank = ctx.world, ctx.rank
    n4, width = WORKLOADS["c4"]["n"], 2
    levels = parallel.choose_levels(n4, world, width)
    plan = parallel.shard_plan(n4, world, width, levels)

    def h2(x):
        return hl.blake2b(x, digest_size=32).digest()

    def frontier_fn(lo, hi):
        cur = [h2(i.to_bytes(8, "little")) for i in range(lo, hi)]
        for _ in range(levels):
            cur = [h2(b"".join(cur[k:k + width])) for k in range(0, len(cur), width)]
        return torch.tensor(list(b"".join(cur)), dtype=torch.uint8).view(-1, 32)

    def root_fn(frontier):
        cur = [bytes(r.tolist()) for r in frontier]
        while len(cur) > 1:
            cur = [h2(b"".join(cur[k:k + width])) for k in range(0, len(cur), width)]
        return torch.tensor(list(cur[0]), dtype=torch.uint8)
    root = parallel.sharded_merkle_root(frontier_fn, root_fn, n4, width, levels, rank, world, "cpu")
    blo, bhi = _block_plan(WORKLOADS["c5"]["blocks"], world, rank)
    mine = torch.tensor([plan[rank][0], plan[rank][1], blo, bhi], dtype=torch.int64)
    allr = [torch.zeros(4, dtype=torch.int64) for _ in range(world)]
    if world > 1:
        dist.all_gather(allr, mine)
    else:
        allr = [mine]
    per = plan[0][1] - plan[0][0]
    return {"c4": {"levels": levels, "block": width ** levels, "ranges": [[int(x[0]), int(x[1])] for x in allr],
                   "per_gpu_txs": per, "kernel_per_gpu": _kernel_name(0, per),
                   "standin_root_blake2b": bytes(root.tolist()).hex()},
            "c5": {"block_ranges": [[int(x[2]), int(x[3])] for x in allr]},
            "devset": list(range(world)) if world > 1 else [0, 0]}


def spawn_ranks(args):
    """--gpus N without a launcher: run this script under torch.distributed.run (one process per GPU,
    RCCL rendezvous on 127.0.0.1) as a child -- before this process touches the GPU -- and return its
    exit status."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


class Ctx:
    def __init__(self, world, rank, dist):
        self.world, self.rank, self.dist = world, rank, dist

    def max(self, x):
        if self.world == 1:
            return x
        import torch
        dev = "cpu" if self.dist.get_backend() == "gloo" else "cuda"
        t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()


EVENT_EVERY = 16  # set from --event-every


def run_leg(ctx, wl_name, steps=None, warmup=3, warm_seconds=0.0, min_seconds=2.0):
    """One workload on this rank; returns the leg's record (rank 0's view, times max over ranks)."""
    import numpy as np
    import torch
    from bcos_gpu import device, parallel, synth

    wl = WORKLOADS[wl_name]
    suite, world, rank = wl["suite"], ctx.world, ctx.rank
    stream = torch.cuda.current_stream()
    txroot = None
    block_off = None
    if wl_name == "c4":
        txroot = parallel.gpu_sharded_tx_root(wl["n"], world, rank, device.KECCAK256, 2, "cuda")
        lo, hi = txroot.local_range
        n = hi - lo
    elif wl_name == "c5":
        per_block = wl["n"] // wl["blocks"]
        blo, bhi = _block_plan(wl["blocks"], world, rank)
        n = (bhi - blo) * per_block
        block_off = np.arange(bhi - blo + 1, dtype=np.uint64) * np.uint64(per_block)
        work = torch.empty(max(device.merkle_roots_work_size(n, bhi - blo, 2), 1), dtype=torch.uint8, device="cuda")
        roots = torch.empty((max(bhi - blo, 1), 32), dtype=torch.uint8, device="cuda")
    else:
        n = wl["n"]
    units_total = wl["n"] if wl["scaling"] == "strong" else wl["n"] * world
    b = synth.make_batch(suite, max(n, 1), seed=0xF15C0BC5 + 7919 * rank)
    txhash = torch.empty((max(n, 1), 32), dtype=torch.uint8, device="cuda")
    sender = torch.empty((max(n, 1), 20), dtype=torch.uint8, device="cuda")
    status = torch.empty(max(n, 1), dtype=torch.uint8, device="cuda")
    evs = []

    def step(timed=False):
        if timed:
            a, c = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
        if n:
            device.tx_verify(suite, b.pre, b.pre_off, b.sig, b.sig_off, txhash, sender, status, stream)
        if timed:
            c.record(stream)
            evs.append((a, c))
        if txroot is not None:
            txroot(txhash[:n])
        elif block_off is not None and n:
            device.merkle_roots_batch(device.KECCAK256, 2, txhash, block_off, work, roots, stream)

    # calibrate, then warm up for >= warmup steps and >= warm_seconds of back-to-back launches (the
    # clock settles under load); step counts are agreed over the ranks (C4 steps hold a collective)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    per = ctx.max((time.perf_counter() - t1) / 3)
    for k in range(max(warmup, int(math.ceil(warm_seconds / max(per, 1e-6))))):
        step()
        if k % 32 == 31:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    if steps is None:  # time-based leg: enough steps for >= min_seconds
        steps = max(3, int(math.ceil(min_seconds / max(per, 1e-6))))
    ctx.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):  # (kernel duration events on every EVENT_EVERY-th step: each pair adds stream packets)
        step(timed=k % EVENT_EVERY == 0)
    torch.cuda.synchronize()
    ctx.barrier()
    torch.cuda.synchronize()
    elapsed = ctx.max(time.perf_counter() - t0)
    kernel_ms = sum(a.elapsed_time(c) for a, c in evs) / len(evs)
    ok_frac = float((status[:n] == 0).float().mean().item()) if n else 1.0
    kname = _kernel_name(suite, n)
    f_alg = F_SECP_RECOVER if suite == 0 else F_SM2_VERIFY
    f_exec = kernel_f_exec(kname)
    ex = n * f_exec * MAC_PER_F / (kernel_ms * 1e-3)
    alg = n * f_alg * MAC_PER_F / (kernel_ms * 1e-3)
    traffic, traffic_src, same_src = _traffic(wl_name, kname)
    valu_issue = _valu_issue(wl_name, kname)
    roofline = {
        "bound": "int-valu", "achieved": ex / 1e12, "peak": PEAK_MAC_PER_S / 1e12, "unit": "TMAC/s",
        "frac": ex / PEAK_MAC_PER_S, "traffic": traffic, "traffic_source": traffic_src,
        "traffic_same_kernel_source": same_src, "valu_issue": valu_issue, "kernel": kname, "kernel_ms": kernel_ms,
        "units_per_launch": n,
        "work_per_unit": "%d F x %d MAC executed (kernel schedule, DESIGN.md 9)" % (f_exec, MAC_PER_F),
        "algorithmic": {"work_per_unit": "%d F x %d MAC (SURVEY.md 8d, non-GLV count)" % (f_alg, MAC_PER_F),
                        "achieved": alg / 1e12, "frac": alg / PEAK_MAC_PER_S,
                        "note": "USEFUL work per second (SURVEY 8d's non-GLV count) against the MAC peak, not an "
                                "issue rate: GLV and the comb execute fewer multiplications than 8d counts, so "
                                "it can exceed 1 (C4/C5); the issue fraction is valu_issue"},
        "algorithmic_bytes_per_unit": 151 + 65 + 53 if suite == 0 else 151 + 128 + 53,
    }
    rec = {"workload": wl["name"], "value": units_total * steps / elapsed, "unit": "tx/s",
           "ms_per_step": elapsed / steps * 1e3, "steps": steps, "timed_s": elapsed, "scaling": wl["scaling"],
           "txs_total": units_total, "txs_rank0": n, "valid_frac": ok_frac, "roofline": roofline}
    state = {"batch": b, "status": status[:n], "n": n}
    return rec, state


MERKLE_SPECS = [(n, hname, width) for n in (100_000, 1_000_000, 16_000_000)
                for hname in ("keccak256", "sm3") for width in (16, 2)]
# hashes/s legs (north_star): (name, hasher, messages, length) -- "c2" = configs[1]'s 10k 151-byte tx
# preimages (synth.preimages, TarsHashable.h:29-40); 1M tx preimages; 1M 64-byte public keys (the
# address hash, KeyPair.h:30-33)
HASH_SPECS = [("keccak256_c2", "keccak256", 10_000, 151), ("sm3_c2", "sm3", 10_000, 151),
              ("keccak256_1M_151B", "keccak256", 1_000_000, 151), ("sm3_1M_151B", "sm3", 1_000_000, 151),
              ("keccak256_1M_64B", "keccak256", 1_000_000, 64), ("sm3_1M_64B", "sm3", 1_000_000, 64)]


def merkle_name(n, hname, width):
    return "%s_w%d_%s" % (hname, width, _count(n))


def merkle_inputs(n):
    import torch
    g = torch.Generator(device="cuda")
    g.manual_seed(n)
    return torch.randint(0, 256, (n, 32), dtype=torch.uint8, device="cuda", generator=g)


def hash_inputs(n, length):
    """Device (data, offsets) of n messages of `length` bytes: the synthetic tx preimages when length is
    151, else seeded random bytes."""
    import torch
    from bcos_gpu import synth
    if length == synth.PREIMAGE_LEN:
        data = torch.from_numpy(synth.preimages(n).reshape(-1)).cuda()
    else:
        g = torch.Generator(device="cuda")
        g.manual_seed(n * 7 + length)
        data = torch.randint(0, 256, (n * length,), dtype=torch.uint8, device="cuda", generator=g)
    off = torch.arange(0, (n + 1) * length, length, dtype=torch.int64, device="cuda")
    return data, off


def _hasher(hname):
    from bcos_gpu import device
    return device.KECCAK256 if hname == "keccak256" else device.SM3


def _hash_units(length, keccak):
    """Keccak-f permutations (rate 136, pad >= 1 byte) / SM3 compressions (64-byte blocks, 9 bytes of
    padding) for one message of `length` bytes."""
    return length // 136 + 1 if keccak else (length + 8) // 64 + 1


def leg_pmc(name):
    """Per-root (per-batch) counters of the Merkle / hash leg `name` from the committed PMC summary
    (tools/leg_prof.py): VALU instructions, GRBM cycles (summed over the 8 XCDs), HBM bytes, and the
    issue fraction derived from them (wave64 VALU instructions x 4 cycles / 1,024 SIMDs / cycles per
    XCD, <= 1 by construction)."""
    try:
        with open(os.path.join(ROOT, "profiles", LEG_PMC)) as f:
            pmc = json.load(f)
    except (OSError, ValueError):
        return None
    c = pmc.get("legs", {}).get(name)
    if not c or not c.get("SQ_INSTS_VALU") or not c.get("GRBM_GUI_ACTIVE"):
        return None
    out = {"valu_issue": c["SQ_INSTS_VALU"] * 4.0 / 1024.0 / (c["GRBM_GUI_ACTIVE"] / 8.0),
           "valu_per_unit": c["SQ_INSTS_VALU"], "source": os.path.join("profiles", LEG_PMC),
           "same_kernel_source": pmc.get("kernel_source_sha") == kernel_source_sha()}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        out["traffic"] = (2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0
    return out


def _event_ms(fn, min_s=0.25, warm=3):
    """Average device time (ms) of fn() over >= min_s of back-to-back calls, HIP events on torch's stream."""
    import torch
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    reps = max(5, int(min_s / max(time.perf_counter() - t1, 1e-6)))
    a, c = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    c.record()
    torch.cuda.synchronize()
    return a.elapsed_time(c) / reps, reps


def _alu_roofline(ms, units, keccak, name):
    """The executed-instruction roofline of a hash / Merkle leg: frac = the PMC issue fraction (<= 1);
    useful_frac = SURVEY 8(d)'s op count per second over the v_alignbit peak, a useful-work figure that
    three-input XORs and paired rotates can push past 1 (not an issue-rate claim)."""
    ops = units * (KECCAK_F_OPS if keccak else SM3_C_OPS)
    pmc = leg_pmc(name)
    return {"bound": "int-valu", "frac": pmc["valu_issue"] if pmc else None,
            "useful_ops_per_s": ops / (ms * 1e-3), "useful_frac": ops / (ms * 1e-3) / PEAK_ALU_PER_S,
            "peak_ops_per_s": PEAK_ALU_PER_S, "units": units,
            "traffic": pmc.get("traffic") if pmc else None, "pmc": pmc}


def hash_legs():
    """hashes/s (north_star): bcosgpu_hash_batch_dev over HBM-resident messages (HASH_SPECS)."""
    import torch
    from bcos_gpu import device
    out = {}
    for name, hname, n, length in HASH_SPECS:
        data, off = hash_inputs(n, length)
        dig = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
        h = _hasher(hname)
        ms, reps = _event_ms(lambda: device.hash_batch(h, data, off, dig))
        keccak = hname == "keccak256"
        units = n * _hash_units(length, keccak)
        rf = _alu_roofline(ms, units, keccak, name)
        rf["algorithmic_bytes"] = n * (length + 8 + 32)
        out[name] = {"hashes_per_s": n / (ms * 1e-3), "ms": ms, "reps": reps, "messages": n, "bytes_each": length,
                     "GB_per_s": n * length / (ms * 1e-3) / 1e9, "roofline": rf}
        del data, off, dig
    torch.cuda.empty_cache()
    return out


def merkle_legs(cpu_threads):
    """configs[0] (merkleBench: width-16 root, 100k leaves) and the 1M / 16M-leaf roofline legs."""
    import torch
    from bcos_gpu import device
    out = {}
    last_n, leaves = None, None
    for n, hname, width in MERKLE_SPECS:
        if n != last_n:
            del leaves
            torch.cuda.empty_cache()
            leaves, last_n = merkle_inputs(n), n
        h = _hasher(hname)
        keccak = hname == "keccak256"
        tree = torch.empty((device.merkle_size(n, width), 32), dtype=torch.uint8, device="cuda")
        root = torch.empty(32, dtype=torch.uint8, device="cuda")
        ms, reps = _event_ms(lambda: device.merkle_root(h, width, leaves, tree, root))
        units, _ = merkle_work(n, width, keccak)
        floor = merkle_floor(n, width, keccak)
        name = merkle_name(n, hname, width)
        rf = _alu_roofline(ms, units, keccak, name)
        rf["algorithmic_bytes"] = n * 32 + device.merkle_size(n, width) * 32
        out[name] = {"ms": ms, "GB_per_s": n * 32 / (ms * 1e-3) / 1e9, "reps": reps,
                     "latency_floor_ms": floor["ms"] if floor else None,
                     "frac_of_latency_floor": floor["ms"] / ms if floor else None, "latency_floor": floor,
                     "roofline": rf}
        del tree, root
    del leaves
    torch.cuda.empty_cache()
    if cpu_threads:
        out["cpu_baseline"] = merkle_cpu(cpu_threads)
    return out


def _count(n):
    return "%dk" % (n // 1000) if n < 1_000_000 else "%dM" % (n // 1_000_000)


HASH_LATENCY = "r04_hash_latency.json"  # tools/keccakpair_check.hip + sm3probe.hip on MI355X: cycles per unit, lone wave
CLOCK_HZ = 2.4e9                        # MI355X peak engine clock (MI355X_MICROARCH.md)


def merkle_floor(n, width, keccak):
    """Serial-hash floor of Merkle<H,width> over n leaves (Merkle.h:243-261): each level waits for its
    slowest node -- a full group of `width` children, or the level's whole input when smaller -- so the
    critical path is the sum over levels of that node's Keccak-f permutations / SM3 compressions, times
    the fastest measured per-unit latency of a lone wave (cooperative 25-lane Keccak-f; SM3 from a block
    expanded beforehand) at the peak clock.  No schedule of this hash on this GPU beats it."""
    try:
        with open(os.path.join(ROOT, "profiles", HASH_LATENCY)) as f:
            lat = json.load(f)
    except (OSError, ValueError):
        return None
    cyc = (min(lat["cycles_per_perm_coop25"], lat["cycles_per_perm_pair"]) if keccak else
           min(lat["cycles_per_sm3_compression"], lat.get("cycles_per_sm3_compression_expanded", 1 << 30)))
    units, m = 0, n
    while m > 1:
        k = min(width, m)
        units += (32 * k // 136 + 1) if keccak else ((32 * k + 8) // 64 + 1)
        m = -(-m // width)
    return {"ms": units * cyc / CLOCK_HZ * 1e3, "serial_units": units, "cycles_per_unit": cyc,
            "source": os.path.join("profiles", HASH_LATENCY),
            "note": "critical-path %s x the measured lone-wave latency at %.1f GHz" % (
                "Keccak-f permutations" if keccak else "SM3 compressions", CLOCK_HZ / 1e9)}


def merkle_work(n, width, keccak):
    """Exact permutation / compression count of Merkle<H,width> over n leaves (Merkle.h:243-261):
    per level, groups of <= width children hashed as 32k-byte messages."""
    units, m = 0, n
    while m > 1:
        full, rem = divmod(m, width)
        for k, cnt in ((width, full), (rem, 1 if rem else 0)):
            if cnt:
                ln = 32 * k
                units += cnt * ((ln // 136 + 1) if keccak else ((ln + 8) // 64 + 1))
        m = full + (1 if rem else 0)
    return units, units * (KECCAK_F_OPS if keccak else SM3_C_OPS)


def _median_time(fn, reps=5):
    """one warm-up, then `reps` timed repetitions; the median (s) and all times."""
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2], ts


def merkle_cpu(threads):
    """The reference's Merkle CPU path on the host: Merkle<H, width>::generateMerkle (Merkle.h:170-261) with
    its OpenSSL 1.1.1 hashers (OpenSSLHasher.h:22-143: EVP_sm3; EVP_sha3_256 with the Keccak pad poke), the
    hashers merkleBench.cpp times -- oracle/standin_openssl.c, levels parallel over `threads` like the
    reference's tbb::parallel_for -- at configs[0]'s 100k leaves and at 1M; median of 5 repetitions.
    Without the OpenSSL stand-in, the oracle's portable C restatement (kind "port")."""
    import numpy as np
    from oracle import oracle
    rng = np.random.default_rng(3)
    leaves = rng.integers(0, 256, size=(1_000_000, 32), dtype=np.uint8)
    use_ossl = oracle.standin() is not None
    res = {}
    for n in (100_000, 1_000_000):
        for hname, h in (("keccak256", oracle.KECCAK256), ("sm3", oracle.SM3)):
            for width in (16, 2):
                lv = leaves[:n]
                if use_ossl:
                    fn = lambda: oracle.standin_merkle_root(h, width, lv, nthreads=threads)  # noqa: E731
                else:
                    fn = lambda: oracle.merkle(h, width, lv, nthreads=threads)  # noqa: E731
                med, ts = _median_time(fn)
                res["%s_w%d_%s" % (hname, width, _count(n))] = {
                    "ms": med * 1e3, "GB_per_s": n * 32 / med / 1e9, "reps_ms": [round(t * 1e3, 3) for t in ts]}
    return {"legs": res, "threads": threads, "kind": "standin-openssl-restatement" if use_ossl else "port",
            "impl": ("Merkle.h:170-261 over the reference's OpenSSL hashers (OpenSSLHasher.h, EVP_sm3 / EVP_sha3_256 "
                     "with the 0x01 pad poke; OpenSSL %s), level-parallel pthreads" % oracle.standin_version())
            if use_ossl else "oracle/merkle.c restatement of Merkle.h:170-261, level-parallel pthreads",
            "note": "median of 5 repetitions after a warm-up (BASELINE.md 3)"}


def _cpu_info():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return model


def _physical_cores():
    """Distinct (package, core) pairs in sysfs -- SMT siblings counted once; os.cpu_count() without sysfs."""
    cores = set()
    base = "/sys/devices/system/cpu"
    try:
        for d in os.listdir(base):
            if d.startswith("cpu") and d[3:].isdigit():
                try:
                    with open(os.path.join(base, d, "topology", "thread_siblings_list")) as f:
                        cores.add(f.read().strip())
                except OSError:
                    pass
    except OSError:
        pass
    return len(cores) or os.cpu_count() or 1


def cpu_threads():
    """Threads for the CPU legs: the box's CPU share (OMP_NUM_THREADS is set to it on the GPU box;
    nproc / the affinity mask show the whole machine there), else the affinity mask."""
    env = os.environ.get("BCOSGPU_CPU_THREADS") or os.environ.get("OMP_NUM_THREADS")
    aff = len(os.sched_getaffinity(0))
    return min(int(env), aff) if env and env.isdigit() and int(env) > 0 else aff


def cpu_baseline(batches, threads):
    """Transaction::verify (Transaction.h:68-82) per tx on the host (TransactionSync.cpp:516-548's
    parallel_for) over bounded samples of the benchmark batches: the OpenSSL 1.1.1 EC stand-in
     and the oracle's portable C restatement, secp256k1 and SM2; each the median of 5
    timed passes after a warm-up.  value = the faster secp256k1 leg (the headline
    metric's CPU counterpart); kind follows that leg."""
    import numpy as np
    from oracle import oracle
    legs = {}
    for suite, b, sample in batches:
        pre = b.pre.cpu().numpy()
        pre_off = np.ascontiguousarray(b.pre_off[: sample + 1].cpu().numpy().astype(np.uint64))
        sig = b.sig.cpu().numpy()
        sig_off = np.ascontiguousarray(b.sig_off[: sample + 1].cpu().numpy().astype(np.uint64))
        impls = [("port", oracle.tx_verify_packed)]
        if oracle.standin() is not None:
            impls.append(("openssl", oracle.standin_tx_verify_packed))
        for name, fn in impls:
            med, ts = _median_time(lambda: fn(suite, pre, pre_off, sig, sig_off, nthreads=threads))
            legs["%s_%s" % ("secp256k1" if suite == 0 else "sm2", name)] = {
                "value": sample / med, "unit": "tx/s", "per_thread": sample / med / threads,
                "sample": "%d txs per pass, median of %d passes (%.2f s total)" % (sample, len(ts), sum(ts)),
                "passes_s": [round(t, 4) for t in ts]}
    best = max((v for k, v in legs.items() if k.startswith("secp256k1")), key=lambda v: v["value"])
    best_name = [k for k, v in legs.items() if v is best][0]
    logical = os.cpu_count()
    openssl = best_name.endswith("openssl")
    return {"value": best["value"], "unit": "tx/s", "cores": threads, "kind": "standin-openssl" if openssl else "port",
            "kind_detail": ("NOT the reference's ECC: the reference's per-tx path with its third-party ECC (wedpr's "
                            "libsecp256k1 / TASSL, absent here) replaced by OpenSSL 1.1.1 libcrypto EC, the "
                            "reference-class library in this image" if openssl
                            else "the oracle's portable C restatement of the path"),
            "impl": best_name, "sample": best["sample"],
            "host": {"cpu_model": _cpu_info(), "nproc": logical, "affinity": len(os.sched_getaffinity(0)),
                     "threads_used": threads, "libcrypto": oracle.standin_version()},
            "full_host_estimate": {"value": best["per_thread"] * _physical_cores(), "unit": "tx/s",
                                   "physical_cores": _physical_cores(), "logical_cpus": logical,
                                   "smt_upper_bound": best["per_thread"] * logical,
                                   "note": "per-thread rate (measured on the box's CPU share, one thread per core) x "
                                           "physical cores; smt_upper_bound counts SMT siblings as cores too"},
            "legs": legs,
            "note": "stand-ins for the reference's third-party ECC (wedpr libsecp256k1 / TASSL, absent and "
                    "unbuildable here, BASELINE.md 3): OpenSSL libcrypto EC and the oracle's 4x64 Montgomery port"}


def host_api_rate(b, suite, n, reps=50):
    """The same batch through the host-pointer ABI (bcosgpu_tx_verify_batch: csrc/txpipe.hip -- for C2's
    10k one launch: the offsets check and the gather into pinned staging on helper threads, one H2D, the
    kernel writing the mapped pinned outputs, one sync, the outputs copied back) -- the PCIe-inclusive rate
    a caller holding host buffers sees.  Not `value`.  `value` here is the C ABI call itself (what a node
    links; arguments prepared once, the caller's output arrays reused as a node reuses its batch buffers);
    `verify_packed_ms` is the same call through the Python mirror, `fresh_outputs_ms` that into newly
    allocated arrays each time (their first-touch page faults land inside the call).  The three alternate
    call by call, so clock ramps and neighbours hit them alike; medians."""
    import numpy as np
    import bcos_gpu
    from bcos_gpu import tx
    from bcos_gpu._lib import check, lib
    pre = np.ascontiguousarray(b.pre.cpu().numpy())
    pre_off = np.ascontiguousarray(b.pre_off[: n + 1].cpu().numpy().astype(np.uint64))
    sig = np.ascontiguousarray(b.sig.cpu().numpy())
    sig_off = np.ascontiguousarray(b.sig_off[: n + 1].cpu().numpy().astype(np.uint64))
    suite_obj = bcos_gpu.sm_suite() if suite else bcos_gpu.secp256k1_suite()
    out = tx.verify_packed(suite_obj, pre, pre_off, sig, sig_off)  # warm-up (pipeline buffers)
    ab = tuple(np.zeros_like(x) for x in out)
    fn = lib().bcosgpu_tx_verify_batch
    args = (suite_obj.suite,) + tuple(x.__array_interface__["data"][0] for x in (pre, pre_off, sig, sig_off)) + (n,) + \
        tuple(x.__array_interface__["data"][0] for x in ab)
    check(fn(*args))
    same = all(np.array_equal(x, y) for x, y in zip(ab, out))
    ta, ts, tf = [], [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        rc = fn(*args)
        t1 = time.perf_counter()
        tx.verify_packed(suite_obj, pre, pre_off, sig, sig_off, out=out)
        t2 = time.perf_counter()
        tx.verify_packed(suite_obj, pre, pre_off, sig, sig_off)
        t3 = time.perf_counter()
        check(rc)
        ta.append(t1 - t0)
        ts.append(t2 - t1)
        tf.append(t3 - t2)
    for v in (ta, ts, tf):
        v.sort()
    da, dt, fresh = ta[len(ta) // 2], ts[len(ts) // 2], tf[len(tf) // 2]
    return {"value": n / da, "unit": "tx/s", "ms_per_batch": da * 1e3, "verify_packed_ms": dt * 1e3,
            "verify_packed_tx_s": n / dt, "fresh_outputs_ms": fresh * 1e3, "abi_matches_python": bool(same),
            "path": "bcosgpu_tx_verify_batch (host buffers: offsets check + gather into pinned staging on helper "
                    "threads, one H2D, kernel writing the mapped pinned outputs, sync, copy out); value = the C ABI "
                    "call, median of %d alternating with the Python mirror (reused / fresh outputs)" % reps}


def interface_legs(batches, threads=(16, 64, 256), calls=1000, reps=20):
    """The reference-interface entry points on the C2-size batches (rank 0, N = 1), per suite:
      recover_batch: SignatureCrypto::recover for a whole batch -- bcosgpu_secp256k1_recover_batch_dev /
                     bcosgpu_sm2_verify_batch_dev (HIP events, the same rounds x latency kernel choice as
                     the tx path) and the host-pointer ABI (bcosgpu_*_batch: H2D + kernel + D2H);
      single_call:   for each T in `threads` (16 = the box's CPU share, 256 = hardware_concurrency here, the
                     reference's submitter pool size, NodeConfig.cpp:486 / TxPool.h:48-49): T host threads x
                     `calls` single calls each (bcosgpu_secp256k1_recover / bcosgpu_sm2_verify, the per-tx
                     SignatureCrypto::recover), coalesced by the engine -- fisco-bcos_amd/lib/callbench,
                     every result checked against the batch path's -- beside the CPU stand-in at T threads."""
    import struct
    import tempfile
    import numpy as np
    import torch
    import bcos_gpu
    from bcos_gpu import device
    out = {}
    for suite, b in batches:
        n, sl = b.n, b.sig_len
        name = "secp256k1" if suite == 0 else "sm2"
        hashes = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
        device.hash_batch(device.SM3 if suite else device.KECCAK256, b.pre, b.pre_off, hashes)
        sigs = b.sig.view(n, sl)
        pub = torch.empty((n, 64), dtype=torch.uint8, device="cuda")
        ok = torch.empty(n, dtype=torch.uint8, device="cuda")

        def launch():
            if suite == 0:
                device.secp256k1_recover(hashes, sigs, pub, None, ok)
            else:
                device.sm2_verify(hashes, sigs, None, ok)
        t0 = time.perf_counter()  # >= 0.5 s of back-to-back launches first: the clock settles under load
        while time.perf_counter() - t0 < 0.5:
            for _ in range(16):
                launch()
            torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            a, c = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            launch()
            c.record()
            c.synchronize()
            ts.append(a.elapsed_time(c))
        ts.sort()
        rec = {"n": n, "kernel_ms_median": ts[len(ts) // 2], "path": "bcosgpu_%s_batch_dev" % (
            "secp256k1_recover" if suite == 0 else "sm2_verify")}
        h_h, h_s = hashes.cpu().numpy(), sigs.cpu().numpy()
        crypto = bcos_gpu.Secp256k1Crypto() if suite == 0 else bcos_gpu.SM2Crypto()
        want_pub, want_ok = crypto.recover_batch(h_h, h_s)
        t0 = time.perf_counter()
        for _ in range(5):
            crypto.recover_batch(h_h, h_s)
        rec["host_abi_ms"] = (time.perf_counter() - t0) / 5 * 1e3
        dev_ok = ok.cpu().numpy().astype(bool)
        rec["matches_host_abi"] = bool(np.array_equal(dev_ok, want_ok)) and (
            suite == 1 or bool(np.array_equal(pub.cpu().numpy()[want_ok], want_pub[want_ok])))
        out["recover_batch_%s" % name] = rec
        exe = os.path.join(ROOT, "fisco-bcos_amd", "lib", "callbench")
        if os.path.exists(exe):
            m = min(n, 8192)
            with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
                f.write(b"BGCT" + struct.pack("<II", suite, m))
                kp = want_pub[:m] if suite == 0 else h_s[:m, 64:128]
                for arr in (h_h[:m], h_s[:m], want_ok[:m].astype(np.uint8), kp):
                    f.write(np.ascontiguousarray(arr, dtype=np.uint8).tobytes())
                path = f.name
            try:
                for t in threads:
                    r = subprocess.run([exe, path, str(t), str(calls)], capture_output=True, text=True, timeout=300)
                    line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else "{}"
                    res = json.loads(line)
                    res["rc"] = r.returncode
                    res["cpu_standin"] = single_call_cpu(b, suite, t)
                    out["single_call_%dt_%s" % (t, name)] = res
            finally:
                os.unlink(path)
    return out


def single_call_cpu(b, suite, threads, sample=4000):
    """The CPU counterpart of `threads` submitter threads each verifying one tx per call: the OpenSSL EC
    stand-in (else the oracle's port) over `threads` threads on a bounded sample; calls/s and the mean
    per-call latency of that closed loop (threads / rate, Little's law)."""
    import numpy as np
    from oracle import oracle
    n = min(sample, b.n)
    pre = b.pre.cpu().numpy()
    pre_off = np.ascontiguousarray(b.pre_off[: n + 1].cpu().numpy().astype(np.uint64))
    sig = b.sig.cpu().numpy()
    sig_off = np.ascontiguousarray(b.sig_off[: n + 1].cpu().numpy().astype(np.uint64))
    ossl = oracle.standin() is not None
    fn = oracle.standin_tx_verify_packed if ossl else oracle.tx_verify_packed
    med, _ = _median_time(lambda: fn(suite, pre, pre_off, sig, sig_off, nthreads=threads), reps=3)
    rate = n / med
    return {"calls_per_s": rate, "mean_latency_us": threads / rate * 1e6, "threads": threads,
            "cores": cpu_threads(), "kind": "standin-openssl" if ossl else "port", "sample": n}


def sealer_verify_leg(threads, reps=100, committee=32):
    """PBFT sealer-signature checks: SignatureCrypto::verify(pub, hash, sig) against the consensus node
    list's keys (BlockValidator::checkSignatureList, bcos-pbft/.../BlockValidator.cpp:141-182, and
    PBFTCacheProcessor::checkPrecommitWeight, PBFTCacheProcessor.cpp:795-821 -> Secp256k1Crypto.cpp:51-63 /
    SM2Crypto.cpp:66-79), per suite, with a committee of `committee` sealers registered up front
    (bcosgpu_register_keys, the node's consensus list):
      block_{k}:   one block's k in {4, 7, 32} sealer signatures as one bcosgpu_verify_batch call (host
                   buffers, coalesced; the registered-key kernel) -- p50 / p99 latency over `reps` blocks;
      unreg_7:     the same call with 7 keys never seen before (the generic verify kernels) -- p50;
      single:      one SignatureCrypto::verify of a sealer signature (bcosgpu_secp256k1_verify /
                   bcosgpu_sm2_verify) -- p50;
      catch_up:    1,000 blocks x 7 sealer signatures (a sync catch-up) in one device-resident call:
                   registered keys (bcosgpu_verify_keyed_batch_dev) and unregistered (bcosgpu_verify_batch_dev),
                   HIP events -- sigs/s;
      cpu:         the OpenSSL stand-in on a 7-signature block (1 thread: the reference verifies a block's
                   list in one loop) and on the 7,000 signatures over `threads` threads.
    Every verdict is checked (all signatures valid)."""
    import numpy as np
    import torch
    import bcos_gpu
    from bcos_gpu import _lib, device
    from oracle import oracle
    out, summ = {}, {}
    L = _lib.lib()
    nb = max(reps, 1000)
    for suite in (0, 1):
        name = "secp256k1" if suite == 0 else "sm2"
        g = torch.Generator(device="cuda")
        g.manual_seed(0x5EA1 + suite)

        def signed(sk, h):
            n = sk.shape[0]
            okd = torch.empty(n, dtype=torch.uint8, device="cuda")
            if suite == 0:
                pub = torch.empty((n, 64), dtype=torch.uint8, device="cuda")
                sig = torch.empty((n, 65), dtype=torch.uint8, device="cuda")
                device.secp256k1_sign(sk, h, pub, sig, okd)
            else:
                sig = torch.empty((n, 128), dtype=torch.uint8, device="cuda")
                device.sm2_sign(sk, h, sig, okd)
                pub = sig[:, 64:128].contiguous()
            torch.cuda.synchronize()
            assert bool(okd.all())
            return pub, sig

        def keys(n):
            sk = torch.randint(0, 256, (n, 32), dtype=torch.uint8, device="cuda", generator=g)
            sk[:, 0] &= 0x7F
            sk[:, 31] |= 1
            return sk
        # the committee; block b's sealers 0..k-1 sign its hash
        csk = keys(committee)
        bh = torch.randint(0, 256, (nb, 32), dtype=torch.uint8, device="cuda", generator=g)
        who = torch.arange(nb * 7, device="cuda") % 7
        h7 = bh.repeat_interleave(7, dim=0)
        pub7, sig7 = signed(csk[who], h7)
        crypto = bcos_gpu.SM2Crypto() if suite else bcos_gpu.Secp256k1Crypto()
        cpub, _ = signed(csk, bh[:committee])
        slots = bcos_gpu.register_keys(suite, cpub.cpu().numpy())
        assert (slots >= 0).all()
        P7, H7, S7 = pub7.cpu().numpy(), h7.cpu().numpy(), sig7.cpu().numpy()
        rec = {}
        for k in (4, 7, 32):
            bk = min(reps, 100)
            whok = torch.arange(bk * k, device="cuda") % k
            hk = bh[:bk].repeat_interleave(k, dim=0)
            pk, sk_ = signed(csk[whok], hk)
            Pk, Hk, Sk = pk.cpu().numpy(), hk.cpu().numpy(), sk_.cpu().numpy()
            assert crypto.verify_batch(Pk[:k], Hk[:k], Sk[:k]).all()
            ts = []
            for r in range(bk):
                t0 = time.perf_counter()
                okb = crypto.verify_batch(Pk[r * k:(r + 1) * k], Hk[r * k:(r + 1) * k], Sk[r * k:(r + 1) * k])
                ts.append(time.perf_counter() - t0)
                assert okb.all()
            ts.sort()
            rec["block_%d" % k] = {"p50_ms": ts[len(ts) // 2] * 1e3, "p99_ms": ts[len(ts) * 99 // 100] * 1e3}
        # unregistered: every block's 7 keys new (each seen once, so never promoted)
        ts = []
        for r in range(min(reps, 50)):
            usk = keys(7)
            up, us = signed(usk, bh[r:r + 1].repeat(7, 1))
            UP, US, UH = up.cpu().numpy(), us.cpu().numpy(), bh[r:r + 1].repeat(7, 1).cpu().numpy()
            t0 = time.perf_counter()
            okb = crypto.verify_batch(UP, UH, US)
            ts.append(time.perf_counter() - t0)
            assert okb.all()
        ts.sort()
        rec["unreg_7"] = {"p50_ms": ts[len(ts) // 2] * 1e3}
        ts = []
        for r in range(reps):
            t0 = time.perf_counter()
            assert crypto.verify(P7[r].tobytes(), H7[r].tobytes(), S7[r].tobytes())
            ts.append(time.perf_counter() - t0)
        ts.sort()
        rec["single_p50_ms"] = ts[len(ts) // 2] * 1e3
        stream = torch.cuda.current_stream()
        n = nb * 7
        okd = torch.empty(n, dtype=torch.uint8, device="cuda")
        dslots = torch.from_numpy(slots.astype(np.int32)).cuda()[who]
        stride = sig7.shape[1]

        def keyed():
            device.verify_keyed(suite, dslots, h7, sig7, okd, stream)

        def generic():
            _lib.check(L.bcosgpu_verify_batch_dev(suite, pub7.data_ptr(), h7.data_ptr(), sig7.data_ptr(), stride, n,
                                                  okd.data_ptr(), stream.cuda_stream))
        for lname, fn in (("catch_up_1000x7", keyed), ("catch_up_1000x7_unreg", generic)):
            t0 = time.perf_counter()  # >= 0.5 s of back-to-back launches first (the clock settles under load)
            while time.perf_counter() - t0 < 0.5:
                for _ in range(8):
                    fn()
                torch.cuda.synchronize()
            kt = []
            for _ in range(20):
                a, c = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                fn()
                c.record(stream)
                c.synchronize()
                kt.append(a.elapsed_time(c))
            kt.sort()
            assert bool(okd.all())
            rec[lname] = {"sigs_per_s": n / (kt[len(kt) // 2] * 1e-3), "kernel_ms": kt[len(kt) // 2]}
        cpu = {}
        if oracle.standin() is not None:
            S64 = np.ascontiguousarray(S7[:, :64])
            med, _ = _median_time(lambda: oracle.standin_verify_batch(suite, P7[:7], H7[:7], S64[:7], nthreads=1))
            cpu["block_7_ms"] = med * 1e3
            med, _ = _median_time(lambda: oracle.standin_verify_batch(suite, P7, H7, S64, nthreads=threads), reps=3)
            cpu["catch_up_sigs_per_s"] = n / med
            cpu.update(threads=threads, kind="standin-openssl")
            assert oracle.standin_verify_batch(suite, P7[:64], H7[:64], S64[:64]).all()
        rec["cpu"] = cpu
        rec["key_cache"] = bcos_gpu.key_cache_info(suite)
        out[name] = rec
        summ[name] = {"blk4_p50_ms": _g(rec["block_4"]["p50_ms"]), "blk7_p50_ms": _g(rec["block_7"]["p50_ms"]),
                      "blk32_p50_ms": _g(rec["block_32"]["p50_ms"]), "unreg7_p50_ms": _g(rec["unreg_7"]["p50_ms"]),
                      "single_p50_ms": _g(rec["single_p50_ms"]),
                      "catchup_sig_s": _g(rec["catch_up_1000x7"]["sigs_per_s"]),
                      "catchup_unreg_sig_s": _g(rec["catch_up_1000x7_unreg"]["sigs_per_s"]),
                      "cpu_blk7_ms": _g(cpu.get("block_7_ms")), "cpu_catchup_sig_s": _g(cpu.get("catch_up_sigs_per_s"))}
    out["summary"] = summ
    return out


def create_transaction_leg(b, suite, n, want_status, reps=20):
    """The same batch from raw Tars encodings (createTransaction(bytes, checkSig = true, checkHash = true),
    TransactionFactoryImpl.h:46-85): device decode + pack + verify + hash check, HBM-resident."""
    import torch
    from bcos_gpu import device, synth
    enc, off = synth.tars_encodings(b)
    pre = torch.empty(enc.numel() + 12 * n, dtype=torch.uint8, device="cuda")
    sig = torch.empty(enc.numel(), dtype=torch.uint8, device="cuda")
    pre_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    sig_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    work = torch.empty(device.tars_decode_work_size(n), dtype=torch.uint8, device="cuda")
    th = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
    snd = torch.empty((n, 20), dtype=torch.uint8, device="cuda")
    st = torch.empty(n, dtype=torch.uint8, device="cuda")

    def timed(fn):
        for _ in range(3):
            fn()
        a, c = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        c.record()
        torch.cuda.synchronize()
        return a.elapsed_time(c) / reps

    full = timed(lambda: device.tars_tx_verify(suite, enc, off, pre, pre_off, sig, sig_off, work, th, snd, st,
                                               check_sig=True, check_hash=True))
    same = bool(torch.equal(st, want_status))
    dec = timed(lambda: device.tars_tx_decode(enc, off, pre, pre_off, sig, sig_off, None, work))
    return {"value": n / (full * 1e-3), "unit": "tx/s", "ms_per_batch": full, "decode_ms": dec,
            "bytes_per_tx": enc.numel() // n, "status_matches_packed_path": same,
            "path": "bcosgpu_tars_tx_verify_batch_dev (decode + pack + verify + dataHash check)"}


def devset_legs(devices, min_seconds=1.0):
    """The topology INTEGRATION.md section 2 prescribes: ONE process drives the device list through the C ABI
    a node links (csrc/multi.hip): C4 = configs[3]'s 1M secp256k1 txs as one block through
    bcosgpu_block_verify_multi (index shards, width-2 frontiers gathered on devices[0] by peer copies);
    C5 = configs[4]'s 64 blocks x 20k txs in one bcosgpu_blocks_verify_multi call (whole blocks per device,
    each device's roots by the many-tree level kernel), and c5_seq = one bcosgpu_block_verify_multi call per
    block in order (each block sharded over the devices).
    Host buffers in and out (H2D + kernels + D2H per call: the PCIe-inclusive rate, not `value`).  Each
    leg's root and statuses are checked against the single-device call."""
    import numpy as np
    import bcos_gpu
    from bcos_gpu import synth, tx
    suite = bcos_gpu.secp256k1_suite()
    out = {"devices": list(devices)}
    b = synth.make_batch(0, WORKLOADS["c5"]["n"], seed=0xDE5)
    pre, po = b.pre.cpu().numpy(), b.pre_off.cpu().numpy().astype(np.uint64)
    sg, so = b.sig.cpu().numpy(), b.sig_off.cpu().numpy().astype(np.uint64)
    del b
    per = WORKLOADS["c5"]["n"] // WORKLOADS["c5"]["blocks"]
    n4 = WORKLOADS["c4"]["n"]

    nall = len(po) - 1
    bufs = (np.zeros((nall, 32), np.uint8), np.zeros((nall, 20), np.uint8), np.zeros(nall, np.uint8))

    def c4(devs, out=None):
        return tx.verify_packed_multi(devs, suite, pre, po[: n4 + 1], sg, so[: n4 + 1], width=2, out=out)

    nblk = WORKLOADS["c5"]["blocks"]
    bo = np.arange(nblk + 1, dtype=np.uint64) * np.uint64(per)

    def c5(devs, out=None):  # the 64 blocks in one call, whole blocks per device (bcosgpu_blocks_verify_multi)
        return tx.blocks_verify_multi(devs, suite, pre, po, sg, so, bo, width=2, out=out)

    def c5_seq(devs, out=None):  # one block at a time, each sharded over the devices (bcosgpu_block_verify_multi)
        return [tx.verify_packed_multi(devs, suite, pre, po[k * per: (k + 1) * per + 1], sg,
                                       so[k * per: (k + 1) * per + 1], width=2,
                                       out=None if out is None else tuple(x[k * per:(k + 1) * per] for x in out))
                for k in range(nblk)]

    def _same(g, w):
        return all(np.array_equal(x, y) for x, y in zip(g[:3], w[:3])) and (
            np.array_equal(g[3], w[3]) if isinstance(g[3], np.ndarray) else g[3] == w[3])

    for wl, fn in (("c4", c4), ("c5", c5), ("c5_seq", c5_seq)):
        want = fn([devices[0]])
        got = fn(devices)
        same = _same(got, want) if wl != "c5_seq" else all(_same(g, w) for g, w in zip(got, want))
        ts = []
        t0 = time.perf_counter()
        while len(ts) < 3 or time.perf_counter() - t0 < min_seconds:
            t1 = time.perf_counter()
            fn(devices, out=bufs)  # the caller's reused output buffers
            ts.append(time.perf_counter() - t1)
        ts.sort()
        dt = ts[len(ts) // 2]
        out[wl] = {"tx_s": WORKLOADS[wl.split("_")[0]]["n"] / dt, "ms_per_step": dt * 1e3, "steps": len(ts),
                   "matches_single_device": bool(same)}
    out["note"] = ("host buffers in and out through the chunked copy / compute pipeline (csrc/txpipe.hip); "
                   "median call, output arrays reused across calls as a node reuses its batch buffers")
    return out


def _safe(name, fn):
    """A rank-0 extra leg: its record, or {"error": ...} (traceback on stderr) when it raises -- one failing
    extra leg must not cost the run its line.  (The tx legs run on every rank, collectives included, and
    are not wrapped: a rank that skipped one would hang the others.)"""
    try:
        return fn()
    except Exception as e:  # noqa: BLE001
        import traceback
        traceback.print_exc()
        return {"error": "%s: %s" % (type(e).__name__, e), "leg": name}


def _g(x, k=4):
    return float("%.*g" % (k, x)) if isinstance(x, (int, float)) and not isinstance(x, bool) else x


def summarize(full, head_name):
    """A compact digest of every leg of the full record (the line's `summary`, its last key): per tx leg
    tx/s, ms/step, kernel ms, the executed and SURVEY-8d roofline fractions, HBM traffic over algorithmic
    bytes and the VALU issue fraction; hashes/s; Merkle; the device-set legs; single-call and sealer-verify
    latencies; the CPU baseline."""
    out = {}

    def leg(rec):
        rf = rec["roofline"]
        alg = rf["algorithmic_bytes_per_unit"] * max(rf["units_per_launch"], 1)
        vi = rf.get("valu_issue")
        return {"tx_s": _g(rec["value"]), "ms_step": _g(rec["ms_per_step"]), "kernel_ms": _g(rf["kernel_ms"]),
                "frac": _g(rf["frac"], 3), "useful_8d": _g(rf["algorithmic"]["frac"], 3),
                "traffic_x": _g(rf["traffic"] / alg, 3) if rf.get("traffic") else None,
                "valu_issue": _g(vi["frac"] if isinstance(vi, dict) else vi, 3)}
    out[head_name] = leg(full["head"])
    for k, rec in (full.get("legs") or {}).items():
        out[k] = leg(rec)
    errs = {k: v["error"] for k, v in full.items() if isinstance(v, dict) and "error" in v}
    if errs:
        out["errors"] = {k: v[:200] for k, v in errs.items()}
    full = {k: v for k, v in full.items() if k not in errs}
    hs = full.get("hashes") or {}
    if hs:
        out["hashes[h/s,frac,useful]"] = {k: [_g(v["hashes_per_s"]), _g(v["roofline"]["frac"], 3),
                                              _g(v["roofline"]["useful_frac"], 3)] for k, v in hs.items()}
    mk = full.get("merkle") or {}
    if mk:
        out["merkle[ms,frac,floor]"] = {k: [_g(v["ms"]), _g(v["roofline"]["frac"], 3), _g(v["frac_of_latency_floor"], 3)]
                                        for k, v in mk.items() if isinstance(v, dict) and "ms" in v}
    ds = full.get("devset")
    if ds:
        out["devset"] = {"devices": ds["devices"], **{k: {"tx_s": _g(v["tx_s"]), "ms": _g(v["ms_per_step"]),
                                                          "ok": v["matches_single_device"]}
                                                      for k, v in ds.items() if isinstance(v, dict)}}
    itf = full.get("interface") or {}
    sc = {}
    for k, v in itf.items():
        if k.startswith("single_call_") and isinstance(v, dict) and "calls_per_s" in v:
            t, suite = k[len("single_call_"):].split("_", 1)
            sc.setdefault(suite, {})[t] = [_g(v["calls_per_s"]), _g(v["latency_us"]["p50"]), _g(v["latency_us"]["p99"]),
                                           _g((v.get("cpu_standin") or {}).get("calls_per_s"))]
    if sc:
        out["single_call[gpu/s,p50us,p99us,cpu/s]"] = sc
    rb = {k[len("recover_batch_"):]: _g(v["kernel_ms_median"]) for k, v in itf.items() if k.startswith("recover_batch_")}
    if rb:
        out["recover_batch_10k_ms"] = rb
    sv = full.get("sealer_verify")
    if sv:
        out["sealer_verify"] = sv.get("summary")
    for k in ("pcie_inclusive", "create_transaction"):
        if full.get(k):
            out[k + "_tx_s"] = _g(full[k]["value"])
    if (full.get("pcie_inclusive") or {}).get("verify_packed_tx_s"):
        out["pcie_inclusive_python_tx_s"] = _g(full["pcie_inclusive"]["verify_packed_tx_s"])
    cb = full.get("cpu_baseline")
    if cb:
        out["cpu"] = {"kind": cb["kind"], "threads": cb["cores"],
                      "tx_s": {k: _g(v["value"]) for k, v in cb["legs"].items()},
                      "full_host_est": _g(cb["full_host_estimate"]["value"])}
        mc = cb.get("merkle")
        if mc:
            out["cpu"]["merkle_ms"] = {k: _g(v["ms"]) for k, v in mc["legs"].items() if k.endswith("100k")}
            out["cpu"]["merkle_kind"] = mc["kind"]
    return out


LINE_MAX = 7000  # the driver keeps ~8 kB of stdout and must parse the whole line


def compact_line(full):
    """The ONE line bench.py prints: the contract's head keys, a lean roofline and cpu_baseline and the
    summary of every leg.  Prose, per-leg notes and nested legs stay in the detail file (--detail-out).
    Strict JSON (no NaN / Infinity); under LINE_MAX bytes (tests/test_bench_line.py)."""
    head = full["head"]
    rf = head["roofline"]
    vi = rf.get("valu_issue")
    line = {k: full[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                 "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config")}
    line["roofline"] = {
        "bound": rf["bound"], "achieved": _g(rf["achieved"], 5), "peak": _g(rf["peak"], 5), "unit": rf["unit"],
        "frac": _g(rf["frac"], 4), "useful_8d": _g(rf["algorithmic"]["frac"], 4), "kernel": rf["kernel"],
        "kernel_ms": _g(rf["kernel_ms"], 5), "traffic": _g(rf["traffic"], 5) if rf.get("traffic") else None,
        "valu_issue": _g(vi["frac"] if isinstance(vi, dict) else vi, 4),
        "work": "%d txs x %s" % (rf["units_per_launch"], rf["work_per_unit"].split(" (")[0]),
        "evidence": rf.get("traffic_source")}
    cb = full.get("cpu_baseline")
    if isinstance(cb, dict) and "error" in cb:
        cb = None
    line["cpu_baseline"] = None if not cb else {
        "value": _g(cb["value"], 5), "unit": cb["unit"], "cores": cb["cores"], "kind": cb["kind"],
        "sample": cb["sample"], "full_host_estimate": _g(cb["full_host_estimate"]["value"], 4),
        "physical_cores": cb["full_host_estimate"]["physical_cores"]}
    line["kernel_source_sha"] = full.get("kernel_source_sha")
    line["detail"] = full.get("detail_path")
    line["summary"] = summarize(full, full["head_name"])
    return line


def dumps_line(line):
    """Strict JSON: a NaN or infinity raises instead of printing a line the driver cannot parse."""
    return json.dumps(line, allow_nan=False, separators=(",", ":"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=4500, help="timed steps of the headline (C2) leg")
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--warm-seconds", type=float, default=2.0, help="minimum warm-up before the timed region")
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS), help="the headline leg")
    ap.add_argument("--legs", default="c2sm2,c3,c4,c5", help="comma-separated sub-legs ('' for none)")
    ap.add_argument("--leg-seconds", type=float, default=2.0)
    ap.add_argument("--event-every", type=int, default=16,
                    help="record the kernel-duration HIP events on every N-th timed step (1 = every step)")
    ap.add_argument("--devset", default="auto",
                    help="device list for the one-process device-set legs (C4/C5 through bcosgpu_block_verify_multi): "
                         "'auto' = every rank's GPU when N > 1, {0, 0} at N = 1; 'none' to skip; or e.g. '0,1'")
    ap.add_argument("--detail-out", default=os.path.join("gpurun_out", "bench_detail.json"),
                    help="where rank 0 writes the full record (every leg, notes, nested objects)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-merkle", action="store_true")
    ap.add_argument("--no-hashes", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the PCIe and createTransaction legs")
    ap.add_argument("--launcher-selftest", action="store_true",
                    help="CPU test of the --gpus launcher path only: spawn, rendezvous (gloo), max over ranks; no GPU work")
    args = ap.parse_args()
    global EVENT_EVERY
    EVENT_EVERY = max(1, args.event_every)

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world), file=sys.stderr)
        return 2
    rank = int(os.environ.get("RANK", "0"))

    import torch
    import torch.distributed as dist
    if args.launcher_selftest:
        if world > 1:
            dist.init_process_group("gloo")
        ctx = Ctx(world, rank, dist)
        slowest = ctx.max(rank)
        rec = launcher_selftest_plans(ctx, dist)
        if rank == 0:
            print(json.dumps({"n_gpus": world, "max_over_ranks": slowest, "launcher_selftest": True, **rec}),
                  flush=True)
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return 0
    import bcos_gpu

    local = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    if world > 1:
        # RCCL over xGMI; BCOSGPU_BENCH_BACKEND=gloo rehearses the multi-rank logic on one GPU
        backend = os.environ.get("BCOSGPU_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    bcos_gpu.ensure_device(local)
    ctx = Ctx(world, rank, dist)

    head, head_state = run_leg(ctx, args.workload, steps=args.steps, warmup=args.warmup,
                               warm_seconds=args.warm_seconds)
    legs = {}
    states = {}
    for wl in [x for x in args.legs.split(",") if x and x != args.workload]:
        legs[wl], states[wl] = run_leg(ctx, wl, steps=None, warmup=3, warm_seconds=0.5,
                                       min_seconds=args.leg_seconds)
        if wl not in ("c3",):
            states.pop(wl)
        torch.cuda.empty_cache()

    full = None
    if rank == 0:
        wl = WORKLOADS[args.workload]
        full = {
            "metric": "sigs_per_sec", "value": head["value"], "unit": "tx/s (hash + recover/verify + sender%s)" % (
                " + tx root" if args.workload in ("c4", "c5") else ""),
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": head["ms_per_step"],
            "higher_is_better": True, "scaling": wl["scaling"], "vs_baseline": None,
            "dtype": "u32 (256-bit integer)",
            "data": "synthetic (distinct key per tx, 1%% bit-flipped s, 0.1%% v=4; valid frac %.4f)" % head["valid_frac"],
            "config": {"workload": wl["name"].split(":")[0], "txs_total": head["txs_total"],
                       "txs_rank0": head["txs_rank0"],
                       "parallelism": "dp%d (%s)" % (world, "block shards" if args.workload == "c5" else "tx-index shards"),
                       "timed_s": _g(head["timed_s"], 5)},
            "workload_detail": wl["name"], "warm_seconds": args.warm_seconds,
            "head_name": args.workload, "head": head, "roofline": head["roofline"], "cpu_baseline": None,
            "legs": legs, "kernel_source_sha": kernel_source_sha(),
        }
    # the one-process device-set legs (the node's topology) on rank 0; the other ranks
    # wait on the rendezvous store, not in a collective, so no RCCL kernel spins on their GPUs meanwhile
    devset = None
    if args.devset != "none":
        if args.devset == "auto":
            devset = list(range(world)) if world > 1 and torch.cuda.device_count() >= world else [local, local]
        else:
            devset = [int(x) for x in args.devset.split(",")]
    if devset is not None and rank == 0:
        full["devset"] = _safe("devset", lambda: devset_legs(devset))
    if devset is not None and world > 1:
        store = dist.distributed_c10d._get_default_store()
        if rank == 0:
            store.set("bench_devset_done", "1")
        else:
            store.wait(["bench_devset_done"])
    if rank == 0 and world == 1:
        threads = cpu_threads()
        if not args.no_extras:
            b = head_state["batch"]
            full["pcie_inclusive"] = _safe("pcie_inclusive", lambda: host_api_rate(b, b.suite, head_state["n"]))
            full["create_transaction"] = _safe("create_transaction", lambda: create_transaction_leg(
                b, b.suite, head_state["n"], head_state["status"]))
            from bcos_gpu import synth
            full["interface"] = _safe("interface", lambda: interface_legs(
                [(0, b), (1, synth.make_batch(1, 10_000, seed=0x5A3))]))
            full["sealer_verify"] = _safe("sealer_verify", lambda: sealer_verify_leg(threads))
        if not args.no_hashes:
            full["hashes"] = _safe("hashes", hash_legs)
        if not args.no_merkle:
            full["merkle"] = _safe("merkle", lambda: merkle_legs(0 if args.no_cpu_baseline else threads))
        if not args.no_cpu_baseline:
            def cpu_leg():
                from bcos_gpu import synth
                batches = [(0, head_state["batch"], min(head_state["n"], 20000))]
                sm2 = states.get("c3", {}).get("batch") or synth.make_batch(1, 20000, seed=0x5A2)
                batches.append((1, sm2, 20000))
                cb = cpu_baseline(batches, threads)
                mk = full.get("merkle") or {}
                cb["merkle"] = mk.pop("cpu_baseline", None) if "error" not in mk else None
                return cb
            full["cpu_baseline"] = _safe("cpu_baseline", cpu_leg)
    if rank == 0:
        full["head"] = {k: v for k, v in head.items()}
        full["detail_path"] = args.detail_out
        if args.detail_out:
            d = os.path.dirname(args.detail_out)
            if d:
                os.makedirs(d, exist_ok=True)
            with open(args.detail_out, "w") as f:
                json.dump(full, f, indent=1, default=str)
        print(dumps_line(compact_line(full)), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
