#!/usr/bin/env python3
"""bench.py -- headline benchmark of the MI355X batch-verification engine.

Default workload (BASELINE.json configs[1], "C2"): per GPU, a batch of 10,000 synthetic
secp256k1-signed transactions resident in HBM; one step = one pass of the hot path over the batch:
Keccak256 tx hash of each preimage (TarsHashable.h:16-41) + ECDSA public-key recovery
(Secp256k1Crypto.cpp:79-93) + sender = right160(Keccak256(pub)) (Transaction.h:68-82), i.e.
bcosgpu_tx_verify_batch_dev.  Multi-GPU: one process per GPU, each verifies its own shard (weak
scaling, no data-path collective); rank 0 prints one JSON line with the whole-job rate.

Other BASELINE.json configs (--workload):
  c3  configs[2]: 1M SM2/SM3 txs per GPU (SM3 tx hash + SM2 verify + sender), weak scaling.
  c4  configs[3]: 1M secp256k1 txs in TOTAL, sharded by index over the ranks (width^L-aligned shard
      plan); step = verify the shard + the block tx root (width-2 Keccak Merkle, BlockImpl.h:111-154):
      per-rank frontier, ONE RCCL all-gather over xGMI, top levels on every rank.  Strong scaling.
  c5  configs[4]: PBFT block-verify replay, 64 blocks x 20k txs in TOTAL, blocks sharded over the
      ranks; step = verify every tx of the rank's blocks + each block's tx root
      (bcosgpu_merkle_roots_batch_dev, one launch per tree level for all blocks).  Strong scaling.

Also reported (same line): the roofline of the dominant kernel (tx_verify) from HIP events on the
launch stream, its HBM traffic from the committed rocprofv3 PMC pass of the same workload
(profiles/), the CPU baseline (the oracle restatement, multi-threaded, on a bounded sample, rank 0 at
N=1 only), and the C1 Merkle rate (merkleBench: width-16 root over 100k 32-byte leaves).
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "fisco-bcos_amd"))
sys.path.insert(0, ROOT)

# Algorithmic work per unit, used for roofline.achieved:
#   1 F = one 256-bit modular multiplication = 136 32x32->64 multiply-accumulates (8-limb CIOS)
MAC_PER_F = 136
F_SECP_RECOVER = 3240
F_SM2_VERIFY = 3210
# Field multiplications this implementation actually executes per unit (counted from the kernel
# schedules; the safegcd inversions are ALU work outside the F count, so these are
# lower bounds on issued work). GLV halves the doublings (128 x 7 F) with 66 mixed adds (11 F) and
# 33 phi lookups (1 F), the R table costs ~130 F, u1*G takes 16 mixed adds on the 16-bit comb
# (32 on the 8-bit comb of the small-batch coop/split kernels), sqrt 270, complete add 16, rest ~10.
# SM2: 256 a=-3 doublings x 8 F, 65 Booth mixed adds x 11 F, table ~133 F, comb 176 F, rest ~20.
F_SECP_EXEC_WIDE = 2255
F_SECP_EXEC_COMB8 = 2431
F_SM2_EXEC = 3092
# integer-MAC peak of gfx950 (v_mad_u64_u32 lane-ops/s), measured by fisco-bcos_amd/tools/intbench.hip
# on MI355X (profiles/r01_intbench.json)
PEAK_MAC_PER_S = 3.0785e13
PMC_FILE = os.path.join(ROOT, "profiles", "r01_pmc_{}.json")

WORKLOADS = {
    "c2": dict(suite=0, n=10_000, scaling="weak", metric="sigs_per_sec",
               name="C2: 10k synthetic secp256k1 txs / GPU: Keccak256 tx hash + ECDSA recover + sender"),
    "c3": dict(suite=1, n=1_000_000, scaling="weak", metric="sm2_verify_per_sec",
               name="C3: 1M synthetic SM2/SM3 txs / GPU: SM3 tx hash + SM2 verify + sender"),
    "c4": dict(suite=0, n=1_000_000, scaling="strong", metric="sigs_per_sec",
               name="C4: 1M synthetic secp256k1 txs sharded over the GPUs: tx hash + recover + sender "
                    "+ width-2 Keccak tx root (per-GPU frontier, RCCL all-gather)"),
    "c5": dict(suite=0, n=64 * 20_000, blocks=64, scaling="strong", metric="sigs_per_sec",
               name="C5: PBFT block-verify replay, 64 blocks x 20k secp256k1 txs sharded by block: "
                    "recover + per-block width-2 Keccak tx root"),
}


def _kernel_name(suite, n):
    """Which tx-verify kernel the library launches for this batch (mirrors ecc_kernels.hip policy)."""
    split = os.environ.get("BCOSGPU_TXV_SPLIT")
    if suite == 0 and (split == "1" or (split != "0" and n <= (1 << 15))):
        return "tx_verify_split_kernel" if os.environ.get("BCOSGPU_TXV_COOP") == "0" else "tx_verify_coop_kernel"
    occ = os.environ.get("BCOSGPU_TXV_OCC")
    occ = int(occ) if occ in ("1", "2") else (2 if n >= (1 << 17) else 1)
    return "tx_verify_kernel<%d,%d>" % (suite, occ)


def _norm(name):
    return name.replace("void ", "").replace("bcosgpu::", "").replace(" ", "").split("(")[0]


def _traffic(workload, kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes of this workload
    (tools/prof_summary.py; FETCH_SIZE doubled per MI355X_MICROARCH.md's gfx950 correction)."""
    path = PMC_FILE.format(workload)
    try:
        with open(path) as f:
            pmc = json.load(f)
    except (OSError, ValueError):
        return None, None
    for name, c in pmc.get("kernels", {}).items():
        if _norm(name) == _norm(kernel) and "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            return (2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0, os.path.relpath(path, ROOT)
    return None, None


def _block_plan(nblocks, world, rank):
    per = math.ceil(nblocks / world)
    lo, hi = min(rank * per, nblocks), min((rank + 1) * per, nblocks)
    return lo, hi


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-merkle", action="store_true")
    ap.add_argument("--no-tars", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    import bcos_gpu
    from bcos_gpu import device, parallel, synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
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
    wl = WORKLOADS[args.workload]
    suite = wl["suite"]
    stream = torch.cuda.current_stream()

    # ---- this rank's share of the work
    txroot = None
    block_off = None
    if args.workload == "c4":
        txroot = parallel.gpu_sharded_tx_root(wl["n"], world, rank, device.KECCAK256, 2, "cuda")
        lo, hi = txroot.local_range
        n = hi - lo
    elif args.workload == "c5":
        per_block = wl["n"] // wl["blocks"]
        blo, bhi = _block_plan(wl["blocks"], world, rank)
        n = (bhi - blo) * per_block
        block_off = np.arange(bhi - blo + 1, dtype=np.uint64) * np.uint64(per_block)
        work = torch.empty(max(device.merkle_roots_work_size(n, bhi - blo, 2), 1), dtype=torch.uint8, device="cuda")
        roots = torch.empty((max(bhi - blo, 1), 32), dtype=torch.uint8, device="cuda")
    else:
        n = wl["n"]
    units_total = wl["n"] if wl["scaling"] == "strong" else wl["n"] * world

    # ---- synthetic, device-resident batch of this rank (distinct keys/txs per rank)
    b = synth.make_batch(suite, max(n, 1), seed=0xF15C0BC5 + 7919 * rank)
    txhash = torch.empty((max(n, 1), 32), dtype=torch.uint8, device="cuda")
    sender = torch.empty((max(n, 1), 20), dtype=torch.uint8, device="cuda")
    status = torch.empty(max(n, 1), dtype=torch.uint8, device="cuda")
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]

    def step(k=None):
        if k is not None:
            ev[k][0].record(stream)
        if n:
            device.tx_verify(suite, b.pre, b.pre_off, b.sig, b.sig_off, txhash, sender, status, stream)
        if k is not None:
            ev[k][1].record(stream)
        if txroot is not None:
            txroot(txhash[:n])
        elif block_off is not None and n:
            device.merkle_roots_batch(device.KECCAK256, 2, txhash, block_off, work, roots, stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kernel_ms = sum(a.elapsed_time(c) for a, c in ev) / args.steps  # tx_verify launch, on its stream
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ok_frac = float((status[:n] == 0).float().mean().item()) if n else 1.0

    if rank == 0:
        value = units_total * args.steps / elapsed
        f_per = F_SECP_RECOVER if suite == 0 else F_SM2_VERIFY
        kname = _kernel_name(suite, n)
        achieved = n * f_per * MAC_PER_F / (kernel_ms * 1e-3)
        traffic, traffic_src = _traffic(args.workload, kname)
        roofline = {"bound": "int-valu", "achieved": achieved / 1e12, "peak": PEAK_MAC_PER_S / 1e12,
                    "unit": "TMAC/s", "frac": achieved / PEAK_MAC_PER_S, "traffic": traffic,
                    "traffic_source": traffic_src, "kernel": kname, "kernel_ms": kernel_ms,
                    "units_per_launch": n,
                    "work_per_unit": "%d F x %d MAC (SURVEY.md 8d)" % (f_per, MAC_PER_F)}
        # achieved/frac above use the fixed non-GLV count of SURVEY 8d (useful work per second), which
        # can exceed 1 because GLV and the 16-bit comb execute fewer multiplications; "executed" is
        # the issue-bound fraction for the multiplications the kernel really performs
        if suite == 0:
            f_exec = F_SECP_EXEC_WIDE if kname.startswith("tx_verify_kernel") else F_SECP_EXEC_COMB8
        else:
            f_exec = F_SM2_EXEC
        ex = n * f_exec * MAC_PER_F / (kernel_ms * 1e-3)
        roofline["executed"] = {"f_per_unit": f_exec, "achieved": ex / 1e12, "frac": ex / PEAK_MAC_PER_S,
                                "note": "F counted from the kernel schedule (DESIGN.md 9); inversions excluded"}
        cpu = None
        host_api = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(b, suite, min(n, 20000), args.cpu_threads)
            host_api = host_api_rate(b, suite, n)
        line = {
            "metric": wl["metric"],
            "value": value, "unit": "tx/s (hash + recover/verify + sender%s)" % (
                " + tx root" if args.workload in ("c4", "c5") else ""),
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": wl["scaling"], "vs_baseline": None,
            "dtype": "u32 (256-bit integer)",
            "data": "synthetic (distinct key per tx, 1%% bit-flipped s, 0.1%% v=4; valid frac %.4f)" % ok_frac,
            "config": {"workload": wl["name"], "txs_total": units_total, "txs_rank0": n,
                       "parallelism": "dp%d (%s)" % (world, "block shards" if args.workload == "c5" else "tx-index shards")},
            "roofline": roofline, "cpu_baseline": cpu, "pcie_inclusive": host_api,
        }
        if not args.no_merkle:
            line["merkle_c1"] = merkle_c1()
        if world == 1 and n and not args.no_tars:
            line["create_transaction"] = create_transaction_leg(b, suite, n, status[:n])
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def cpu_baseline(b, suite, sample, threads, min_seconds=1.0):
    """The oracle (C restatement, multi-threaded) on `sample` txs of the same batch, host cores,
    repeated until >= min_seconds of wall time (~16 CPU-seconds at 16 threads)."""
    import numpy as np
    from oracle import oracle
    pre = b.pre.cpu().numpy()
    pre_off = b.pre_off[: sample + 1].cpu().numpy().astype(np.uint64)
    sig = b.sig.cpu().numpy()
    sig_off = b.sig_off[: sample + 1].cpu().numpy().astype(np.uint64)
    oracle.tx_verify_packed(suite, pre, pre_off[:65], sig, sig_off[:65], nthreads=threads)  # warm-up
    reps, t0 = 0, time.perf_counter()
    while True:
        oracle.tx_verify_packed(suite, pre, pre_off, sig, sig_off, nthreads=threads)
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= min_seconds:
            break
    return {"value": reps * sample / dt, "unit": "tx/s", "cores": threads, "kind": "port",
            "sample": "%d x %d txs of the same batch (%.1f s wall), oracle/ C restatement (4x64-bit Montgomery, "
                      "4-bit Straus), %d threads" % (reps, sample, dt, threads)}


def host_api_rate(b, suite, n, reps=5):
    """The same batch through the host-pointer ABI (bcosgpu_tx_verify_batch: H2D copy, kernel, D2H,
    synchronise) -- the PCIe-inclusive rate a caller holding host buffers sees.  Not `value`."""
    import numpy as np
    import bcos_gpu
    from bcos_gpu import tx
    pre = np.ascontiguousarray(b.pre.cpu().numpy())
    pre_off = np.ascontiguousarray(b.pre_off[: n + 1].cpu().numpy().astype(np.uint64))
    sig = np.ascontiguousarray(b.sig.cpu().numpy())
    sig_off = np.ascontiguousarray(b.sig_off[: n + 1].cpu().numpy().astype(np.uint64))
    suite_obj = bcos_gpu.sm_suite() if suite else bcos_gpu.secp256k1_suite()
    tx.verify_packed(suite_obj, pre, pre_off, sig, sig_off)  # warm-up (workspace growth)
    t0 = time.perf_counter()
    for _ in range(reps):
        tx.verify_packed(suite_obj, pre, pre_off, sig, sig_off)
    dt = (time.perf_counter() - t0) / reps
    return {"value": n / dt, "unit": "tx/s", "ms_per_batch": dt * 1e3,
            "path": "bcosgpu_tx_verify_batch (host buffers: H2D + kernel + D2H + sync)"}


def create_transaction_leg(b, suite, n, want_status, reps=20):
    """The same batch from raw Tars encodings (createTransaction(bytes, checkSig = true, checkHash = true),
    TransactionFactoryImpl.h:46-85): device decode + pack + verify + hash check, HBM-resident.  Reported
    beside `value` (which starts from packed preimages); decode_ms is the decode + pack share."""
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


def merkle_c1():
    """C1: merkleBench width-16 Merkle root over 100k leaves (Keccak256 and SM3), device-resident."""
    import numpy as np
    import torch
    from bcos_gpu import device
    n = 100_000
    rng = np.random.default_rng(1)
    leaves = torch.from_numpy(rng.integers(0, 256, size=(n, 32), dtype=np.uint8)).cuda()
    out = {}
    for hname, h in (("keccak256", device.KECCAK256), ("sm3", device.SM3)):
        tree = torch.empty((device.merkle_size(n, 16), 32), dtype=torch.uint8, device="cuda")
        root = torch.empty(32, dtype=torch.uint8, device="cuda")
        for _ in range(3):
            device.merkle_root(h, 16, leaves, tree, root)
        torch.cuda.synchronize()
        reps = 20
        t0 = time.perf_counter()
        for _ in range(reps):
            device.merkle_root(h, 16, leaves, tree, root)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        out[hname] = {"ms": dt * 1e3, "GB_per_s": n * 32 / dt / 1e9}
    return out


if __name__ == "__main__":
    main()
