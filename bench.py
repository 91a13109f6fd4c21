#!/usr/bin/env python3
"""bench.py -- headline benchmark of the MI355X batch-verification engine.

Workload (BASELINE.json configs[1], "C2"): per GPU, a batch of 10,000 synthetic secp256k1-signed
transactions resident in HBM; one step = one pass of the hot path over the batch:
Keccak256 tx hash of each preimage (TarsHashable.h:16-41) + ECDSA public-key recovery
(Secp256k1Crypto.cpp:79-93) + sender = right160(Keccak256(pub)) (Transaction.h:68-82), i.e.
bcosgpu_tx_verify_batch_dev.  --workload c3 runs configs[2] instead (1M SM2/SM3 txs on one GPU).
Multi-GPU: one process per GPU, each verifies its own shard (weak scaling, no data-path
collective); rank 0 prints one JSON line with the whole-job rate.

Also reported (same line): the roofline of the dominant kernel from HIP events on the launch stream,
the CPU baseline (the oracle restatement, multi-threaded, on a bounded sample), and the C1 Merkle
rate (merkleBench: width-16 root over 100k 32-byte leaves).
"""
import argparse
import json
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
# integer-MAC peak of gfx950 (v_mad_u64_u32 lane-ops/s), measured by fisco-bcos_amd/tools/intbench.hip
# on MI355X (profiles/r01_intbench.json)
PEAK_MAC_PER_S = 3.0785e13

WORKLOADS = {
    "c2": dict(suite=0, n=10_000, name="C2: 10k synthetic secp256k1 txs / GPU: Keccak256 tx hash + ECDSA recover + sender"),
    "c3": dict(suite=1, n=1_000_000, name="C3: 1M synthetic SM2/SM3 txs / GPU: SM3 tx hash + SM2 verify + sender"),
}


def _kernel_name(suite, n):
    """Which tx-verify kernel the library launches for this batch (mirrors ecc_kernels.hip policy)."""
    split = os.environ.get("BCOSGPU_TXV_SPLIT")
    if suite == 0 and (split == "1" or (split != "0" and n <= (1 << 15))):
        return "tx_verify_split_kernel"
    occ = os.environ.get("BCOSGPU_TXV_OCC")
    occ = int(occ) if occ in ("1", "2") else (2 if n >= (1 << 17) else 1)
    return "tx_verify_kernel<%d,%d>" % (suite, occ)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    import bcos_gpu
    from bcos_gpu import device, synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    bcos_gpu.ensure_device(local)
    wl = WORKLOADS[args.workload]
    suite, n = wl["suite"], wl["n"]

    # ---- synthetic, device-resident shard of this rank (distinct keys/txs per rank)
    b = synth.make_batch(suite, n, seed=0xF15C0BC5 + 7919 * rank)
    txhash = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
    sender = torch.empty((n, 20), dtype=torch.uint8, device="cuda")
    status = torch.empty(n, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream()

    def step():
        device.tx_verify(suite, b.pre, b.pre_off, b.sig, b.sig_off, txhash, sender, status, stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / args.steps  # one tx_verify kernel per step on this stream
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ok_frac = float((status == 0).float().mean().item())

    if rank == 0:
        total = n * world * args.steps
        value = total / elapsed
        f_per = F_SECP_RECOVER if suite == 0 else F_SM2_VERIFY
        achieved = n * f_per * MAC_PER_F / (kernel_ms * 1e-3)
        roofline = {"bound": "int-valu", "achieved": achieved / 1e12, "peak": PEAK_MAC_PER_S / 1e12,
                    "unit": "TMAC/s", "frac": achieved / PEAK_MAC_PER_S, "traffic": None,
                    "kernel": _kernel_name(suite, n), "kernel_ms": kernel_ms,
                    "work_per_unit": "%d F x %d MAC (SURVEY.md 8d)" % (f_per, MAC_PER_F)}
        cpu = None
        if not args.no_cpu_baseline:
            cpu = cpu_baseline(b, suite, min(n, 20000), args.cpu_threads)
        merkle = merkle_c1()
        line = {
            "metric": "sigs_per_sec" if suite == 0 else "sm2_verify_per_sec",
            "value": value, "unit": "tx/s (hash + recover/verify + sender)", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32 (256-bit integer)",
            "data": "synthetic (distinct key per tx, 1%% bit-flipped s, 0.1%% v=4; valid frac %.4f)" % ok_frac,
            "config": {"workload": wl["name"], "txs_per_gpu": n, "parallelism": "dp%d (tx-index shards)" % world},
            "roofline": roofline, "cpu_baseline": cpu, "merkle_c1": merkle,
        }
        print(json.dumps(line))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def cpu_baseline(b, suite, sample, threads):
    """The oracle (C restatement, multi-threaded) on `sample` txs of the same batch, host cores."""
    import numpy as np
    from oracle import oracle
    pre = b.pre.cpu().numpy()
    pre_off = b.pre_off[: sample + 1].cpu().numpy().astype(np.uint64)
    sig = b.sig.cpu().numpy()
    sig_off = b.sig_off[: sample + 1].cpu().numpy().astype(np.uint64)
    oracle.tx_verify_packed(suite, pre, pre_off[:65], sig, sig_off[:65], nthreads=threads)  # warm-up
    t0 = time.perf_counter()
    oracle.tx_verify_packed(suite, pre, pre_off, sig, sig_off, nthreads=threads)
    dt = time.perf_counter() - t0
    return {"value": sample / dt, "unit": "tx/s", "cores": threads, "kind": "port",
            "sample": "%d txs of the same batch, oracle/ C restatement (4x64-bit Montgomery, 4-bit Straus), %d threads" % (sample, threads)}


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
