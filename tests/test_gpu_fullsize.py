"""Full-size parity: the HIP path at BASELINE.json's own config sizes against the oracle -- every tx
hash, every verdict, every sender, every root.  These batches run the throughput kernels the bench
measures (occupancy-2 tx_verify_kernel with the 16-bit comb tables, the sharded width-2 tx root, the
many-block root kernel), which smaller tests reach only through forced variants.

  C3  configs[2]: 1M SM2/SM3 txs (SM2Crypto.cpp:66-92, fast_sm2.cpp:139-227)
  C4  configs[3]: 1M secp256k1 txs + the width-2 Keccak tx root through the sharded-root path at
      world 1 (TransactionSync.cpp:516-548, BlockImpl.h:111-154)
  C5  configs[4]: 64 blocks x 20k secp256k1 txs + 64 per-block tx roots (merkle_roots_batch)

The oracle (multi-threaded C restatement) needs ~1 min of the box's CPU share per million txs.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _threads():
    env = os.environ.get("OMP_NUM_THREADS")
    aff = len(os.sched_getaffinity(0))
    return min(int(env), aff) if env and env.isdigit() and int(env) > 0 else aff


def _verify(suite, b):
    import torch
    from bcos_gpu import device
    n = b.n
    th = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
    snd = torch.empty((n, 20), dtype=torch.uint8, device="cuda")
    st = torch.empty(n, dtype=torch.uint8, device="cuda")
    device.tx_verify(suite, b.pre, b.pre_off, b.sig, b.sig_off, th, snd, st)
    torch.cuda.synchronize()
    return th, snd, st


def _oracle_verify(oracle, suite, b):
    pre, po, sg, so = (x.cpu().numpy() for x in (b.pre, b.pre_off, b.sig, b.sig_off))
    return oracle.tx_verify_packed(suite, pre, po.astype(np.uint64), sg, so.astype(np.uint64), nthreads=_threads())


def _check_all(th, snd, st, want, b, suite):
    wh, ws, wst = want
    assert np.array_equal(th.cpu().numpy(), wh)
    st_h = st.cpu().numpy()
    assert np.array_equal(st_h, wst)
    assert np.array_equal(snd.cpu().numpy(), ws)
    assert (st_h[b.corrupted == 0] == 0).all()
    if suite == 1:
        assert (st_h[b.corrupted == 1] == 1).all()
    else:
        assert (st_h[b.corrupted == 2] == 1).all()


@pytest.mark.timeout(600)
def test_c3_1m_sm2(gpu, oracle):
    from bcos_gpu import synth
    b = synth.make_batch(1, 1_000_000, seed=0xC3)
    th, snd, st = _verify(1, b)
    _check_all(th, snd, st, _oracle_verify(oracle, 1, b), b, 1)


@pytest.mark.timeout(600)
def test_c4_1m_secp256k1_and_tx_root(gpu, oracle):
    import torch
    from bcos_gpu import device, parallel, synth
    n = 1_000_000
    b = synth.make_batch(0, n, seed=0xC4)
    th, snd, st = _verify(0, b)
    want = _oracle_verify(oracle, 0, b)
    _check_all(th, snd, st, want, b, 0)
    root = parallel.gpu_sharded_tx_root(n, 1, 0, device.KECCAK256, 2, "cuda")(th)
    torch.cuda.synchronize()
    assert root.cpu().numpy().tobytes() == oracle.merkle(oracle.KECCAK256, 2, want[0], nthreads=_threads())


@pytest.mark.timeout(600)
def test_c5_64_blocks_x_20k(gpu, oracle):
    import torch
    from bcos_gpu import device, synth
    nb, per = 64, 20_000
    n = nb * per
    b = synth.make_batch(0, n, seed=0xC5)
    th, snd, st = _verify(0, b)
    want = _oracle_verify(oracle, 0, b)
    _check_all(th, snd, st, want, b, 0)
    block_off = np.arange(nb + 1, dtype=np.uint64) * np.uint64(per)
    work = torch.empty(device.merkle_roots_work_size(n, nb, 2), dtype=torch.uint8, device="cuda")
    roots = torch.empty((nb, 32), dtype=torch.uint8, device="cuda")
    device.merkle_roots_batch(device.KECCAK256, 2, th, block_off, work, roots)
    torch.cuda.synchronize()
    got = roots.cpu().numpy()
    for k in range(nb):
        assert got[k].tobytes() == oracle.merkle(oracle.KECCAK256, 2, want[0][k * per:(k + 1) * per]), k


@pytest.mark.timeout(600)
@pytest.mark.parametrize("suite", [0, 1])
def test_c4_8gpu_shard_size(gpu, oracle, suite):
    """One rank's C4 shard at world 8 (parallel.shard_plan: 125,952 txs, width^L-aligned): the size the
    scaling run launches per GPU, where the rounds x latency rule picks the occupancy-2 one-lane kernel
    (profiles/r03_occ_sweep.json: 1.71 vs 1.99 ms at occupancy 1).  Both suites against the oracle,
    plus the SigIO recover / SM2-verify batch at the same size."""
    import torch
    from bcos_gpu import device, parallel, synth
    n = 125_952
    plan = parallel.gpu_sharded_tx_root(1_000_000, 8, 0, device.KECCAK256, 2, "cuda")
    assert plan.local_range == (0, n)
    b = synth.make_batch(suite, n, seed=0xC48 + suite)
    th, snd, st = _verify(suite, b)
    want = _oracle_verify(oracle, suite, b)
    _check_all(th, snd, st, want, b, suite)
    sigs = b.sig.view(n, b.sig_len)
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    addr = torch.empty((n, 20), dtype=torch.uint8, device="cuda")
    if suite == 0:
        pub = torch.empty((n, 64), dtype=torch.uint8, device="cuda")
        device.secp256k1_recover(th, sigs, pub, addr, ok)
    else:
        device.sm2_verify(th, sigs, addr, ok)
    torch.cuda.synchronize()
    assert np.array_equal(ok.cpu().numpy(), (want[2] == 0).astype(np.uint8))
    assert np.array_equal(addr.cpu().numpy(), want[1])
