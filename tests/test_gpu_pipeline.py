"""The host-pointer tx batches' chunked copy / compute pipeline (csrc/txpipe.hip): bcosgpu_tx_verify_batch
(TransactionSync.cpp:516-548's batch site), the device-set shards (bcosgpu_block_verify_multi /
bcosgpu_blocks_verify_multi, BlockImpl.h:111-154) and concurrent callers on one device (TxPool.h:48-49).
  - chunk boundaries at oracle-sized batches: BCOSGPU_PIPE_CHUNK (read per call) forces small chunks, so
    batches of one chunk +- 1 tx, several chunks and a 1-tx tail run against the oracle, both suites;
  - offsets that do not start at 0 (a sub-range of a caller's packed buffer: the pipeline indexes the
    device copy with the caller's own offsets);
  - the default chunking at full size (2 rounds + 1 tx of the occupancy-2 kernel: 3 chunks, the last one
    a single tx) against the device-resident single launch and a sampled oracle;
  - several host threads calling at once (each on its own pipeline of the pool)."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _host(b):
    return (b.pre.cpu().numpy(), b.pre_off.cpu().numpy().astype(np.uint64), b.sig.cpu().numpy(),
            b.sig_off.cpu().numpy().astype(np.uint64))


def _suite(gpu, suite):
    return gpu.sm_suite() if suite else gpu.secp256k1_suite()


@pytest.mark.parametrize("suite", [0, 1])
def test_pipeline_chunk_boundaries_vs_oracle(gpu, oracle, suite, monkeypatch):
    from bcos_gpu import synth, tx
    b = synth.make_batch(suite, 3001, seed=0x91 + suite, flip_frac=0.05, bad_v_frac=0.02)
    pre, po, sg, so = _host(b)
    wh, ws, wst = oracle.tx_verify_packed(suite, pre, po, sg, so, nthreads=8)
    s = _suite(gpu, suite)
    monkeypatch.setenv("BCOSGPU_PIPE_CHUNK", "1000")
    for n in (999, 1000, 1001, 2000, 2999, 3000, 3001):
        th, snd, st = tx.verify_packed(s, pre, po[: n + 1], sg, so[: n + 1])
        assert np.array_equal(th, wh[:n]) and np.array_equal(snd, ws[:n]) and np.array_equal(st, wst[:n]), n
    # a sub-range whose offsets start inside the buffers (pre_off[0] != 0), split into chunks of 7
    monkeypatch.setenv("BCOSGPU_PIPE_CHUNK", "7")
    for lo, hi in ((5, 6), (5, 40), (1000, 1301)):
        th, snd, st = tx.verify_packed(s, pre, po[lo: hi + 1], sg, so[lo: hi + 1])
        assert np.array_equal(th, wh[lo:hi]) and np.array_equal(st, wst[lo:hi]) and np.array_equal(snd, ws[lo:hi])
    # device sets: every shard multi-chunk, the roots behind the last chunk
    monkeypatch.setenv("BCOSGPU_PIPE_CHUNK", "333")
    hasher = oracle.SM3 if suite else oracle.KECCAK256
    for devs in ([0], [0, 0], [0, 0, 0]):
        th, snd, st, root = tx.verify_packed_multi(devs, s, pre, po, sg, so, width=2)
        assert np.array_equal(th, wh) and np.array_equal(snd, ws) and np.array_equal(st, wst), devs
        assert root == oracle.merkle(hasher, 2, wh), devs
        bo = np.array([0, 0, 1, 500, 1999, 1999, 3001], dtype=np.uint64)
        th, snd, st, roots = tx.blocks_verify_multi(devs, s, pre, po, sg, so, bo, width=2)
        assert np.array_equal(th, wh) and np.array_equal(st, wst), devs
        want = [oracle.merkle(hasher, 2, wh[int(bo[k]):int(bo[k + 1])]) if bo[k + 1] > bo[k] else bytes(32)
                for k in range(len(bo) - 1)]
        assert [r.tobytes() for r in roots] == want, devs


@pytest.mark.timeout(600)
def test_pipeline_default_chunks_full_size(gpu, oracle):
    """2 x 512 x CUs + 1 secp256k1 txs through the host-pointer path (the default chunking: a quarter-round
    head chunk, a full round of the occupancy-2 kernel, the rest) == the device-resident single launch, and
    with the head chunk off (two full rounds, then one tx); the oracle on every tx around every chunk
    boundary and on a 1-in-509 sample."""
    import torch
    from bcos_gpu import device, synth, tx
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    c = 512 * cus
    n = 2 * c + 1
    b = synth.make_batch(0, n, seed=0xF11, flip_frac=0.01, bad_v_frac=0.001)
    th_d = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
    snd_d = torch.empty((n, 20), dtype=torch.uint8, device="cuda")
    st_d = torch.empty(n, dtype=torch.uint8, device="cuda")
    device.tx_verify(0, b.pre, b.pre_off, b.sig, b.sig_off, th_d, snd_d, st_d)
    torch.cuda.synchronize()
    pre, po, sg, so = _host(b)
    import os
    for head in ("1", "0"):
        os.environ["BCOSGPU_PIPE_HEAD"] = head
        try:
            th, snd, st = tx.verify_packed(gpu.secp256k1_suite(), pre, po, sg, so)
        finally:
            os.environ.pop("BCOSGPU_PIPE_HEAD")
        assert np.array_equal(th, th_d.cpu().numpy()), head
        assert np.array_equal(snd, snd_d.cpu().numpy()), head
        assert np.array_equal(st, st_d.cpu().numpy()), head
    q = c // 4
    idx = sorted(set(range(q - 3, q + 3)) | set(range(q + c - 3, q + c + 3)) | set(range(c - 3, c + 3))
                 | set(range(2 * c - 3, n)) | set(range(0, n, 509)))
    idx = np.array(idx)
    pre_l = [pre[int(po[i]):int(po[i + 1])].tobytes() for i in idx]
    sig_l = [sg[int(so[i]):int(so[i + 1])].tobytes() for i in idx]
    from bcos_gpu.crypto import pack_messages
    p2, o2 = pack_messages(pre_l)
    s2, t2 = pack_messages(sig_l)
    wh, ws, wst = oracle.tx_verify_packed(0, p2, o2.astype(np.uint64), s2, t2.astype(np.uint64), nthreads=8)
    assert np.array_equal(th[idx], wh) and np.array_equal(snd[idx], ws) and np.array_equal(st[idx], wst)
    assert 0 < int((st != 0).sum()) < n // 10


def test_pipeline_concurrent_callers(gpu, oracle):
    """Six host threads each verifying its own batch (sizes 1 .. 40,000, both suites) at once, twice:
    each call on its own pipeline from the device's pool; every result equals the oracle's."""
    from bcos_gpu import synth, tx
    jobs = []
    for k, (suite, n) in enumerate(((0, 1), (1, 7), (0, 10_000), (1, 4_000), (0, 40_000), (1, 257))):
        b = synth.make_batch(suite, n, seed=0xCC0 + k, flip_frac=0.05, bad_v_frac=0.02)
        pre, po, sg, so = _host(b)
        jobs.append((suite, (pre, po, sg, so), oracle.tx_verify_packed(suite, pre, po, sg, so, nthreads=8)))
    errors = []

    def run(j):
        suite, args, want = jobs[j]
        try:
            for _ in range(2):
                got = tx.verify_packed(_suite(gpu, suite), *args)
                if not all(np.array_equal(x, y) for x, y in zip(got, want)):
                    errors.append(("mismatch", j))
        except Exception as e:  # noqa: BLE001
            errors.append((repr(e), j))
    th = [threading.Thread(target=run, args=(j,)) for j in range(len(jobs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors


def test_pipeline_rejects_bad_offsets_mid_batch(gpu, oracle, monkeypatch):
    """Offsets are checked chunk by chunk inside the pipeline: a decreasing offset in the third chunk is
    BCOSGPU_E_ARG (after the chunks already launched have drained), for the single-device and the
    device-set calls; the same pipelines then verify a good batch correctly."""
    from bcos_gpu import synth, tx
    from bcos_gpu._lib import E_ARG, BcosGpuError
    b = synth.make_batch(0, 900, seed=0xBAD0)
    pre, po, sg, so = _host(b)
    s = gpu.secp256k1_suite()
    monkeypatch.setenv("BCOSGPU_PIPE_CHUNK", "100")
    bad_po, bad_so = po.copy(), so.copy()
    bad_po[250] = bad_po[249] - 1
    bad_so[250] = bad_so[249] - 1
    for args in ((pre, bad_po, sg, so), (pre, po, sg, bad_so)):
        with pytest.raises(BcosGpuError) as e:
            tx.verify_packed(s, *args)
        assert e.value.code == E_ARG
        with pytest.raises(BcosGpuError) as e:
            tx.verify_packed_multi([0, 0], s, *args, width=2)
        assert e.value.code == E_ARG
    wh, ws, wst = oracle.tx_verify_packed(0, pre, po, sg, so, nthreads=8)
    th, snd, st = tx.verify_packed(s, pre, po, sg, so)
    assert np.array_equal(th, wh) and np.array_equal(snd, ws) and np.array_equal(st, wst)
