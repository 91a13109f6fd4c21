"""Multi-GPU behind the C ABI a FISCO node links (include/bcos_gpu.h "device sets", csrc/multi.hip): one
process, a device list, batches sharded by index over it (TransactionSync.cpp:516-548) and the block tx
root from per-GPU frontiers gathered on the first device (BlockImpl.h:111-154).

The box has one GPU, so the device lists repeat device 0 ({0, 0}, {0, 0, 0}): every shard still runs from
its own host thread on its own stream and buffers, and the frontier gather is the same code (a device-local
copy; BCOSGPU_MULTI_PEER=1 sends it through the hipMemcpyPeerAsync branch that distinct devices take --
across two physical GPUs that branch is still unmeasured on hardware).  Everything is compared with the
oracle."""
import os
import struct
import subprocess

import numpy as np
import pytest

from test_cpp_adapter import LIBDIR, ROOT


def _build(tmp_path):
    exe = str(tmp_path / "multi_test")
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-o", exe,
                    os.path.join(ROOT, "tests", "cpp", "multi_test.cpp"), "-L" + LIBDIR, "-lbcosgpu",
                    "-Wl,-rpath," + LIBDIR], check=True)
    return exe


def test_multi_test_compiles(tmp_path):
    exe = _build(tmp_path)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2  # usage


def test_device_set_argument_errors_without_gpu():
    """Argument errors come back before any device is touched; without a GPU the set is BCOSGPU_E_NODEV."""
    import ctypes
    from bcos_gpu import _lib
    L = _lib.lib()
    assert L.bcosgpu_init_devices(None, 0) == _lib.E_ARG
    devs = (ctypes.c_int * 65)()
    assert L.bcosgpu_init_devices(devs, 65) == _lib.E_ARG
    root = ctypes.create_string_buffer(32)
    assert L.bcosgpu_merkle_root_multi(devs, 1, 0, 2, None, 0, root) == _lib.E_EMPTY
    assert L.bcosgpu_merkle_root_multi(devs, 1, 0, 1, None, 0, root) == _lib.E_ARG  # width
    assert L.bcosgpu_block_verify_multi(devs, 1, 0, None, None, None, None, 0, 2, None, None, None, None) == _lib.E_ARG
    assert L.bcosgpu_block_verify_multi(devs, 1, 5, None, None, None, None, 0, 2, None, None, None, root) == _lib.E_ARG
    bo = (ctypes.c_uint64 * 3)(1, 2, 3)
    assert L.bcosgpu_blocks_verify_multi(devs, 1, 0, None, None, None, None, bo, 2, 2, None, None, None, root) == _lib.E_ARG
    bo = (ctypes.c_uint64 * 3)(0, 2, 1)  # decreasing
    assert L.bcosgpu_blocks_verify_multi(devs, 1, 0, None, None, None, None, bo, 2, 2, None, None, None, root) == _lib.E_ARG
    assert L.bcosgpu_blocks_verify_multi(devs, 1, 0, None, None, None, None, bo, 2, 1, None, None, None, root) == _lib.E_ARG
    if L.bcosgpu_device_count() == 0:
        assert L.bcosgpu_init_devices(devs, 1) == _lib.E_NODEV


def _threads():
    env = os.environ.get("OMP_NUM_THREADS")
    aff = len(os.sched_getaffinity(0))
    return min(int(env), aff) if env and env.isdigit() and int(env) > 0 else aff


def _host(b):
    return (b.pre.cpu().numpy(), b.pre_off.cpu().numpy().astype(np.uint64), b.sig.cpu().numpy(),
            b.sig_off.cpu().numpy().astype(np.uint64))


@pytest.mark.gpu
@pytest.mark.parametrize("suite", [0, 1])
def test_device_sets_match_oracle(gpu, oracle, suite):
    """bcosgpu_block_verify_multi / _tx_verify_batch_multi / _merkle_root_multi over device lists of 1-3
    entries, sizes from 1 tx to 20,001 (shards empty, ragged, width^L-aligned), widths 2 and 16: every hash,
    verdict, sender and root equals the oracle's."""
    from bcos_gpu import synth, tx
    suite_obj = gpu.sm_suite() if suite else gpu.secp256k1_suite()
    hasher = oracle.SM3 if suite else oracle.KECCAK256
    for n in (1, 2, 3, 1000, 20_001):
        b = synth.make_batch(suite, n, seed=0x3A + n + suite, flip_frac=0.05, bad_v_frac=0.02)
        pre, po, sg, so = _host(b)
        wh, ws, wst = oracle.tx_verify_packed(suite, pre, po, sg, so, nthreads=_threads())
        for devs in ([0], [0, 0], [0, 0, 0]):
            th, snd, st = tx.verify_packed_multi(devs, suite_obj, pre, po, sg, so)
            assert np.array_equal(th, wh) and np.array_equal(snd, ws) and np.array_equal(st, wst), (n, devs)
            for width in (2, 16):
                th, snd, st, root = tx.verify_packed_multi(devs, suite_obj, pre, po, sg, so, width=width)
                want_root = oracle.merkle(hasher, width, wh)
                assert np.array_equal(st, wst) and np.array_equal(th, wh), (n, devs, width)
                assert root == want_root, (n, devs, width)
                assert tx.merkle_root_multi(devs, hasher, width, wh) == want_root, (n, devs, width)
    # BlockImpl.h:114-119: no transactions -> the zero root
    e8, e64 = np.zeros(1, np.uint8), np.zeros(1, np.uint64)
    assert tx.verify_packed_multi([0, 0], suite_obj, e8, e64, e8, e64, width=2)[3] == bytes(32)


@pytest.mark.gpu
@pytest.mark.parametrize("suite", [0, 1])
def test_device_sets_peer_copy_branch(gpu, oracle, suite, monkeypatch):
    """The cross-device code of the device-set path on a one-GPU box: BCOSGPU_MULTI_PEER=1 (read by
    multi.hip at each call) sends shards that live on devices[0] itself through enable_peers' probe and
    the hipMemcpyPeerAsync frontier gather (multi.hip gather_root) -- the branch a node with several GPUs
    takes.  Every root, hash, verdict and sender against the oracle at sizes whose shards are empty,
    ragged and width^L-aligned; device lists {0, 0} and {0, 0, 0}."""
    from bcos_gpu import synth, tx
    monkeypatch.setenv("BCOSGPU_MULTI_PEER", "1")
    suite_obj = gpu.sm_suite() if suite else gpu.secp256k1_suite()
    hasher = oracle.SM3 if suite else oracle.KECCAK256
    for n in (2, 999, 20_001, 65_537):
        b = synth.make_batch(suite, n, seed=0x9E + n + suite, flip_frac=0.05, bad_v_frac=0.02)
        pre, po, sg, so = _host(b)
        wh, ws, wst = oracle.tx_verify_packed(suite, pre, po, sg, so, nthreads=_threads())
        for devs in ([0, 0], [0, 0, 0]):
            for width in (2, 16):
                th, snd, st, root = tx.verify_packed_multi(devs, suite_obj, pre, po, sg, so, width=width)
                want_root = oracle.merkle(hasher, width, wh)
                assert np.array_equal(st, wst) and np.array_equal(th, wh) and np.array_equal(snd, ws), (n, devs)
                assert root == want_root, (n, devs, width)
                assert tx.merkle_root_multi(devs, hasher, width, wh) == want_root, (n, devs, width)


@pytest.mark.gpu
@pytest.mark.parametrize("suite", [0, 1])
def test_many_blocks_over_device_sets(gpu, oracle, suite):
    """bcosgpu_blocks_verify_multi (a sync catch-up / configs[4]'s replay in one call): 37 blocks of 0 to
    3,000 txs (empty and one-tx blocks included) over {0}, {0, 0}, {0, 0, 0}: every hash, sender and
    verdict, and every block's root (width 2 and 16; the zero hash for an empty block, BlockImpl.h:114-119)
    against the oracle."""
    from bcos_gpu import synth, tx
    rng = np.random.default_rng(0xB10C + suite)
    sizes = [int(x) for x in rng.integers(0, 3000, size=37)]
    sizes[3], sizes[4], sizes[20] = 0, 1, 0
    bo = np.zeros(len(sizes) + 1, dtype=np.uint64)
    bo[1:] = np.cumsum(sizes)
    n = int(bo[-1])
    b = synth.make_batch(suite, n, seed=0x77 + suite, flip_frac=0.05, bad_v_frac=0.02)
    pre, po, sg, so = _host(b)
    wh, ws, wst = oracle.tx_verify_packed(suite, pre, po, sg, so, nthreads=_threads())
    hasher = oracle.SM3 if suite else oracle.KECCAK256
    suite_obj = gpu.sm_suite() if suite else gpu.secp256k1_suite()
    for width in (2, 16):
        want_roots = [oracle.merkle(hasher, width, wh[int(bo[k]):int(bo[k + 1])]) if sizes[k] else bytes(32)
                      for k in range(len(sizes))]
        for devs in ([0], [0, 0], [0, 0, 0]):
            th, snd, st, roots = tx.blocks_verify_multi(devs, suite_obj, pre, po, sg, so, bo, width=width)
            assert np.array_equal(th, wh) and np.array_equal(snd, ws) and np.array_equal(st, wst), (devs, width)
            assert [r.tobytes() for r in roots] == want_roots, (devs, width)


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_c4_1m_block_on_two_shards_through_cpp(gpu, oracle, tmp_path):
    """configs[3]'s 1M secp256k1 txs as ONE block through the C ABI from a C++ process (tests/cpp/multi_test.cpp)
    with the device list {0, 0}: two shards on two streams, width-2 Keccak tx root from their frontiers --
    every tx hash, sender, verdict and the root against the oracle, plus the sharded recover batch."""
    from bcos_gpu import synth
    n = 1_000_000
    b = synth.make_batch(0, n, seed=0xC4)
    pre, po, sg, so = _host(b)
    wh, ws, wst = oracle.tx_verify_packed(0, pre, po, sg, so, nthreads=_threads())
    root = oracle.merkle(oracle.KECCAK256, 2, wh, nthreads=_threads())
    data = str(tmp_path / "block.bin")
    with open(data, "wb") as f:
        f.write(b"BGMT" + struct.pack("<III", 0, n, 2))
        f.write(struct.pack("<Q", pre.size) + pre.tobytes() + po.tobytes())
        f.write(struct.pack("<Q", sg.size) + sg.tobytes() + so.tobytes())
        for a in (wh, ws, wst):
            f.write(np.ascontiguousarray(a, dtype=np.uint8).tobytes())
        f.write(root)
    exe = _build(tmp_path)
    r = subprocess.run([exe, data, "0,0"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "multi_test: ok" in r.stdout


@pytest.mark.gpu
def test_eight_entry_device_list_peer_branch(gpu, oracle, monkeypatch):
    """The list an 8-GPU node passes, {0} x 8 on this one-GPU box, with BCOSGPU_MULTI_PEER=1 (the
    cross-device branches: peer-access probe, hipMemcpyPeerAsync frontier gather): one block through
    bcosgpu_block_verify_multi (8 shards, width 2 and 16) and 64 blocks of 0 .. 700 txs through
    bcosgpu_blocks_verify_multi (whole blocks per entry) -- every hash, sender, verdict and root against the
    oracle."""
    from bcos_gpu import synth, tx
    monkeypatch.setenv("BCOSGPU_MULTI_PEER", "1")
    rng = np.random.default_rng(0x8E)
    sizes = [int(x) for x in rng.integers(0, 700, size=64)]
    sizes[0], sizes[17], sizes[63] = 0, 1, 0
    bo = np.zeros(len(sizes) + 1, dtype=np.uint64)
    bo[1:] = np.cumsum(sizes)
    n = int(bo[-1])
    b = synth.make_batch(0, n, seed=0x8E8, flip_frac=0.05, bad_v_frac=0.02)
    pre, po, sg, so = _host(b)
    wh, ws, wst = oracle.tx_verify_packed(0, pre, po, sg, so, nthreads=_threads())
    s = gpu.secp256k1_suite()
    devs = [0] * 8
    for width in (2, 16):
        th, snd, st, root = tx.verify_packed_multi(devs, s, pre, po, sg, so, width=width)
        assert np.array_equal(th, wh) and np.array_equal(snd, ws) and np.array_equal(st, wst), width
        assert root == oracle.merkle(oracle.KECCAK256, width, wh), width
    th, snd, st, roots = tx.blocks_verify_multi(devs, s, pre, po, sg, so, bo, width=2)
    assert np.array_equal(th, wh) and np.array_equal(snd, ws) and np.array_equal(st, wst)
    want = [oracle.merkle(oracle.KECCAK256, 2, wh[int(bo[k]):int(bo[k + 1])]) if sizes[k] else bytes(32)
            for k in range(len(sizes))]
    assert [r.tobytes() for r in roots] == want
