"""GPU parity: batch Keccak256 / SM3 and the Merkle kernels against the oracle and the golden vectors.

Mirrors HashTest.cpp (KATs), testMerkle.cpp (widths 2..16, counts 0..63, empty throws) and
merkleBench (100k leaves), plus sizes past the level boundaries and 1M leaves.
"""
import hashlib
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _bench_leaves(n):
    return np.frombuffer(b"".join(hashlib.new("sm3", struct.pack("<Q", i)).digest() for i in range(n)),
                         dtype=np.uint8).reshape(n, 32)


def test_hash_kats(gpu, kat):
    for v in kat["hash"]:
        h = gpu.Keccak256() if v["hasher"] == "keccak256" else gpu.SM3()
        assert h.hash(v["msg"].encode()).hex() == v["digest"]


@pytest.mark.parametrize("hasher", [0, 1])
def test_hash_batch_ragged(gpu, oracle, hasher):
    rng = np.random.default_rng(11 + hasher)
    lens = list(range(0, 300)) + list(rng.integers(0, 2000, size=700))
    msgs = [rng.bytes(int(n)) for n in lens]
    data, off = gpu.pack_messages(msgs)
    h = gpu.SM3() if hasher else gpu.Keccak256()
    got = h.hash_packed(data, off)
    want = oracle.hash_packed(hasher, data, off, nthreads=8)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("hasher", [0, 1])
def test_hash_batch_large_unaligned(gpu, oracle, hasher):
    """100k tx-sized messages (150-170 B) packed back to back at arbitrary byte offsets."""
    rng = np.random.default_rng(5)
    lens = rng.integers(150, 171, size=100_000)
    off = np.zeros(len(lens) + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    data = rng.integers(0, 256, size=int(off[-1]), dtype=np.uint8)
    got = (gpu.SM3() if hasher else gpu.Keccak256()).hash_packed(data, off)
    assert np.array_equal(got, oracle.hash_packed(hasher, data, off, nthreads=16))


def test_merkle_golden(gpu, merkle_golden):
    cache = {}
    for c in merkle_golden["cases"]:
        n = c["n"]
        if n not in cache:
            cache[n] = _bench_leaves(n)
        h = gpu.SM3() if c["hasher"] == "sm3" else gpu.Keccak256()
        leaves = [cache[n][i].tobytes() for i in range(n)]
        if c["variant"] == "old":
            assert gpu.calculate_merkle_proof_root(h, cache[n]).hex() == c["root"], c
            continue
        if "tree" in c:
            tree = gpu.Merkle(h, c["width"]).generate_merkle(leaves)
            assert [e.hex() for e in tree] == c["tree"], c
        assert gpu.Merkle(h, c["width"]).root(cache[n]).hex() == c["root"], c


def test_merkle_property_small(gpu, oracle):
    """testMerkle.cpp:62-142 shape: widths 2..16 x counts 1..63, full output vector equal."""
    rng = np.random.default_rng(3)
    for width in range(2, 17):
        for n in range(1, 64):
            leaves = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
            for hasher, H in ((0, gpu.Keccak256()), (1, gpu.SM3())):
                if (width + n + hasher) % 3:
                    continue
                got = gpu.Merkle(H, width).generate_merkle([leaves[i].tobytes() for i in range(n)])
                _, want = oracle.merkle(hasher, width, leaves, want_tree=True)
                assert got == [want[i].tobytes() for i in range(want.shape[0])], (width, n, hasher)


@pytest.mark.parametrize("width", [2, 3, 16, 64])
def test_merkle_full_tree_through_top_kernel(gpu, oracle, width):
    """Trees tall enough for the single-workgroup top kernel (levels kept in LDS between passes, cooperative
    and one-lane passes): every entry of the output vector, both hashers, a generic width included."""
    rng = np.random.default_rng(40 + width)
    n = 70_001
    leaves = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    for hasher, H in ((0, gpu.Keccak256()), (1, gpu.SM3())):
        got = gpu.Merkle(H, width).generate_merkle([leaves[i].tobytes() for i in range(n)])
        _, want = oracle.merkle(hasher, width, leaves, want_tree=True)
        assert len(got) == want.shape[0]
        assert got == [want[i].tobytes() for i in range(want.shape[0])], (width, hasher)


def test_merkle_empty_throws(gpu):
    with pytest.raises(ValueError):
        gpu.Merkle(gpu.SM3(), 2).generate_merkle([])
    assert gpu.calculate_merkle_proof_root(gpu.SM3(), []) == hashlib.new("sm3", b"").digest()


@pytest.mark.parametrize("width", [2, 16])
@pytest.mark.parametrize("hasher", [0, 1])
def test_merkle_1m(gpu, oracle, width, hasher):
    rng = np.random.default_rng(width + hasher)
    leaves = rng.integers(0, 256, size=(1_000_000, 32), dtype=np.uint8)
    H = gpu.SM3() if hasher else gpu.Keccak256()
    assert gpu.Merkle(H, width).root(leaves) == oracle.merkle(hasher, width, leaves, nthreads=16)


@pytest.mark.parametrize("hasher", [0, 1])
def test_merkle_16m_width2_root(gpu, oracle, hasher):
    """The bench's 16M-leaf width-2 tree (subtree kernel over levels 0..6, then the climb kernel): root
    against the oracle."""
    rng = np.random.default_rng(16 + hasher)
    leaves = rng.integers(0, 256, size=(16_000_000, 32), dtype=np.uint8)
    H = gpu.SM3() if hasher else gpu.Keccak256()
    assert gpu.Merkle(H, 2).root(leaves) == oracle.merkle(hasher, 2, leaves, nthreads=16)


def test_device_api_torch(gpu, oracle):
    """The *_dev entry points on HBM-resident torch tensors, launched on torch's stream."""
    import torch
    from bcos_gpu import device
    rng = np.random.default_rng(9)
    msgs = [rng.bytes(int(n)) for n in rng.integers(0, 400, size=4096)]
    data, off = gpu.pack_messages(msgs)
    d_data = torch.from_numpy(data.copy()).cuda()
    d_off = torch.from_numpy(off.astype(np.int64)).cuda()
    d_out = torch.zeros((len(msgs), 32), dtype=torch.uint8, device="cuda")
    device.hash_batch(device.KECCAK256, d_data, d_off, d_out)
    torch.cuda.synchronize()
    assert np.array_equal(d_out.cpu().numpy(), oracle.hash_packed(0, data, off))
    leaves = d_out
    tree = torch.zeros((device.merkle_size(4096, 2), 32), dtype=torch.uint8, device="cuda")
    root = torch.zeros(32, dtype=torch.uint8, device="cuda")
    device.merkle_root(device.KECCAK256, 2, leaves, tree, root)
    torch.cuda.synchronize()
    assert root.cpu().numpy().tobytes() == oracle.merkle(0, 2, d_out.cpu().numpy())


@pytest.mark.parametrize("hasher", [0, 1])
def test_merkle_bytes_layout_vs_oracle(gpu, oracle, hasher):
    """BlockImpl's stored tree (vector<vector<char>>, BlockImpl.h:136) and merkleBench's vector<bytes>
    (merkleBench.cpp:53-56): 4-byte count records, 32-byte nodes -- through the host ABI
    (BCOSGPU_MERKLE_NEW_BYTES) and the device conversion (bcosgpu_merkle_tree_bytes_dev), against the
    restatement of Merkle.h:213-217 + Basic.h:50-61; the 32-byte-entry layout of the same call stays the
    fixed-size HashType one (LedgerTypeDef.h:27)."""
    import torch
    import bcos_gpu
    from bcos_gpu import device
    hs = gpu.Keccak256() if hasher == 0 else gpu.SM3()
    rng = np.random.default_rng(90 + hasher)
    for width in (2, 3, 16):
        for n in (1, 2, 3, 16, 17, 257, 4097, 70000):
            leaves = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
            want = oracle.merkle_bytes_vector(hasher, width, leaves)
            got = gpu.Merkle(hs, width).generate_merkle_bytes([leaves[i].tobytes() for i in range(n)])
            assert got == want, (width, n)
            d_leaves = torch.from_numpy(leaves).cuda()
            tree = torch.empty((max(device.merkle_size(n, width), 1), 32), dtype=torch.uint8, device="cuda")
            root = torch.empty(32, dtype=torch.uint8, device="cuda")
            device.merkle_root(hasher, width, d_leaves, tree, root)
            size = int(bcos_gpu.lib().bcosgpu_merkle_bytes_size(n, width))
            flat = torch.zeros(size + 4, dtype=torch.uint8, device="cuda")
            bcos_gpu.check(bcos_gpu.lib().bcosgpu_merkle_tree_bytes_dev(width, tree.data_ptr(), n, flat.data_ptr(),
                                                                        torch.cuda.current_stream().cuda_stream))
            torch.cuda.synchronize()
            assert flat[:size].cpu().numpy().tobytes() == b"".join(want), (width, n)
            assert int(flat[size:].sum()) == 0  # nothing written past the packed size


def test_merkle_one_launch_path_trees(gpu, oracle):
    """The one-launch Keccak path (merkle_fused_kernel: waves publish their subtree roots and the wave that
    completes a group hashes the parent) over widths 2..64 and sizes around its wave boundaries
    (S = width^a level-1 nodes per wave): every entry of the output vector.  (Widths 2..4 take the
    four-wave kernel by default, test_merkle_four_wave_climb_trees.)"""
    rng = np.random.default_rng(77)
    H = gpu.Keccak256()
    for width in (2, 3, 4, 5, 7, 16, 17, 31, 32, 33, 64):
        S = 1
        while S * width <= 32:
            S *= width
        for n in sorted({1, 2, width, width + 1, S * width, S * width + 1, 3 * S * width - 1, 40 * S * width + 5}):
            leaves = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
            got = gpu.Merkle(H, width).generate_merkle([leaves[i].tobytes() for i in range(n)])
            _, want = oracle.merkle(0, width, leaves, want_tree=True)
            assert got == [want[i].tobytes() for i in range(want.shape[0])], (width, n)


def test_merkle_four_wave_climb_trees(gpu, oracle):
    """The four-wave one-launch Keccak path for narrow trees (hash_kernels.hip merkle_climb_kernel: B =
    width^kin <= 256 level-1 nodes per workgroup, then climb steps of g levels) over widths 2..4 and sizes
    around its workgroup and climb-group boundaries, up to more workgroups than CUs (the throughput
    schedule): every entry of the output vector."""
    rng = np.random.default_rng(78)
    H = gpu.Keccak256()
    for width in (2, 3, 4):
        B = 1
        while B * width <= 256:
            B *= width
        G = 1
        while G <= 8:
            G *= width  # width^g children per climb step
        for n in sorted({1, 2, 3, width, width + 1, B * width, B * width + 1, G * B * width, G * B * width + 1,
                         3 * G * B * width - 1, 300 * B * width + 7}):
            leaves = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
            got = gpu.Merkle(H, width).generate_merkle([leaves[i].tobytes() for i in range(n)])
            _, want = oracle.merkle(0, width, leaves, want_tree=True)
            assert got == [want[i].tobytes() for i in range(want.shape[0])], (width, n)


@pytest.mark.parametrize("hasher", [0, 1])
def test_merkle_subtree_then_climb(gpu, oracle, hasher):
    """Throughput-sized trees (more level-1 nodes than 256 per CU, up to width 16): the subtree kernel hashes
    levels 0..k one thread per level-k node, then the climb kernel runs on level k (k = 0, 1, 2 at these
    sizes for width 2 on 256 CUs); every entry of the output vector, both hashers."""
    rng = np.random.default_rng(79 + hasher)
    H = gpu.Keccak256() if hasher == 0 else gpu.SM3()
    # (widths 7 and 8: the climb step is capped so its width^g gathered children fit one LDS half)
    for width, n in ((2, 153_607), (2, 400_005), (2, 1_000_003), (4, 1_000_001), (3, 600_001), (5, 400_001),
                     (7, 1_500_001), (8, 1_200_007), (16, 2_000_003)):
        leaves = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
        got = gpu.Merkle(H, width).generate_merkle([leaves[i].tobytes() for i in range(n)])
        _, want = oracle.merkle(hasher, width, leaves, want_tree=True)
        assert len(got) == want.shape[0], (width, n)
        assert b"".join(got) == want.tobytes(), (width, n)


def test_merkle_sm3_expanded_levels(gpu, oracle):
    """SM3 levels whose blocks are all expanded at once (hash_kernels.hip sm3_level_x: the workgroup
    kernel's LDS levels, up to 256 blocks, and the top kernel's, up to 448) and the one-lane levels past
    those limits, widths with 2..17 blocks per node, sizes around the limits; every entry of the output
    vector."""
    rng = np.random.default_rng(81)
    H = gpu.SM3()
    for width in (3, 5, 16, 33):
        nb = (32 * width + 8) // 64 + 1
        cap = 448 // nb  # top-kernel nodes per level expanded at once
        for n in sorted({width * width + 1, cap * width, cap * width + 1, (cap + 1) * width * width - 1, 70_001}):
            leaves = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
            got = gpu.Merkle(H, width).generate_merkle([leaves[i].tobytes() for i in range(n)])
            _, want = oracle.merkle(1, width, leaves, want_tree=True)
            assert b"".join(got) == want.tobytes(), (width, n)


def test_merkle_one_launch_repeat_two_streams(gpu, oracle):
    """The one-launch path's arrival counters reset themselves (back-to-back launches on one stream) and
    are per stream (two torch streams at once): 40 C1-sized roots per stream, each equal to the oracle.
    Every tensor a side stream writes is held until the final synchronize and is ready (default-stream
    fill) before that stream starts: a tree freed while its stream still runs goes back to torch's caching
    allocator, which may hand its memory to the next allocation (the other stream's roots) while the first
    stream's kernels still write it.  tools/merkle_stream_diag.py runs this with the two streams measured
    overlapping (profiles/r06_merkle_two_stream_overlap.json)."""
    import torch
    from bcos_gpu import device
    rng = np.random.default_rng(78)
    cases = []
    for width in (16, 2):
        leaves = rng.integers(0, 256, size=(100_000, 32), dtype=np.uint8)
        cases.append((width, torch.from_numpy(leaves).cuda(), oracle.merkle(0, width, leaves, nthreads=16)))
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = []
    for k, st in enumerate(streams):
        width, d_leaves, _ = cases[k]
        tree = torch.empty((device.merkle_size(100_000, width), 32), dtype=torch.uint8, device="cuda")
        roots = torch.zeros((40, 32), dtype=torch.uint8, device="cuda")
        outs.append((roots, tree))  # both held until the synchronize below
        st.wait_stream(torch.cuda.current_stream())  # after the zero fill
        with torch.cuda.stream(st):
            for r in range(40):
                device.merkle_root(device.KECCAK256, width, d_leaves, tree, roots[r], st)
    torch.cuda.synchronize()
    for (width, _, want), (roots, _) in zip(cases, outs):
        got = roots.cpu().numpy()
        assert all(got[r].tobytes() == want for r in range(40)), width


def test_merkle_one_launch_per_thread_streams(gpu, oracle):
    """hipStreamPerThread is ONE handle naming a different stream on each thread: the one-launch path keys
    its arrival-counter slot by (device, handle, thread) for it (and for the null stream), so two host
    threads launching through that handle at once never share counters.  Two threads x 30 C1 roots each,
    every root equal to the oracle's."""
    import threading
    import torch
    from bcos_gpu import _lib, device
    rng = np.random.default_rng(79)
    per_thread = 2  # hipStreamPerThread
    cases, results, errs = [], {}, []
    for width in (16, 2):
        leaves = rng.integers(0, 256, size=(100_000, 32), dtype=np.uint8)
        tree = torch.empty((device.merkle_size(100_000, width), 32), dtype=torch.uint8, device="cuda")
        roots = torch.zeros((30, 32), dtype=torch.uint8, device="cuda")
        cases.append((width, torch.from_numpy(leaves).cuda(), tree, roots, oracle.merkle(0, width, leaves, nthreads=16)))
    torch.cuda.synchronize()
    lib = _lib.lib()

    def run(k):
        try:
            width, d_leaves, tree, roots, _ = cases[k]
            for r in range(30):
                rc = lib.bcosgpu_merkle_root_dev(0, width, d_leaves.data_ptr(), 100_000, tree.data_ptr(),
                                                 roots[r].data_ptr(), per_thread)
                assert rc == 0, _lib.lib().bcosgpu_last_error()
            torch.cuda.synchronize()  # before the thread (and its per-thread stream) ends
        except Exception as e:  # noqa: BLE001
            errs.append(e)
    ts = [threading.Thread(target=run, args=(k,)) for k in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    torch.cuda.synchronize()
    assert not errs, errs
    for width, _, _, roots, want in cases:
        got = roots.cpu().numpy()
        assert all(got[r].tobytes() == want for r in range(30)), width


SM3_CLIMBX_CHILD = r"""
import sys, numpy as np
sys.path[:0] = [sys.argv[1]]
import bcos_gpu
bcos_gpu.ensure_device(0)
rng = np.random.default_rng(int(sys.argv[2]))
H = bcos_gpu.SM3()
for spec in sys.argv[3:]:
    n, w = (int(x) for x in spec.split("x"))
    leaves = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    got = bcos_gpu.Merkle(H, w).generate_merkle([leaves[i].tobytes() for i in range(n)])
    sys.stdout.write(spec + " " + __import__("hashlib").sha256(b"".join(got)).hexdigest() + "\n")
"""


def test_merkle_sm3_climb_expanded_opt_in(gpu, oracle):
    """The opt-in one-launch SM3 path (BCOSGPU_MERKLE_SM3CLIMB=1, read once per process: a child process):
    merkle_climb_kernel<SM3, W, true> with the in-workgroup and climb-step levels' blocks expanded at once,
    widths 3 .. 33 and sizes around the workgroup / climb-group boundaries, C1 included; every entry of the
    output vector (compared through its SHA-256) equals the oracle's."""
    import hashlib
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    specs = ["%dx%d" % (n, w) for w, ns in ((3, (10, 244, 6562, 59050)), (5, (626, 3126, 70001)),
                                             (16, (257, 4097, 65537, 100000)), (17, (290, 4914)), (33, (1090, 40000)))
             for n in ns]
    env = dict(os.environ, BCOSGPU_MERKLE_SM3CLIMB="1")
    r = subprocess.run([sys.executable, "-c", SM3_CLIMBX_CHILD, os.path.join(root, "fisco-bcos_amd"), "83"] + specs,
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    got = dict(line.split() for line in r.stdout.splitlines())
    rng = np.random.default_rng(83)
    for spec in specs:
        n, w = (int(x) for x in spec.split("x"))
        leaves = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
        _, want = oracle.merkle(1, w, leaves, want_tree=True)
        assert got[spec] == hashlib.sha256(want.tobytes()).hexdigest(), spec
