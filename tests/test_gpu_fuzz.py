"""Randomised parity sweep of Transaction::verify through the automatic kernel choice: batch sizes at
and around every rounds boundary of the small-batch kernels (40 / 64 / 256 / 512 txs per CU on 256
CUs: trio, pair, one-lane at occupancy 1 and 2) plus seeded random sizes, both suites, each batch with
corrupted signatures and bad recovery ids, every tx hash, verdict and sender compared with the oracle
(TxValidator.cpp:56 -> Transaction.h:68-82).  GPU only."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

BOUNDARY_SIZES = [1, 2, 3, 39, 40, 41, 63, 64, 65, 10_239, 10_240, 10_241, 16_384, 16_385, 20_480, 20_481,
                  40_961, 65_537]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("suite", [0, 1])
def test_auto_path_boundary_and_random_sizes(gpu, oracle, suite):
    import torch
    from bcos_gpu import device, synth
    rng = np.random.default_rng(2024 + suite)
    sizes = BOUNDARY_SIZES + [int(x) for x in rng.integers(1, 30_000, size=6)]
    for k, n in enumerate(sizes):
        b = synth.make_batch(suite, n, seed=1000 * suite + k, flip_frac=0.05, bad_v_frac=0.02)
        th = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
        snd = torch.empty((n, 20), dtype=torch.uint8, device="cuda")
        st = torch.full((n,), 9, dtype=torch.uint8, device="cuda")
        device.tx_verify(suite, b.pre, b.pre_off, b.sig, b.sig_off, th, snd, st)
        torch.cuda.synchronize()
        pre, po, sg, so = (x.cpu().numpy() for x in (b.pre, b.pre_off, b.sig, b.sig_off))
        wh, ws, wst = oracle.tx_verify_packed(suite, pre, po.astype(np.uint64), sg, so.astype(np.uint64),
                                              nthreads=16)
        assert np.array_equal(th.cpu().numpy(), wh), (suite, n)
        assert np.array_equal(st.cpu().numpy(), wst), (suite, n)
        assert np.array_equal(snd.cpu().numpy(), ws), (suite, n)
        assert 0 < int((st == 0).sum()) <= n or n < 4, (suite, n)
