"""GPU reductions (reduce.hip) against the oracle (oracle/reduce_np.py, which follows
compute_expecto_features.py:88-124 and predict.py:87-124) BIT FOR BIT: the kernels round every
product before the sum (no FMA contraction) and sum the shifts sequentially in order, as
numpy's reductions over a non-contiguous axis and predict.py's functools.reduce do.  The
2-feature-per-thread kernels are bitwise equal to the scalar ones (a misaligned ``out`` view
forces the scalar kernel)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _misaligned(shape):
    buf = torch.empty(int(np.prod(shape)) + 1, dtype=torch.float64, device="cuda")
    return buf[1:].view(*shape)          # 8-byte but not 16-byte aligned


@pytest.mark.parametrize("nfeat,S", [(2002, 200), (37, 200), (2002, 13)])
def test_tss_reduce_matches_oracle_and_scalar_kernel(nfeat, S):
    """S = 13: a shift count that is not a multiple of the kernels' 8-shift load chunk."""
    from expecto_amd.features import tss_pos_weights, tss_reduce
    from oracle.reduce_np import tss_reduce as tss_ref
    rng = np.random.default_rng(3)
    G = 5
    f = rng.random((G, S, nfeat), dtype=np.float32)
    r = rng.random((G, S, nfeat), dtype=np.float32)
    wn = np.ascontiguousarray(tss_pos_weights()[:, :S])
    w = torch.from_numpy(wn).cuda()
    fd, rd = torch.from_numpy(f).cuda(), torch.from_numpy(r).cuda()
    out = tss_reduce(fd, rd, w).cpu().numpy()
    out_s = tss_reduce(fd, rd, w, out=_misaligned((G, 10 * nfeat))).cpu().numpy()
    np.testing.assert_array_equal(out, out_s)
    for g in range(G):
        np.testing.assert_array_equal(out[g], tss_ref(f[g], r[g], wn))


@pytest.mark.parametrize("nfeat", [2002, 37, 8, 1000])
def test_variant_features_match_oracle_and_scalar_kernel(nfeat):
    """2002 / 8 / 1000: the row-staged kernel (one or two 256-pair workgroups per variant, ragged
    last workgroup, pieces shorter than a line); 37: the scalar kernel."""
    from expecto_amd.features import variant_features
    from oracle.reduce_np import variant_reduce, variant_weights
    rng = np.random.default_rng(4)
    shifts = [0, -200, 200, -400, 400, -800, 800, -1600, 1600]
    n = 300
    eff = rng.standard_normal((len(shifts), n, nfeat)).astype(np.float32)
    dist = rng.integers(-60000, 60000, n)
    dist[:3] = [0, 200, -199]
    strand = rng.random(n) < 0.5
    ed = torch.from_numpy(eff).cuda()
    out = variant_features(ed, dist, strand, shifts).cpu().numpy()
    out_s = variant_features(ed, dist, strand, shifts, out=_misaligned((n, 10 * nfeat))).cpu().numpy()
    np.testing.assert_array_equal(out, out_s)
    ref = variant_reduce(list(eff), variant_weights(dist, strand, shifts), nfeat)
    np.testing.assert_array_equal(out, ref)


def test_variant_features_beyond_32_shifts():
    """predict --maxshift above 3000 (33+ shifts): the weight table is sized per launch."""
    from expecto_amd.features import variant_features
    from expecto_amd.pipeline import shift_order
    from oracle.reduce_np import variant_reduce, variant_weights
    rng = np.random.default_rng(5)
    shifts = shift_order(5000)                      # 51 shifts
    n, nfeat = 40, 2002
    eff = rng.standard_normal((len(shifts), n, nfeat)).astype(np.float32)
    dist = rng.integers(-30000, 30000, n)
    strand = rng.random(n) < 0.5
    out = variant_features(torch.from_numpy(eff).cuda(), dist, strand, shifts).cpu().numpy()
    np.testing.assert_array_equal(out, variant_reduce(list(eff), variant_weights(dist, strand, shifts), nfeat))


def test_variant_features_past_the_row_kernels_lds():
    """720 shifts: the weight table and the row slots exceed 64 KB of LDS, so the 2-feature
    kernel without row staging runs; the same bits as the oracle."""
    from expecto_amd.features import variant_features
    from oracle.reduce_np import variant_reduce, variant_weights
    rng = np.random.default_rng(7)
    shifts = [200 * (i // 2) * (1 if i % 2 else -1) for i in range(720)]
    n, nfeat = 3, 2002
    eff = rng.standard_normal((len(shifts), n, nfeat)).astype(np.float32)
    dist = rng.integers(-30000, 30000, n)
    strand = rng.random(n) < 0.5
    out = variant_features(torch.from_numpy(eff).cuda(), dist, strand, shifts).cpu().numpy()
    np.testing.assert_array_equal(out, variant_reduce(list(eff), variant_weights(dist, strand, shifts), nfeat))


@pytest.mark.parametrize("S", [200, 13])
def test_shift_reduce_matches_numpy_bitwise(S):
    """geuvadis_sed_for_top_eqtls.py:83-121: float64 fwd/rc mean, then
    np.sum(pos_weights[None,:,:,None] * preds[:,None], axis=2) with the legacy zero column
    (S = 13: the first 13 shifts' weights, a ragged last load chunk)."""
    from expecto_amd import _lib
    from expecto_amd.features import tss_pos_weights
    rng = np.random.default_rng(6)
    n, F = 3, 2002
    fwd = rng.random((n, S, F), dtype=np.float32)
    rc = rng.random((n, S, F), dtype=np.float32)
    w = np.ascontiguousarray(tss_pos_weights()[:, :S])
    out = torch.empty((n, 20030), dtype=torch.float64, device="cuda")
    lib = _lib.load()
    fd, rd, wd = torch.from_numpy(fwd).cuda(), torch.from_numpy(rc).cuda(), torch.from_numpy(w).cuda()
    _lib.check(lib.expecto_shift_reduce(_lib.dptr(fd), _lib.dptr(rd), _lib.dptr(wd), n, S, F, 3, _lib.dptr(out),
                                        _lib.stream_ptr()), "shift_reduce")
    preds = (fwd.astype(np.float64) + rc.astype(np.float64)) / 2
    want = np.sum(w[None, :, :, None] * preds[:, None, :, :], axis=2).reshape(-1, 10 * F)
    want = np.concatenate([np.zeros((n, 10, 1)), want.reshape(n, 10, F)], axis=2).reshape(n, 20030)
    np.testing.assert_array_equal(out.cpu().numpy(), want)
