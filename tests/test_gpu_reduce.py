"""GPU reductions (reduce.hip) against the oracle (oracle/reduce_np.py, which follows
compute_expecto_features.py:88-124 and predict.py:87-124), and the 2-feature-per-thread
kernels bitwise equal to the scalar ones (a misaligned ``out`` view forces the scalar kernel)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _misaligned(shape):
    buf = torch.empty(int(np.prod(shape)) + 1, dtype=torch.float64, device="cuda")
    return buf[1:].view(*shape)          # 8-byte but not 16-byte aligned


@pytest.mark.parametrize("nfeat", [2002, 37])
def test_tss_reduce_matches_oracle_and_scalar_kernel(nfeat):
    from expecto_amd.features import tss_pos_weights, tss_reduce
    from oracle.reduce_np import tss_reduce as tss_ref
    rng = np.random.default_rng(3)
    G, S = 5, 200
    f = rng.random((G, S, nfeat), dtype=np.float32)
    r = rng.random((G, S, nfeat), dtype=np.float32)
    w = torch.from_numpy(tss_pos_weights()).cuda()
    fd, rd = torch.from_numpy(f).cuda(), torch.from_numpy(r).cuda()
    out = tss_reduce(fd, rd, w).cpu().numpy()
    out_s = tss_reduce(fd, rd, w, out=_misaligned((G, 10 * nfeat))).cpu().numpy()
    np.testing.assert_array_equal(out, out_s)
    for g in range(G):
        # per-output sums run in a different order than numpy's pairwise sum
        np.testing.assert_allclose(out[g], tss_ref(f[g], r[g]), rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("nfeat", [2002, 37])
def test_variant_features_match_oracle_and_scalar_kernel(nfeat):
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
    np.testing.assert_allclose(out, ref, rtol=1e-12, atol=1e-12)
