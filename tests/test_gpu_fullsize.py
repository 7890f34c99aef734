"""configs[2] at its full size (BASELINE.json: 10k SNVs, the +-800 shift sweep, then the
spatial reduction) through size-independent properties, since the oracle cannot run 360k
windows in a test: every output finite and in [0, 1]; a seeded sample of variants recomputed
by the independent per-window path (its own windows, no trunk sharing, no alt cone) is
bitwise equal; diff == alt - ref exactly; the variant reduction of the full batch equals the
oracle's (oracle/reduce_np.py, predict.py:87-124) on the sampled variants."""
import math

import numpy as np
import pytest
import torch

from conftest import sweep_in_roles

pytestmark = pytest.mark.gpu


def test_configs2_full_size_properties():
    from expecto_amd import beluga, synthetic
    from expecto_amd.features import fwd_rc_average, variant_features
    from expecto_amd.genome import DeviceGenome, Fasta
    from expecto_amd.pipeline import VariantPipeline, VariantSet, shift_order
    from oracle.reduce_np import variant_reduce, variant_weights

    genome = synthetic.genome_bytes(n_contigs=4, contig_len=1_000_000, seed=5)
    fa = Fasta.from_dict(genome)
    dg = DeviceGenome(fa)
    snv = synthetic.snvs(genome, 10000, seed=9)
    vs = VariantSet([s[0] for s in snv], np.array([s[1] for s in snv]), [s[2] for s in snv], [s[3] for s in snv])
    shifts = shift_order(800)
    S, n = len(shifts), len(snv)
    eng = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=8192).cuda().engine()
    pipe = VariantPipeline(eng, fa, dg)
    y = pipe.predict(vs, shifts)                       # [2 strands, 2 alleles, S, n, 2002]
    d = pipe.diff(y)
    torch.cuda.synchronize()
    assert y.shape == (2, 2, S, n, 2002)
    assert bool(torch.isfinite(y).all()) and float(y.min()) >= 0.0 and float(y.max()) <= 1.0

    rng = np.random.default_rng(17)
    idx = np.sort(rng.choice(n, 48, replace=False))
    it = torch.from_numpy(idx).cuda()
    sub = VariantSet([vs.chrom[i] for i in idx], vs.pos[idx], [vs.ref[i] for i in idx], [vs.alt[i] for i in idx])
    pw = VariantPipeline(eng, fa, dg, use_segments=False, use_pairs=False)
    yw = sweep_in_roles(eng, lambda: pw.predict(sub, shifts), shifts)   # each window in its FC1 role
    assert torch.equal(yw, y.index_select(3, it))
    assert torch.equal(d.index_select(2, it), y[:, 1].index_select(2, it) - y[:, 0].index_select(2, it))

    # predict.py:186 fwd/rc average of the diffs, then the 9-shift exponential-decay reduction
    dist = rng.integers(-30000, 30000, n)
    plus = rng.random(n) < 0.5
    eff = fwd_rc_average(d.reshape(2, S * n * 2002).reshape(2 * S * n, 2002)).reshape(S, n, 2002)
    feats = variant_features(eff, dist, plus, shifts)
    e_s = eff.index_select(1, it).cpu().numpy()
    ref = variant_reduce(list(e_s), variant_weights(dist[idx], plus[idx], shifts), 2002)
    np.testing.assert_allclose(feats.index_select(0, it).cpu().numpy(), ref, rtol=1e-12, atol=1e-12)
