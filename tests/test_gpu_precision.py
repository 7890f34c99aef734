"""The headline arithmetic (f16x3) on the metric's own workload, and its range safety.

* 200-window variants through the segment-pair path (forward_segment_pairs, rows by variant as
  the bench runs them): every window holding the SNV and two others per variant, both strands,
  both alleles, against a float64 forward of the same windows (oracle/beluga_np.py in float64):
  f16x3's error on ref, alt and alt - ref is within the exact fp32 MFMA kernel's (x 1.25 for
  sampling noise) and well inside the parity bar 1e-4|y| + 1e-5 (Beluga.py:18-51 in fp32).
* Weight and activation ranges stretched by 2^+-10 per layer (each layer's output scaled by
  2^a_l and the next layer's weights by 2^-a_l: the same function): the calibrated f16x3 scales
  absorb it exactly, so the outputs are bit for bit those of the unstretched model.
* Headroom: a calibration target of 2^0 instead of 2^10 (small activations pushed 2^10 deeper
  towards fp16's subnormals) stays inside the parity bar; a target past fp16's range makes the
  overflow fallback fire, per call or deferred to the caller's release point, and the result
  is the bf16x6 one bit for bit.
* The production forward does not block the host: with the deferred check a 200-window call
  returns while its kernels still run.
"""
import math
import os

import numpy as np
import pytest
import torch

from conftest import assert_close

pytestmark = pytest.mark.gpu

SHIFTS_200 = list(range(-20000, 20000, 200))     # geuvadis_sed_for_top_eqtls.py:61


def _ratio(got, want):
    return float(np.max(np.abs(np.asarray(got, np.float64) - want) / (1e-4 * np.abs(want) + 1e-5)))


@pytest.fixture(scope="module")
def sed_setup():
    from expecto_amd import beluga, synthetic
    from expecto_amd.genome import DeviceGenome, Fasta
    from expecto_amd.pipeline import VariantPipeline, VariantSet
    genome = synthetic.genome_bytes(n_contigs=2, contig_len=200_000, seed=31)
    fa = Fasta.from_dict(genome)
    snv = synthetic.snvs(genome, 4, seed=32, margin=25_000)
    vs = VariantSet([s[0] for s in snv], np.array([s[1] for s in snv]), [s[2] for s in snv], [s[3] for s in snv])
    m = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=2048)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    eng = m.cuda().engine()
    pipe = VariantPipeline(eng, fa, DeviceGenome(fa))
    return fa, vs, sd, eng, pipe


def test_metric_workload_f16x3_accuracy_vs_float64(sed_setup):
    from expecto_amd.encode import codes_to_onehot, seq_codes
    from oracle.beluga_np import forward_torch_cpu
    fa, vs, sd, eng, pipe = sed_setup
    prep = pipe.prepare(vs, SHIFTS_200, rows="variant")
    ys = {}
    for prec in ("f16x3", "fp32", "bf16x6"):
        with eng.precision_override(prec):
            ys[prec] = pipe.predict(prep).cpu().numpy()          # [2 strands, 2 alleles, n, 200, 2002]
    rng = np.random.default_rng(7)
    snv_j = [j for j, s in enumerate(SHIFTS_200) if -1000 <= s <= 999]          # windows holding the SNV
    other = [j for j in range(len(SHIFTS_200)) if j not in snv_j]
    ref_sel, alt_sel = [], []                                   # (variant, shift index)
    for v in range(len(vs)):
        picks = snv_j + list(rng.choice(other, 2, replace=False))
        ref_sel += [(v, j) for j in picks]
        alt_sel += [(v, j) for j in snv_j]
    def win(v, j, allele):
        """The window at shift j with `allele` at the SNV when the window holds it (chromatin.py's
        fetchSeqs geometry: the SNV at crop index 999 - shift)."""
        p, sh = int(vs.pos[v]), SHIFTS_200[j]
        c = seq_codes(fa.sequence({"chr": vs.chrom[v], "start": p + sh - 999, "stop": p + sh + 1000}))
        if 0 <= 999 - sh < 2000:
            c[999 - sh] = seq_codes(allele, 1)[0]
        return c
    codes = np.stack([win(v, j, vs.ref[v]) for v, j in ref_sel] + [win(v, j, vs.alt[v]) for v, j in alt_sel])
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    x = torch.from_numpy(codes_to_onehot(codes, with_rc=True).astype(np.float64)).unsqueeze(2)
    sd64 = {k: v.double() for k, v in sd.items()}
    y64 = np.concatenate([forward_torch_cpu(sd64, x[i:i + 32]).numpy() for i in range(0, x.shape[0], 32)])
    nr, na, nw = len(ref_sel), len(alt_sel), len(codes)
    want = {"ref": np.concatenate([y64[:nr], y64[nw:nw + nr]]),
            "alt": np.concatenate([y64[nr:nw], y64[nw + nr:]])}
    # alt - ref on the SNV windows (the rows of ref_sel that are SNV windows, in alt_sel order)
    ref_pos = {vj: i for i, vj in enumerate(ref_sel)}
    ri = [ref_pos[vj] for vj in alt_sel]
    want["diff"] = want["alt"] - np.concatenate([want["ref"][:nr][ri], want["ref"][nr:][ri]])
    res = {}
    for prec, y in ys.items():
        got = {"ref": np.stack([y[s, 0, v, j] for s in (0, 1) for v, j in ref_sel]),
               "alt": np.stack([y[s, 1, v, j] for s in (0, 1) for v, j in alt_sel])}
        got["diff"] = got["alt"].astype(np.float64) - np.stack([y[s, 0, v, j] for s in (0, 1) for v, j in alt_sel])
        res[prec] = {k: _ratio(got[k], want[k]) for k in got}
    print("fraction of the parity bound used (max over elements):", res)
    for k in ("ref", "alt", "diff"):
        for prec in res:
            assert res[prec][k] < 0.5, (prec, k, res)
        assert res["f16x3"][k] <= 1.25 * res["fp32"][k], (k, res)


def _stretched(sd, a):
    """Layer l's weight x 2^(a_l - a_{l-1}) and bias x 2^a_l for conv1..fc1; fc2's weight x
    2^-a_fc1 (its bias and the sigmoid unchanged): the same function, activations x 2^a_l."""
    keys = ["model.0.0", "model.0.2", "model.0.6", "model.0.8", "model.0.12", "model.0.14", "model.1.2.1"]
    out = {k: v.clone() for k, v in sd.items()}
    prev = 0
    for key, e in zip(keys, a):
        out[key + ".weight"].mul_(2.0 ** (e - prev))
        out[key + ".bias"].mul_(2.0 ** e)
        prev = e
    out["model.1.4.1.weight"].mul_(2.0 ** -prev)
    return out


def test_f16x3_ranges_stretched_2pow10_are_absorbed_bitwise():
    from expecto_amd import beluga
    m0 = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=128)
    a = [10, -10, 10, -10, 10, -10, 10]
    sd1 = _stretched(m0.state_dict(), a)
    m1 = beluga.Beluga(max_batch=128)
    m1.load_state_dict(sd1)
    m0, m1 = m0.cuda(), m1.eval().cuda()
    rng = np.random.default_rng(12)
    codes = torch.from_numpy(rng.integers(0, 5, (48, 2000)).astype(np.uint8)).cuda()
    y0 = m0.forward_codes(codes, 2)
    y1 = m1.forward_codes(codes, 2)
    n0, sx0 = m0.engine().f16_state()
    n1, sx1 = m1.engine().f16_state()
    assert n0 == 0 and n1 == 0
    assert sx1 == [s - e for s, e in zip(sx0, a)], (sx0, sx1)
    assert torch.equal(y0, y1)


def test_f16x3_headroom_underflow_side_and_overflow_fallback():
    from expecto_amd import beluga
    from expecto_amd.encode import codes_to_onehot
    from oracle.beluga_np import forward_torch_cpu
    m = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=128)
    sd64 = {k: v.detach().double() for k, v in m.state_dict().items()}
    m = m.cuda()
    mb = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=128).cuda()
    mb.engine().set_precision("bf16x6")
    eng = m.engine()
    rng = np.random.default_rng(13)
    codes_np = rng.integers(0, 5, (12, 2000)).astype(np.uint8)
    codes = torch.from_numpy(codes_np).cuda()
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    y64 = forward_torch_cpu(sd64, torch.from_numpy(codes_to_onehot(codes_np).astype(np.float64)).unsqueeze(2)).numpy()
    # small side: every activation 2^10 closer to fp16's subnormal range
    eng.set_f16_target(0)
    y = m.forward_codes(codes, 2).cpu().numpy()
    assert eng.f16_state()[0] == 0
    assert_close(y, y64, what="f16x3 at calibration target 2^0")
    # large side: past fp16's range -> bf16x6 recompute inside the call
    eng.set_f16_target(20)
    n0 = eng.f16_state()[0]
    y = m.forward_codes(codes, 2)
    assert eng.f16_state()[0] == n0 + 1
    yb = mb.forward_codes(codes, 2)
    assert torch.equal(y, yb)
    # deferred: the call only enqueues; the release point reports it and the caller recomputes
    eng.set_overflow_check(True)
    m.forward_codes(codes, 2)
    assert eng.overflow_pending()
    assert not eng.overflow_pending()
    with eng.precision_override("bf16x6"):
        y = m.forward_codes(codes, 2)
    assert not eng.overflow_pending()
    assert torch.equal(y, yb)
    eng.set_overflow_check(False)
    eng.set_f16_target(10)
    assert_close(m.forward_codes(codes, 2).cpu().numpy(), y64, what="f16x3 re-calibrated")


def test_deferred_forward_returns_before_its_kernels_finish(sed_setup):
    """No host sync inside a production forward: the segment-pair call of 4 x 200-window
    variants (a few ms of GPU work) returns while the GPU is still busy with it."""
    fa, vs, sd, eng, pipe = sed_setup
    prep = pipe.prepare(vs, SHIFTS_200, rows="variant")
    eng.set_overflow_check(True)
    try:
        y = pipe.predict(prep)
        torch.cuda.synchronize()
        busy = 0
        for _ in range(3):
            pipe.predict(prep, out=y)
            pipe.predict(prep, out=y)
            e = torch.cuda.Event()
            e.record()
            busy += int(not e.query())          # still running when the calls returned
            torch.cuda.synchronize()
        assert busy >= 2, busy
        assert not eng.overflow_pending()
    finally:
        eng.set_overflow_check(False)
