"""f16x3 on repeat-rich sequence: real genomes are ~50 % low-complexity
(homopolymer runs, (CA)n / (CAG)n tandem repeats, duplicated blocks, interspersed repeat
families, N gaps), where a filter that matches the repeat fires at every position of a window
-- activations i.i.d. sequence never produces.  Inputs per chromatin.py:138-172 (fetchSeqs +
encodeSeqs geometry), model Beluga.py:18-51.

* Extreme windows (all-A, all-N, pure (CA)n, (CAG)n, (GGGGCC)n, tiled 300-bp blocks, half
  poly-T) through the per-window path, both strands, against a float64 forward at the parity
  bar; the f16x3 fallback count is reported (a fallback recomputes in bf16x6, so the result is
  at the bar either way).
* SNVs placed inside repeats of the repeat-rich synthetic genome (synthetic.genome_bytes(
  repeats=True), the bench's genome) through the 200-window segment-pair path exactly as the
  bench runs them, deferred overflow check at the release point, slice-level recovery
  (VariantPipeline.recompute_overflowed): sampled windows against float64 at the parity bar.
* The slice-level recovery itself: a calibration target past fp16's range makes every slice
  overflow; recompute_overflowed must then return the bf16x6 result bit for bit.
"""
import math
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SHIFTS_200 = list(range(-20000, 20000, 200))     # geuvadis_sed_for_top_eqtls.py:61
_COMP = np.array([3, 2, 1, 0, 4], np.uint8)      # codes A G C T N -> complement


def _ratio(got, want):
    return float(np.max(np.abs(np.asarray(got, np.float64) - want) / (1e-4 * np.abs(want) + 1e-5)))


def _f64(sd, codes):
    from expecto_amd.encode import codes_to_onehot
    from oracle.beluga_np import forward_torch_cpu
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    x = torch.from_numpy(codes_to_onehot(codes, with_rc=False).astype(np.float64)).unsqueeze(2)
    sd64 = {k: v.double() for k, v in sd.items()}
    return np.concatenate([forward_torch_cpu(sd64, x[i:i + 32]).numpy() for i in range(0, x.shape[0], 32)])


def _extreme_windows():
    from expecto_amd.encode import seq_codes
    rng = np.random.default_rng(5)
    blk = "".join(rng.choice(list("ACGT"), 300))
    rnd = "".join(rng.choice(list("ACGT"), 1000))
    seqs = ["A" * 2000, "N" * 2000, "G" * 2000, ("CA" * 1000), ("CAG" * 667)[:2000], ("GGGGCC" * 334)[:2000],
            (blk * 7)[:2000], rnd + "T" * 1000, ("AT" * 500) + "N" * 1000, ("TTAGGG" * 334)[:2000]]
    return np.stack([seq_codes(s) for s in seqs])


@pytest.fixture(scope="module")
def setup():
    from expecto_amd import beluga, synthetic
    from expecto_amd.genome import DeviceGenome, Fasta
    from expecto_amd.pipeline import VariantPipeline, VariantSet
    genome = synthetic.genome_bytes(n_contigs=2, contig_len=200_000, seed=41, repeats=True)
    fa = Fasta.from_dict(genome)
    # SNVs at soft-masked (repeat) positions with an upper-case-able base
    rng = np.random.default_rng(42)
    snv = []
    while len(snv) < 4:
        c = sorted(genome)[int(rng.integers(0, 2))]
        s = genome[c]
        p = int(rng.integers(25_000, len(s) - 25_000))
        b = chr(s[p - 1])
        if b not in "acgt":
            continue
        ref = b.upper()
        snv.append((c, p, ref, "ACGT".replace(ref, "")[int(rng.integers(0, 3))]))
    vs = VariantSet([s[0] for s in snv], np.array([s[1] for s in snv]), [s[2] for s in snv], [s[3] for s in snv])
    m = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=2048)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    eng = m.cuda().engine()
    pipe = VariantPipeline(eng, fa, DeviceGenome(fa))
    return fa, vs, sd, eng, pipe


def test_extreme_low_complexity_windows_vs_float64(setup):
    fa, vs, sd, eng, pipe = setup
    codes = _extreme_windows()
    eng.set_overflow_check(deferred=False)        # per call: a flagged call recomputes itself
    fb0 = eng.f16_state()[0]
    got = eng.forward_codes(torch.from_numpy(codes).cuda(), strand_mode=2).cpu().numpy()
    fb = eng.f16_state()[0] - fb0
    want = _f64(sd, np.concatenate([codes, _COMP[codes[:, ::-1]]]))
    r = _ratio(got, want)
    print(f"extreme windows: {len(codes)} x fwd/rc, f16x3 fallbacks {fb}, fraction of the parity bound {r:.3f}")
    assert r < 0.5, r


def test_repeat_rich_sed_workload_vs_float64(setup):
    from expecto_amd.encode import seq_codes
    fa, vs, sd, eng, pipe = setup
    prep = pipe.prepare(vs, SHIFTS_200, rows="variant")
    eng.set_overflow_check(deferred=True)
    flag = torch.zeros(1, dtype=torch.int32).pin_memory()
    try:
        y = pipe.predict(prep)
        eng.overflow_take(flag)
        torch.cuda.synchronize()
        flagged = int(flag[0])
        redone = pipe.recompute_overflowed(vs, SHIFTS_200, y, rows="variant") if flagged else 0
    finally:
        eng.set_overflow_check(deferred=False)
    y = y.cpu().numpy()                           # [2 strands, 2 alleles, n, 200, 2002]
    rng = np.random.default_rng(9)
    snv_j = [j for j, s in enumerate(SHIFTS_200) if -1000 <= s <= 999]
    other = [j for j in range(len(SHIFTS_200)) if j not in snv_j]
    sel = []
    for v in range(len(vs)):
        sel += [(v, j, a) for j in snv_j[::2] + list(rng.choice(other, 2, replace=False)) for a in (0, 1)]

    def win(v, j, a):
        p, sh = int(vs.pos[v]), SHIFTS_200[j]
        c = seq_codes(fa.sequence({"chr": vs.chrom[v], "start": p + sh - 999, "stop": p + sh + 1000}))
        if a and 0 <= 999 - sh < 2000:
            c[999 - sh] = seq_codes(vs.alt[v], 1)[0]
        return c
    codes = np.stack([win(*s) for s in sel])
    want = _f64(sd, np.concatenate([codes, _COMP[codes[:, ::-1]]]))
    got = np.stack([y[0, a, v, j] for v, j, a in sel] + [y[1, a, v, j] for v, j, a in sel])
    r = _ratio(got, want)
    print(f"repeat-rich 200-window SNVs: flag {flagged}, slices recomputed {redone}, "
          f"{len(sel)} windows x fwd/rc, fraction of the parity bound {r:.3f}")
    assert r < 0.5, r


def test_slice_recovery_equals_bf16x6(setup):
    """Every slice flagged (target past fp16's range): the recovered output is bf16x6's bit for
    bit, and the engine counts one fallback per recomputed slice."""
    fa, vs, sd, eng, pipe = setup
    shifts = [-400, -200, 0, 200, 400]
    prep = pipe.prepare(vs, shifts)
    with eng.precision_override("bf16x6"):
        want = pipe.predict(prep).cpu()
    eng.set_overflow_check(deferred=True)
    try:
        eng.set_f16_target(20)
        y = pipe.predict(prep)
        fb0 = eng.f16_state()[0]
        n = pipe.recompute_overflowed(vs, shifts, y, parts=2)
        assert n == 2 and eng.f16_state()[0] - fb0 == 2
        assert torch.equal(y.cpu(), want)
    finally:
        eng.set_f16_target(10)
        eng.overflow_pending()
        eng.set_overflow_check(deferred=False)
