"""BASELINE.json configs run as written, checked against the reference and the oracle.

* configs[0]: the reference's own ``example/example.vcf`` through the HIP ``chromatin`` CLI at
  the default ``--maxshift 800`` over a seeded 12 Mb chr1, against the reference chromatin.py
  run on the same inputs (tests/golden/make_golden_example.py).
* configs[1]: the bench workload itself (1k SNVs, shift 0: device window generation + the
  pair path + diff) with 32 sampled windows recomputed by the torch-CPU oracle.
* configs[3]: one rank's shard (12,500 SNVs x 9 shifts): sampled windows vs the oracle, exact
  diff, and the two halves of a 2-rank split equal to the whole bit for bit.
* configs[4]: one rank's shard of the TSS tiling (2,560 genes x 200 windows x fwd/rc through
  the segment path + the exp-decay reduction) with sampled genes against the oracle forward
  and reduction (compute_expecto_features.py:88-128).
"""
import math
import os
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN, assert_close

pytestmark = pytest.mark.gpu
sys.path.insert(0, GOLDEN)


def _oracle_forward(sd, codes: np.ndarray) -> np.ndarray:
    """torch-CPU fp32 oracle (oneDNN, the reference's arithmetic) of windows given as codes,
    fwd rows then rc rows (encodeSeqs order)."""
    from expecto_amd.encode import codes_to_onehot
    from oracle.beluga_np import forward_torch_cpu
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    x = torch.from_numpy(codes_to_onehot(codes, with_rc=True).astype(np.float32)).unsqueeze(2)
    return np.concatenate([forward_torch_cpu(sd, x[i:i + 64]).numpy() for i in range(0, x.shape[0], 64)])


def test_configs0_example_vcf_maxshift_800(tmp_path, capsys):
    import make_golden_example as mg
    from expecto_amd import chromatin, h5, synthetic
    synthetic.write_fasta(str(tmp_path / "hg19.fa"), mg.genome())
    gold = np.load(os.path.join(GOLDEN, "example_chromatin.npz"))
    out = tmp_path / "out"
    chromatin.main([os.path.join(GOLDEN, "example.vcf"), "--output_dir", str(out), "--genome",
                    str(tmp_path / "hg19.fa"), "--synthetic-weights", "0"])
    printed = [l for l in capsys.readouterr().out.splitlines() if l.startswith("Number of")]
    assert printed == list(gold["stdout"])
    assert open(out / "snps_hg19.vcf").read() == str(gold["snps_hg19"])
    for s in mg.SHIFTS:
        got = h5.read(str(out / f"snps.shift_{s}.diff.h5"))
        for k in ("diff", "ref", "alt"):
            assert got[k].shape == tuple(gold[f"{k}_shape_{s}"]) and got[k].dtype == np.float32
            assert_close(got[k][:, ::4], gold[f"{k}_{s}"], what=f"example.vcf shift {s} {k}")
            np.testing.assert_allclose(got[k].astype(np.float64).sum(1), gold[f"{k}_sum_{s}"], rtol=1e-6,
                                       atol=2e-4, err_msg=f"shift {s} {k} row sums")


def test_configs1_bench_workload_sampled_against_oracle():
    from expecto_amd import beluga, synthetic
    from expecto_amd.encode import seq_codes
    from expecto_amd.genome import DeviceGenome, Fasta
    from expecto_amd.pipeline import VariantPipeline, VariantSet, fetch_window
    genome = synthetic.genome_bytes(n_contigs=4, contig_len=2_000_000, seed=0)
    fa = Fasta.from_dict(genome)
    snv = synthetic.snvs(genome, 1000, seed=1)
    vs = VariantSet([s[0] for s in snv], np.array([s[1] for s in snv]), [s[2] for s in snv], [s[3] for s in snv])
    m = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=8192)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    eng = m.cuda().engine()
    pipe = VariantPipeline(eng, fa, DeviceGenome(fa))
    prep = pipe.prepare(vs, [0])
    y = pipe.predict(prep)                                  # [2 strands, 2 alleles, 1, 1000, 2002]
    d = pipe.diff(y)
    assert torch.equal(d, y[:, 1] - y[:, 0])
    rng = np.random.default_rng(3)
    pick = rng.choice(1000, 16, replace=False)
    codes = np.stack([seq_codes(fetch_window(fa, vs.chrom[v], int(vs.pos[v]), vs.ref[v], al, 0))
                      for v in pick for al in (vs.ref[v], vs.alt[v])])          # 32 windows
    want = _oracle_forward(sd, codes)                       # [fwd 32 ; rc 32]
    yc = y.cpu().numpy()
    got = np.stack([yc[st, a, 0, v] for st in (0, 1) for v in pick for a in (0, 1)])
    assert_close(got, want, what="configs[1] sampled windows vs oracle")


def test_configs4_tss_shard_sampled_against_oracle():
    from expecto_amd import beluga, synthetic
    from expecto_amd.encode import seq_codes
    from expecto_amd.features import tss_pos_weights
    from expecto_amd.genome import DeviceGenome, Fasta
    from expecto_amd.tss import TSSPipeline
    from oracle.reduce_np import tss_reduce
    genome = synthetic.genome_bytes(n_contigs=4, contig_len=2_000_000, seed=21)
    fa = Fasta.from_dict(genome)
    rng = np.random.default_rng(8)
    G = 2560
    names = sorted(genome)
    chroms = [names[i] for i in rng.integers(0, len(names), G)]
    tss = [int(rng.integers(30000, 2_000_000 - 30000)) for _ in range(G)]
    strands = rng.choice([-1, 1], G)
    m = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=8192)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    pipe = TSSPipeline(m.cuda().engine(), DeviceGenome(fa))
    feats = torch.cat([pipe.features(chroms[i:i + 128], tss[i:i + 128], strands[i:i + 128]) for i in range(0, G, 128)])
    assert feats.shape == (G, 20020) and bool(torch.isfinite(feats).all())
    w = tss_pos_weights()
    for g in rng.choice(G, 2, replace=False):
        y = pipe.predict([chroms[g]], [tss[g]], [strands[g]]).cpu().numpy()[:, 0]      # [2, 200, 2002]
        codes = np.stack([seq_codes(fa.sequence({"chr": chroms[g], "start": tss[g] + s * strands[g] - 999,
                                                 "stop": tss[g] + s * strands[g] + 1000}))
                          for s in pipe.shifts])
        want = _oracle_forward(sd, codes)
        assert_close(y.reshape(400, 2002), want, what=f"gene {g} window predictions")
        f_got = feats[g].cpu().numpy()
        # the reduction of our predictions is the oracle's bit for bit; against the oracle's own
        # predictions it is within the parity bar carried through the weights
        np.testing.assert_array_equal(f_got, tss_reduce(y[0], y[1], w))
        assert_close(f_got, tss_reduce(want[:200], want[200:], w), what=f"gene {g} features")


def test_configs3_rank_shard_12500_snvs_9_shifts():
    """configs[3]'s per-rank shape (100k SNVs over 8 GPUs = 12,500 SNVs x 9 shifts, +-800):
    sampled windows of every shift against the torch-CPU oracle, diff == alt - ref exactly, and
    the shard computed as the two halves a 2-rank split would hold (dist.shard_range) equals the
    whole bit for bit -- rank boundaries never change a row."""
    from expecto_amd import beluga, dist as edist, synthetic
    from expecto_amd.encode import seq_codes
    from expecto_amd.genome import DeviceGenome, Fasta
    from expecto_amd.pipeline import VariantPipeline, VariantSet, fetch_window, shift_order
    genome = synthetic.genome_bytes(n_contigs=8, contig_len=2_000_000, seed=33)
    fa = Fasta.from_dict(genome)
    n = 12_500
    snv = synthetic.snvs(genome, n, seed=3)
    vs = VariantSet([s[0] for s in snv], np.array([s[1] for s in snv]), [s[2] for s in snv], [s[3] for s in snv])
    shifts = shift_order(800)
    m = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=8192)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    eng = m.cuda().engine()
    pipe = VariantPipeline(eng, fa, DeviceGenome(fa))
    y = pipe.predict(vs, shifts)                           # [2 strands, 2 alleles, 9, n, 2002]
    assert y.shape == (2, 2, 9, n, 2002) and bool(torch.isfinite(y).all())
    d = pipe.diff(y)
    assert torch.equal(d, y[:, 1] - y[:, 0])
    for r in range(2):
        lo, hi = edist.shard_range(n, r, 2)
        part = VariantSet(vs.chrom[lo:hi], vs.pos[lo:hi], vs.ref[lo:hi], vs.alt[lo:hi])
        assert torch.equal(pipe.predict(part, shifts), y[:, :, :, lo:hi]), f"rank {r} half differs"
    rng = np.random.default_rng(5)
    pick = [(int(v), int(j)) for v, j in zip(rng.choice(n, 16, replace=False), rng.integers(0, 9, 16))]
    codes = np.stack([seq_codes(fetch_window(fa, vs.chrom[v], int(vs.pos[v]), vs.ref[v], al, shifts[j]))
                      for v, j in pick for al in (vs.ref[v], vs.alt[v])])         # 32 windows
    want = _oracle_forward(sd, codes)
    yc = y.cpu().numpy()
    got = np.stack([yc[st, a, j, v] for st in (0, 1) for v, j in pick for a in (0, 1)])
    assert_close(got, want, what="configs[3] rank shard sampled windows vs oracle")
