"""End-to-end CLI parity on the GPU: chromatin.py shift sweep -> .diff.h5, TSS features,
replicate per-gene predictions, and predict.py's variant feature reduction -- each against
the golden vectors produced by running the reference (tests/golden/make_golden.py)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, assert_close, run_in_roles, sweep_in_roles

pytestmark = pytest.mark.gpu

GENOME_ARGS = dict(n_contigs=3, contig_len=60000, seed=7)   # = make_golden.GENOME_ARGS


@pytest.fixture(scope="module")
def workdir(tmp_path_factory):
    from expecto_amd import synthetic
    d = tmp_path_factory.mktemp("pipe")
    synthetic.write_fasta(str(d / "hg19.fa"), synthetic.genome_bytes(**GENOME_ARGS))
    return d


def test_chromatin_cli_matches_reference(workdir, capsys):
    from expecto_amd import chromatin, h5
    vcf = workdir / "in.vcf"
    with open(vcf, "w") as f:
        f.write("##fileformat=VCFv4.1\n")
        f.write(open(os.path.join(GOLDEN, "chromatin_vcf.txt")).read())
    out = workdir / "chrom_out"
    chromatin.main([str(vcf), "--maxshift", "200", "--output_dir", str(out), "--genome", str(workdir / "hg19.fa"),
                    "--synthetic-weights", "0", "--max-batch", "40"])
    printed = [l for l in capsys.readouterr().out.splitlines() if l.startswith("Number of")]
    assert printed == open(os.path.join(GOLDEN, "chromatin_stdout.txt")).read().splitlines()
    assert open(out / "snps_hg19.vcf").read() == open(os.path.join(GOLDEN, "chromatin_snps_hg19.vcf")).read()
    gold = np.load(os.path.join(GOLDEN, "chromatin.npz"))
    for s in (0, -200, 200):
        got = h5.read(str(out / f"snps.shift_{s}.diff.h5"))
        assert sorted(got) == ["alt", "diff", "ref"]
        for k in ("ref", "alt", "diff"):
            assert got[k].dtype == np.float32 and got[k].shape == gold[f"{k}_{s}"].shape
            assert_close(got[k], gold[f"{k}_{s}"], what=f"shift {s} {k}")


def test_tss_compute_and_replicate_match_reference(workdir):
    from expecto_amd import tss
    anno = workdir / "anno.csv"
    anno.write_text("id,symbol,seqnames,strand,TSS,CAGE_representative_TSS,type\n"
                    "ENSGT0001,G1,chr1,+,30000,30000,protein_coding\n"
                    "ENSGT0002,G2,chr2,-,29000,29123,protein_coding\n")
    tssf = workdir / "tss.tsv"
    tssf.write_text("idx\tens_id\tchrom\ttss\tstrand\tcount\tis_default\n0\tENSGT0002\tchr2\t29123\t-\t5\tTrue\n")
    out = workdir / "tss_out"
    feats = tss.compute_main([str(anno), str(tssf), "-o", str(out), "--no-liftover", "--genome",
                              str(workdir / "hg19.fa"), "--synthetic-weights", "0", "--gene-batch", "1"])
    gold = np.load(os.path.join(GOLDEN, "tss.npz"))
    saved = np.load(out / "Xreducedall.2002.representative_tss_top.npy")
    assert saved.dtype == np.float64 and saved.shape == (2, 20020)
    assert_close(saved, gold["features"], what="TSS features")
    assert_close(feats, gold["features"], what="TSS features (returned)")
    anno1 = workdir / "anno1.csv"
    anno1.write_text("id,symbol,seqnames,strand,TSS,CAGE_representative_TSS,type\n"
                     "ENSGT0002,G2,chr2,-,29000,29123,protein_coding\n")
    rep = workdir / "rep_out"
    tss.replicate_main([str(anno1), "-o", str(rep), "--genome", str(workdir / "hg19.fa"), "--synthetic-weights",
                        "0"])
    pr = np.load(rep / "ENSGT0002.npy")
    assert pr.dtype == np.float32 and tuple(pr.shape) == tuple(gold["rep_shape"])
    assert_close(pr[::8], gold["rep_rows"], what="replicate rows")
    assert abs(pr.astype(np.float64).sum() - gold["rep_sum"][0]) <= 1e-4 * abs(gold["rep_sum"][0])


def test_variant_feature_reduction_matches_predict_py():
    """predict.py:87-136 on the reference's own chromatin outputs (captured golden)."""
    import torch
    from expecto_amd.features import fwd_rc_average, variant_features
    gold = np.load(os.path.join(GOLDEN, "chromatin.npz"))
    feats = np.load(os.path.join(GOLDEN, "predict_features.npz"))
    rows = [r.split("\t") for r in feats["gene_rows"]]
    coor = [r.split("\t") for r in feats["coor_rows"]]
    key = lambda r: (r[0].replace("chr", ""), r[2] if len(r) > 5 else r[1])
    vidx = [next(i for i, c in enumerate(coor) if c[0].replace("chr", "") == r[0] and c[1] == r[2]) for r in rows]
    shifts = [0, -200, 200]
    out = {}
    for name in ("diff", "ref", "alt"):
        eff = []
        for s in shifts:
            x = torch.from_numpy(gold[f"{name}_{s}"]).cuda()
            eff.append(fwd_rc_average(x)[torch.tensor(vidx, device="cuda")])
        eff = torch.stack(eff, 0)
        dist = -np.array([int(r[-1]) for r in rows])
        strand = np.array([r[-3] == "+" for r in rows])
        out[name] = variant_features(eff, dist, strand, shifts).cpu().numpy()
        assert_close(out[name], feats[name], rtol=1e-9, atol=1e-12, what=f"variant features {name}")


def _engine(precision="bf16x6", max_batch=300):
    import math
    from expecto_amd import beluga
    eng = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=max_batch).cuda().engine()
    eng.set_precision(precision)
    return eng


@pytest.mark.parametrize("precision", ["bf16x6", "f16x3", "fp32"])
def test_segment_path_is_bitwise_equal_to_per_window_variants(precision):
    """Trunk sharing across shifts (segment path) reproduces the per-window forward exactly."""
    import torch
    from expecto_amd import synthetic
    from expecto_amd.genome import DeviceGenome, Fasta
    from expecto_amd.pipeline import VariantPipeline, VariantSet, shift_order
    g = synthetic.genome_bytes(**GENOME_ARGS)
    fa = Fasta.from_dict(g)
    snv = synthetic.snvs(g, 23, seed=4)
    vs = VariantSet([s[0] for s in snv], np.array([s[1] for s in snv]), [s[2] for s in snv], [s[3] for s in snv])
    eng = _engine(precision)
    dg = DeviceGenome(fa)
    full = VariantPipeline(eng, fa, dg, use_segments=False, use_pairs=False)
    for shifts in (shift_order(800), shift_order(200), [0, 400, -400]):
        for pairs in (True, False):
            b = sweep_in_roles(eng, lambda: full.predict(vs, shifts), shifts, pairs)   # each window in its FC1 role
            seg = VariantPipeline(eng, fa, dg, use_segments=True, use_pairs=pairs)
            ps = seg.prepare(vs, shifts)
            assert ps["seg"] is not None and ps["seg"]["pairs"] == pairs
            a = seg.predict(ps)
            assert torch.equal(a, b), f"segment path (pairs={pairs}) differs for shifts {shifts}: " \
                                      f"{float((a - b).abs().max())}"


def test_segment_path_mixed_snv_and_indel_batch():
    import torch
    from expecto_amd import synthetic
    from expecto_amd.genome import DeviceGenome, Fasta
    from expecto_amd.pipeline import VariantPipeline, VariantSet, shift_order
    g = synthetic.genome_bytes(**GENOME_ARGS)
    fa = Fasta.from_dict(g)
    snv = synthetic.snvs(g, 6, seed=9)
    rows = [(c, p, r, a) for c, p, r, a in snv]
    base = chr(g["chr2"][30000 - 1]).upper()
    rows.insert(2, ("chr2", 30000, base, base + "GA"))
    rows.insert(5, ("chr1", 25000, chr(g["chr1"][24999]).upper() + chr(g["chr1"][25000]).upper(),
                    chr(g["chr1"][24999]).upper()))
    vs = VariantSet([r[0] for r in rows], np.array([r[1] for r in rows]), [r[2] for r in rows], [r[3] for r in rows])
    eng = _engine()
    dg = DeviceGenome(fa)
    a = VariantPipeline(eng, fa, dg, use_segments=True).predict(vs, shift_order(400))
    b = VariantPipeline(eng, fa, dg, use_segments=False, use_pairs=False).predict(vs, shift_order(400))
    assert torch.equal(a, b)


def test_segment_path_is_bitwise_equal_to_per_window_tss():
    import torch
    from expecto_amd import synthetic
    from expecto_amd.genome import DeviceGenome, Fasta
    from expecto_amd.tss import TSSPipeline
    fa = Fasta.from_dict(synthetic.genome_bytes(**GENOME_ARGS))
    pipe = TSSPipeline(_engine(), DeviceGenome(fa))
    genes = (["chr1", "chr2", "chr3"], [30000, 29123, 31000], [1, -1, -1])
    a = pipe.predict(*genes, use_segments=True)
    b = pipe.predict(*genes, use_segments=False)
    assert torch.equal(a, b)


@pytest.mark.parametrize("precision", ["bf16x6", "f16x3", "fp32"])
def test_pair_path_alt_cone_is_bitwise_equal(precision):
    """Alt-cone reuse (only the SNV's receptive-field rows recomputed) == full alt forward,
    for SNVs anywhere in the window, both strands."""
    import torch
    eng = _engine(precision)
    rng = np.random.default_rng(7)
    pos = np.array([0, 5, 100, 308, 309, 310, 500, 998, 999, 1000, 1500, 1690, 1700, 1701, 1990, 1999], np.int32)
    n = pos.size
    ref = torch.from_numpy(rng.integers(0, 5, (n, 2000)).astype(np.uint8)).cuda()
    alt = ref.clone()
    newb = torch.from_numpy(((ref.cpu().numpy()[np.arange(n), pos] + 1 + rng.integers(0, 3, n)) % 4)
                            .astype(np.uint8)).cuda()
    alt[torch.arange(n), torch.from_numpy(pos).long()] = newb
    y = torch.empty((2, 2, n, 2002), device="cuda")
    yv = y.view(4 * n, 2002)
    eng.forward_pairs(ref, alt, pos, yv[0:], yv[n:], 2 * n, 2)
    want_ref = eng.forward_codes(ref, 2)
    want_alt = eng.forward_codes(alt, 2)
    assert torch.equal(y[:, 0].reshape(2 * n, 2002), want_ref)
    d = (y[:, 1].reshape(2 * n, 2002) - want_alt).abs().amax(-1).view(2, n).cpu().numpy()
    assert (d == 0).all(), f"alt rows differ: strand x window max|diff| = {d} (positions {pos})"
    assert not torch.equal(want_ref, want_alt)


def test_variant_pipeline_pairs_equal_per_window():
    import torch
    from expecto_amd import synthetic
    from expecto_amd.genome import DeviceGenome, Fasta
    from expecto_amd.pipeline import VariantPipeline, VariantSet
    g = synthetic.genome_bytes(**GENOME_ARGS)
    fa = Fasta.from_dict(g)
    snv = synthetic.snvs(g, 37, seed=12)
    vs = VariantSet([s[0] for s in snv], np.array([s[1] for s in snv]), [s[2] for s in snv], [s[3] for s in snv])
    eng = _engine()
    dg = DeviceGenome(fa)
    a = VariantPipeline(eng, fa, dg, use_pairs=True).predict(vs, [0])
    b = VariantPipeline(eng, fa, dg, use_pairs=False).predict(vs, [0])
    assert torch.equal(a, b)


@pytest.mark.parametrize("precision,max_batch", [("bf16x6", 300), ("f16x3", 300), ("fp32", 300), ("f16x3", 40)])
def test_segment_pairs_alt_runs_are_bitwise_equal(precision, max_batch):
    """forward_segment_pairs == full forwards of every ref and alt window, for SNVs at the
    segment edges and in the middle, windows at the first/last offsets, both strands.
    max_batch 40: 10-segment chunks of 80 windows, each chunk's FC in two slices of 40 rows with
    alt windows in both (the alt FC of a slice reuses that slice's ref partials)."""
    import torch
    eng = _engine(precision, max_batch)
    rng = np.random.default_rng(11)
    L = 2000 + 1600
    q = np.array([0, 3, 7, 500, 1234, 1799, 1800, 2001, 3000, L - 9, L - 2, L - 1], np.int32)
    n = q.size
    ref = torch.from_numpy(rng.integers(0, 5, (n, L)).astype(np.uint8)).cuda()
    alt_code = torch.from_numpy(((ref.cpu().numpy()[np.arange(n), q] + 1 + rng.integers(0, 3, n)) % 4)
                                .astype(np.uint8)).cuda()
    alt = ref.clone()
    alt[torch.arange(n), torch.from_numpy(q).long()] = alt_code
    offs = np.array([0, 4, 200, 796, 800, 1000, 1596, 1600], np.int32)   # some windows miss some SNVs
    S = offs.size
    v_i, j_i = np.meshgrid(np.arange(n), np.arange(S), indexing="ij")
    win_seg, win_off, win_row = v_i.ravel().astype(np.int32), offs[j_i.ravel()], (j_i * n + v_i).ravel().astype(np.int32)
    y = torch.full((2, 2, S * n, 2002), float("nan"), device="cuda")
    yf = y.view(4 * S * n, 2002)
    eng.forward_segment_pairs(ref, L, q, alt_code, win_seg, win_off, win_row, yf[0:],
                              yf[S * n:], 2 * S * n)
    from expecto_amd.pipeline import fc1_role
    for a, src in enumerate((ref, alt)):
        wins = torch.stack([src[:, o:o + 2000] for o in offs], 0).reshape(S * n, 2000).contiguous()  # row j*n + v
        by_role = run_in_roles(eng, lambda: eng.forward_codes(wins, 2).view(2, S, n, 2002))
        # each window in its FC1 role; the direct FC1 (role 4) when > 1/3 of the windows hold the SNV
        n_alt = int(sum(((o <= q) & (q < o + 2000)).sum() for o in offs))
        role = (lambda o, sd: 4) if 3 * n_alt > S * n else (lambda o, sd: fc1_role(int(o), L, sd == 1))
        want = torch.stack([torch.stack([by_role[role(o, sd)][sd, j] for j, o in enumerate(offs)])
                            for sd in range(2)]).view(2, S * n, 2002)
        d = (y[:, a] - want).abs().amax(-1).view(2, S, n).cpu().numpy()
        assert (d == 0).all(), f"allele {a}: strand x offset x variant max|diff| {d} (q={q}, offsets={offs})"


def test_second_stream_overlap_is_bitwise_equal(monkeypatch):
    """The alt-delta launches on the handle's second stream (pair and segment-pair paths,
    EXPECTO_OVERLAP=1, the default) give exactly the single-stream results, on batches large
    enough that the ref launches run many rounds beside them."""
    import math
    import torch
    from expecto_amd import beluga
    rng = np.random.default_rng(21)
    n = 1200
    pos = rng.integers(0, 2000, n).astype(np.int32)
    ref = torch.from_numpy(rng.integers(0, 5, (n, 2000)).astype(np.uint8)).cuda()
    alt = ref.clone()
    newb = torch.from_numpy(((ref.cpu().numpy()[np.arange(n), pos] + 1) % 4).astype(np.uint8)).cuda()
    alt[torch.arange(n), torch.from_numpy(pos).long()] = newb
    L, ns = 3600, 150
    q = rng.integers(0, L, ns).astype(np.int32)
    seg = torch.from_numpy(rng.integers(0, 5, (ns, L)).astype(np.uint8)).cuda()
    alt_code = torch.from_numpy(((seg.cpu().numpy()[np.arange(ns), q] + 2) % 4).astype(np.uint8)).cuda()
    offs = np.arange(0, 1601, 200, dtype=np.int32)
    v_i, j_i = np.meshgrid(np.arange(ns), np.arange(offs.size), indexing="ij")
    win_seg, win_off = v_i.ravel().astype(np.int32), offs[j_i.ravel()]
    win_row = (j_i * ns + v_i).ravel().astype(np.int32)
    W = win_seg.size
    out = {}
    for ov in ("0", "1"):
        monkeypatch.setenv("EXPECTO_OVERLAP", ov)
        eng = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=2400).cuda().engine()
        y = torch.empty((2, 2, n, 2002), device="cuda")
        yv = y.view(4 * n, 2002)
        eng.forward_pairs(ref, alt, pos, yv[0:], yv[n:], 2 * n, 2)
        ys = torch.empty((2, 2, W, 2002), device="cuda")
        yf = ys.view(4 * W, 2002)
        eng.forward_segment_pairs(seg, L, q, alt_code, win_seg, win_off, win_row, yf[0:], yf[W:], 2 * W)
        torch.cuda.synchronize()
        out[ov] = (y.cpu(), ys.cpu())
        del eng
    assert torch.equal(out["0"][0], out["1"][0])
    assert torch.equal(out["0"][1], out["1"][1])


@pytest.mark.parametrize("ranks", [2, 4])
def test_chromatin_cli_two_ranks_equals_one(workdir, ranks):
    """The CLI sharded over 2 or 4 ranks (torch.distributed.run; gloo, every rank on this one GPU:
    the 8-GPU RCCL run is the driver's) and streamed in batches of 2 variants (uneven last
    batches) writes the same files byte for byte as one rank in one batch, in both output modes:
    every rank writing its own rows into the files rank 0 created (default), and each batch
    gathered to rank 0 which writes it (4 ranks: shards of 2, 2, 1, 1 variants, so
    gather_blocks_to pads 4 unequal blocks).  Shards are contiguous variant
    ranges; only rank 0 writes snps_hg19.vcf; no .part file is left.  One rank streaming 2-variant
    batches writes the same bytes too."""
    import socket
    import subprocess
    import sys
    from expecto_amd import chromatin, h5
    vcf = workdir / "in2.vcf"
    with open(vcf, "w") as f:
        f.write("##fileformat=VCFv4.1\n")
        f.write(open(os.path.join(GOLDEN, "chromatin_vcf.txt")).read())
    common = ["--maxshift", "200", "--genome", str(workdir / "hg19.fa"), "--synthetic-weights", "0",
              "--max-batch", "40"]
    one = workdir / "out_1rank"
    chromatin.main([str(vcf), "--output_dir", str(one)] + common)
    one_b2 = workdir / "out_1rank_b2"
    chromatin.main([str(vcf), "--output_dir", str(one_b2), "--variant-batch", "2"] + common)
    names = ["snps_hg19.vcf"] + [f"snps.shift_{sh}.diff.h5" for sh in (0, -200, 200)]
    for mode in ("rank", "gather"):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        two = workdir / f"out_{ranks}rank_{mode}"
        env = dict(os.environ, EXPECTO_DIST_BACKEND="gloo", EXPECTO_SHARE_GPUS="1")
        r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(ranks),
                            "--master-addr", "127.0.0.1", "--master-port", str(port), "-m", "expecto_amd.chromatin",
                            str(vcf), "--output_dir", str(two), "--variant-batch", "2", "--output-mode", mode] + common,
                           env=env, cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                           capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-3000:]
        assert sorted(os.listdir(two)) == sorted(names), mode
        for name in names:
            want = open(one / name, "rb").read()
            assert open(two / name, "rb").read() == want, (mode, name)
            assert open(one_b2 / name, "rb").read() == want, name
        a = h5.read(str(two / "snps.shift_200.diff.h5"))
        assert a["ref"].shape == (12, 2002) and float(np.abs(a["ref"]).min()) > 0


def test_chromatin_cli_failed_batch_leaves_no_output(workdir):
    """A batch that fails after earlier batches were written (here: an invalid alt base in the
    4th 2-variant batch -> KeyError, as encodeSeqs raises in the reference) leaves no
    snps.shift_*.diff.h5 (nor .part) behind: the files are written as .part and renamed only
    once every batch succeeded (the reference computes everything before it writes)."""
    from expecto_amd import chromatin
    vcf = workdir / "bad.vcf"
    lines = [l for l in open(os.path.join(GOLDEN, "chromatin_vcf.txt")).read().splitlines()
             if l and not l.startswith("#")]
    snv = [l for l in lines if len(l.split("\t")[3]) == 1 and len(l.split("\t")[4]) == 1]
    assert len(snv) >= 3
    with open(vcf, "w") as f:
        for l in snv[:3] * 2:
            f.write(l + "\n")
        c = snv[0].split("\t")
        c[4] = "Z"
        f.write("\t".join(c) + "\n")
    out = workdir / "out_bad"
    with pytest.raises(KeyError):
        chromatin.main([str(vcf), "--output_dir", str(out), "--maxshift", "200", "--genome", str(workdir / "hg19.fa"),
                        "--synthetic-weights", "0", "--max-batch", "40", "--variant-batch", "2"])
    left = sorted(os.listdir(out))
    assert left == ["snps_hg19.vcf"], left


def test_chromatin_cli_overflowed_batches_are_recomputed(workdir, monkeypatch):
    """The streamed CLI's f16x3 overflow recovery: with every activation pushed past
    fp16's range (calibration target 2^20) every 2-variant batch flags; complete() recomputes the
    flagged variant slices in bf16x6 before the batch's rows are written, so the files equal a
    bf16x6 run byte for byte and the engine counts one fallback per recomputed slice."""
    from expecto_amd import chromatin
    vcf = workdir / "ovf.vcf"
    with open(vcf, "w") as f:
        f.write("##fileformat=VCFv4.1\n")
        f.write(open(os.path.join(GOLDEN, "chromatin_vcf.txt")).read())
    common = ["--maxshift", "200", "--genome", str(workdir / "hg19.fa"), "--synthetic-weights", "0",
              "--max-batch", "40", "--variant-batch", "2"]
    monkeypatch.setenv("EXPECTO_PRECISION", "bf16x6")
    ref = workdir / "out_bf16x6"
    chromatin.main([str(vcf), "--output_dir", str(ref)] + common)
    monkeypatch.setenv("EXPECTO_PRECISION", "f16x3")
    real, engines = chromatin.load_model, []

    def forced(args):
        m = real(args)
        eng = m.engine()
        eng.set_f16_target(20)
        engines.append((eng, eng.f16_state()[0]))
        return m
    monkeypatch.setattr(chromatin, "load_model", forced)
    out = workdir / "out_f16_forced"
    chromatin.main([str(vcf), "--output_dir", str(out)] + common)
    run = dict(chromatin.LAST_RUN)
    assert run["batches"] > 1 and run["recomputed_batches"] == run["batches"], run
    eng, fb0 = engines[0]
    assert eng.f16_state()[0] - fb0 == run["bf16x6_recomputes"] >= run["batches"], run
    assert run["recomputed_slices"] >= run["bf16x6_recomputes"], run
    eng.set_f16_target(10)
    names = sorted(os.listdir(ref))
    assert sorted(os.listdir(out)) == names
    for name in names:
        assert open(out / name, "rb").read() == open(ref / name, "rb").read(), name


def test_recompute_overflowed_without_relocated_slice_redoes_the_batch(monkeypatch):
    """a batch whose deferred flag fired but whose slice reruns all report no
    overflow (forced here by routing the reruns' flag copies to a scratch tensor) is recomputed
    whole in bf16x6 instead of keeping its f16x3 rows."""
    import torch
    from expecto_amd import synthetic
    from expecto_amd.genome import DeviceGenome, Fasta
    from expecto_amd.pipeline import VariantPipeline, VariantSet, shift_order
    g = synthetic.genome_bytes(**GENOME_ARGS)
    fa = Fasta.from_dict(g)
    snv = synthetic.snvs(g, 10, seed=9)
    vs = VariantSet([s[0] for s in snv], np.array([s[1] for s in snv]), [s[2] for s in snv], [s[3] for s in snv])
    shifts = shift_order(200)
    eng = _engine("f16x3")
    eng.set_overflow_check(deferred=True)
    eng.set_f16_target(20)
    pipe = VariantPipeline(eng, fa, DeviceGenome(fa))
    y = pipe.predict(vs, shifts)
    flag = torch.zeros(1, dtype=torch.int32).pin_memory()
    eng.overflow_take(flag)
    torch.cuda.synchronize()
    assert int(flag[0]) == 1
    real, scratch = eng.overflow_take, torch.zeros(1, dtype=torch.int32).pin_memory()
    monkeypatch.setattr(eng, "overflow_take", lambda dst, stream=None: real(scratch, stream))
    fb0 = eng.f16_state()[0]
    redone = pipe.recompute_overflowed(vs, shifts, y)
    torch.cuda.synchronize()
    assert redone == 1 and eng.f16_state()[0] - fb0 == 1   # one whole-batch recompute, counted once
    assert pipe.last_recomputed_slices == min(8, len(vs))    # ... which rewrote every slice
    with eng.precision_override("bf16x6"):
        want = pipe.predict(vs, shifts)
    assert torch.equal(y, want)
    eng.set_f16_target(10)
    eng.set_overflow_check(deferred=False)


def test_chromatin_cli_batch_gb_caps_the_batch():
    """--batch-gb lowers --variant-batch so one batch's y + diff of every shift fits the cap
    (a 201-shift sweep at the default 4096 variants would pin ~79 GB)."""
    from expecto_amd import chromatin
    a = chromatin.build_parser().parse_args(["x.vcf"])
    assert chromatin.batch_variants(a, 9) == 4096
    per_variant = 6 * 201 * 2002 * 4
    b = chromatin.batch_variants(a, 201)
    assert b * per_variant <= 4 * (1 << 30) < (b + 1) * per_variant
    a = chromatin.build_parser().parse_args(["x.vcf", "--batch-gb", "0"])
    assert chromatin.batch_variants(a, 9) == 1


def test_replicate_streamed_equals_one_batch(workdir, monkeypatch):
    """The streamed replicate CLI (two pinned slots, batch k's .npy files
    written while batch k+1 computes, deferred overflow check) writes the same bytes in batches
    of 2 genes as in one batch; a duplicated gene id keeps its last row's file, as the
    reference's sequential writes leave it; with every activation forced past fp16's range each
    batch is recomputed in bf16x6 and the files equal a bf16x6 run byte for byte."""
    from expecto_amd import tss
    rows = [("ENSGT0001", "chr1", 30000, "+"), ("ENSGT0002", "chr2", 29123, "-"), ("ENSGT0003", "chr3", 25000, "+"),
            ("ENSGT0004", "chr1", 34000, "-"), ("ENSGT0002", "chr3", 33000, "+"), ("ENSGT0005", "chr2", 23000, "+"),
            ("ENSGT0006", "chr3", 37000, "-")]
    anno = workdir / "anno_rep.csv"
    anno.write_text("id,symbol,seqnames,strand,TSS,CAGE_representative_TSS,type\n" +
                    "".join(f"{g},S{k},{c},{s},{t},{t},protein_coding\n" for k, (g, c, t, s) in enumerate(rows)))
    last = workdir / "anno_rep_last.csv"
    last.write_text("id,symbol,seqnames,strand,TSS,CAGE_representative_TSS,type\n"
                    "ENSGT0002,S4,chr3,+,33000,33000,protein_coding\n")
    common = ["--genome", str(workdir / "hg19.fa"), "--synthetic-weights", "0", "--max-batch", "400"]
    outs = {}
    for name, extra in (("b2", ["--gene-batch", "2"]), ("b16", ["--gene-batch", "16"])):
        outs[name] = workdir / f"rep_{name}"
        r = tss.replicate_main([str(anno), "-o", str(outs[name])] + common + extra)
        assert r["genes"] == 6 and r["batches"] == (3 if name == "b2" else 1), r
    names = sorted(os.listdir(outs["b16"]))
    assert names == sorted({f"{g}.npy" for g, _, _, _ in rows})
    for n in names:
        assert open(outs["b2"] / n, "rb").read() == open(outs["b16"] / n, "rb").read(), n
    one = workdir / "rep_last"
    tss.replicate_main([str(last), "-o", str(one)] + common)
    assert open(one / "ENSGT0002.npy", "rb").read() == open(outs["b2"] / "ENSGT0002.npy", "rb").read()
    monkeypatch.setenv("EXPECTO_PRECISION", "bf16x6")
    ref = workdir / "rep_bf16x6"
    tss.replicate_main([str(anno), "-o", str(ref), "--gene-batch", "2"] + common)
    monkeypatch.setenv("EXPECTO_PRECISION", "f16x3")
    real = tss._load_model

    def forced(args):
        m = real(args)
        m.engine().set_f16_target(20)
        return m
    monkeypatch.setattr(tss, "_load_model", forced)
    ovf = workdir / "rep_forced"
    r = tss.replicate_main([str(anno), "-o", str(ovf), "--gene-batch", "2"] + common)
    assert r["recomputed_batches"] == r["batches"] == 3, r
    for n in names:
        assert open(ovf / n, "rb").read() == open(ref / n, "rb").read(), n


def test_tss_compute_two_ranks_equals_one(workdir):
    """compute_expecto_features over 2 ranks (torch.distributed.run, gloo on this one GPU): genes
    shard by rank ranges and rank 0 gathers the f64 [G_r, 20020] blocks; the .npy equals the
    one-rank file bit for bit."""
    import socket
    import subprocess
    import sys
    from expecto_amd import tss
    anno = workdir / "anno3.csv"
    anno.write_text("id,symbol,seqnames,strand,TSS,CAGE_representative_TSS,type\n"
                    "ENSGT0001,G1,chr1,+,30000,30000,protein_coding\n"
                    "ENSGT0002,G2,chr2,-,29000,29123,protein_coding\n"
                    "ENSGT0003,G3,chr3,+,31000,31000,protein_coding\n")
    tssf = workdir / "tss3.tsv"
    tssf.write_text("idx\tens_id\tchrom\ttss\tstrand\tcount\tis_default\n")
    common = [str(anno), str(tssf), "--no-liftover", "--genome", str(workdir / "hg19.fa"), "--synthetic-weights",
              "0", "--gene-batch", "1"]
    one = workdir / "tss_1rank"
    tss.compute_main(common + ["-o", str(one)])
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    two = workdir / "tss_2rank"
    env = dict(os.environ, EXPECTO_DIST_BACKEND="gloo", EXPECTO_SHARE_GPUS="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "-m", "expecto_amd.tss",
                        "compute"] + common + ["-o", str(two)],
                       env=env, cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    name = "Xreducedall.2002.representative_tss_top.npy"
    a, b = np.load(one / name), np.load(two / name)
    assert a.shape == (3, 20020)
    np.testing.assert_array_equal(a, b)


def test_indel_windows_device_equal_host_splice():
    """Indel / MNP windows built by expecto_indel_windows equal the host fetch_window +
    seq_codes (chromatin.py:164,202-209) for insertions, deletions, MNPs, an N in the allele,
    deletions longer than 100 bp (spliced length < 2000: the host's Python-slicing path) and a
    window cut by the contig end (host path)."""
    from expecto_amd import synthetic
    from expecto_amd.encode import seq_codes
    from expecto_amd.genome import DeviceGenome, Fasta
    from expecto_amd.pipeline import VariantPipeline, VariantSet, fetch_window, shift_order
    g = synthetic.genome_bytes(**GENOME_ARGS)
    fa = Fasta.from_dict(g)
    pipe = VariantPipeline(_engine(), fa, DeviceGenome(fa))
    rng = np.random.default_rng(31)
    rows = []
    names = sorted(g)
    for lr, la in [(1, 2), (1, 7), (1, 60), (2, 1), (9, 1), (40, 1), (3, 3), (5, 2), (2, 5), (150, 1), (120, 4),
                   (1, 1200)]:
        c = names[int(rng.integers(0, len(names)))]
        p = int(rng.integers(3000, len(g[c]) - 3000))
        ref = g[c][p - 1:p - 1 + lr].decode().upper()
        alt = "".join("ACGT"[int(x)] for x in rng.integers(0, 4, la))
        rows.append((c, p, ref, alt))
    rows.append((names[0], 5000, g[names[0]][4999:5001].decode().upper(), "ANT"))
    c = names[1]
    p = len(g[c]) - 900                                   # the +800 windows run past the contig end
    rows.append((c, p, g[c][p - 1:p + 1].decode().upper(), "G"))
    vs = VariantSet([r[0] for r in rows], np.array([r[1] for r in rows]), [r[2] for r in rows], [r[3] for r in rows])
    shifts = shift_order(800)
    got = pipe._indel_window_codes(vs, np.arange(len(rows)), shifts).cpu().numpy()
    want = np.full(got.shape, 4, np.uint8)
    for k, (c, p, r, a) in enumerate(rows):
        for j, sh in enumerate(shifts):
            for ai, allele in enumerate((r, a)):
                cc = seq_codes(fetch_window(fa, c, p, r, allele, sh))
                want[ai, j, k, :cc.size] = cc
    bad = np.argwhere((got != want).any(-1))
    assert bad.size == 0, f"(allele, shift, item) rows differ: {bad[:8].tolist()}"


def test_chromatin_cli_shift0_rows_equal_across_maxshift(workdir):
    """The reference's two sweep modes (chromatin.py:243: --maxshift 0 and the default 800) write
    the same shift-0 `.diff.h5` byte for byte: per-window forwards and the +-800 segment pairs both
    run the direct FC1 (role 4, include/expecto_hip.h expecto_beluga_set_fc1_role).  And the
    operator API on those windows -- Beluga.forward of encodeSeqs' one-hot [fwd; rc] rows
    (chromatin.py:266-279) -- returns the same bits as the +-800 file's `ref` and `alt` rows
    (VERDICT r05 item 2).  SNVs, a ref mismatch, an insertion and a deletion (the golden VCF)."""
    import math
    import torch
    from expecto_amd import beluga, chromatin, h5
    from expecto_amd.encode import encodeSeqs
    from expecto_amd.genome import Fasta
    from expecto_amd.pipeline import fetch_window
    vcf = workdir / "in_modes.vcf"
    with open(vcf, "w") as f:
        f.write("##fileformat=VCFv4.1\n")
        f.write(open(os.path.join(GOLDEN, "chromatin_vcf.txt")).read())
    common = ["--genome", str(workdir / "hg19.fa"), "--synthetic-weights", "0", "--max-batch", "40"]
    files = {}
    for ms in (0, 800):
        d = workdir / f"modes_{ms}"
        chromatin.main([str(vcf), "--maxshift", str(ms), "--output_dir", str(d)] + common)
        files[ms] = d / "snps.shift_0.diff.h5"
    assert open(files[0], "rb").read() == open(files[800], "rb").read()
    got = h5.read(str(files[800]))
    vs = chromatin.read_variants(chromatin.build_parser().parse_args([str(vcf), "--output_dir", str(workdir)]
                                                                     + common), write_side_files=False)
    fa = Fasta(str(workdir / "hg19.fa"))
    m = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=40).cuda()
    for k, alleles in (("ref", vs.ref), ("alt", vs.alt)):
        seqs = [fetch_window(fa, c, int(p), r, a, 0) for c, p, r, a in zip(vs.chrom, vs.pos, vs.ref, alleles)]
        x = torch.from_numpy(encodeSeqs(seqs).astype(np.float32)).unsqueeze(2).cuda()
        y = torch.cat([m(x[i:i + 32]) for i in range(0, x.shape[0], 32)]).cpu().numpy()   # batchSize 32
        assert y.shape == got[k].shape
        assert np.array_equal(y.view(np.uint32), got[k].view(np.uint32)), k
