"""CPU: host-side logic of the drop-in CLIs (no GPU): genome access, window geometry,
VCF handling, allele checks -- against the oracle and the reference's golden files."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

GENOME_ARGS = dict(n_contigs=3, contig_len=60000, seed=7)


@pytest.fixture(scope="module")
def genome():
    from expecto_amd import synthetic
    return synthetic.genome_bytes(**GENOME_ARGS)


def test_fasta_roundtrip_and_one_based_slices(tmp_path, genome):
    from expecto_amd import synthetic
    from expecto_amd.genome import Fasta
    p = str(tmp_path / "g.fa")
    synthetic.write_fasta(p, genome)
    fa = Fasta(p)
    assert list(fa.keys()) == ["chr1", "chr2", "chr3"]
    for c in fa.keys():
        assert bytes(fa.raw(c)) == genome[c]
    s = fa.sequence({"chr": "chr2", "start": 101, "stop": 110})
    assert s == genome["chr2"][100:110].decode() and len(s) == 10


def test_code_genome_layout(genome):
    from expecto_amd.encode import seq_codes
    from expecto_amd.genome import GUARD, CodeGenome, Fasta
    cg = CodeGenome(Fasta.from_dict(genome))
    for c in genome:
        o = cg.offsets[c]
        assert np.array_equal(cg.codes[o:o + 5000], seq_codes(genome[c][:5000], 5000))
        assert (cg.codes[o - GUARD:o] == 4).all()
    assert cg.invalid_offsets.size == 0
    bad = dict(genome)
    bad["chr2"] = genome["chr2"][:100] + b"R" + genome["chr2"][101:]
    cg2 = CodeGenome(Fasta.from_dict(bad))
    assert cg2.invalid_offsets.tolist() == [cg2.offsets["chr2"] + 100] and bytes(cg2.invalid_chars) == b"R"


@pytest.mark.parametrize("shift", [0, -200, 200, -800, 800])
def test_snv_window_geometry_equals_fetchseqs(genome, shift):
    """What expecto_variant_windows computes on the device (genome[off+shift-999+i] with the
    allele at 999-shift) equals fetchSeqs + the encodeSeqs crop (oracle)."""
    from expecto_amd.encode import seq_codes
    from expecto_amd.genome import CodeGenome, Fasta
    from oracle.encode_np import fetch_seqs
    fa = Fasta.from_dict(genome)
    cg = CodeGenome(fa)
    rng = np.random.default_rng(abs(shift) + 1)
    for pos in rng.integers(3000, 57000, 5):
        pos = int(pos)
        refb = chr(genome["chr1"][pos - 1]).upper()
        for allele in ("A", "G"):
            r, a, _, _ = fetch_seqs(fa, "chr1", pos, refb, allele, shift=shift)
            want_ref, want_alt = seq_codes(r), seq_codes(a)
            off = cg.offset("chr1", pos) + shift - 999
            win = cg.codes[off:off + 2000].copy()
            win_ref = win.copy()
            win_ref[999 - shift] = seq_codes(refb, 1)[0]
            win[999 - shift] = seq_codes(allele, 1)[0]
            assert np.array_equal(win_ref, want_ref)
            assert np.array_equal(win, want_alt)


def test_tss_window_geometry_equals_reference(genome):
    from expecto_amd.encode import seq_codes
    from expecto_amd.genome import CodeGenome, Fasta
    from oracle.encode_np import tss_window
    fa = Fasta.from_dict(genome)
    cg = CodeGenome(fa)
    for strand in (1, -1):
        for s in (-20000, -200, 0, 19800):
            want = seq_codes(tss_window(fa, "chr2", 30000, strand, s))
            off = cg.offset("chr2", 30000) + s * strand - 999
            assert np.array_equal(cg.codes[off:off + 2000], want)


def test_indel_windows_host_path(genome):
    from expecto_amd.encode import seq_codes
    from expecto_amd.genome import Fasta
    from expecto_amd.pipeline import fetch_window
    from oracle.encode_np import encode_seqs, fetch_seqs
    fa = Fasta.from_dict(genome)
    g = genome["chr3"]
    pos = 40000
    ref = chr(g[pos - 1]).upper()
    for r, a in ((ref, ref + "TT"), (ref + chr(g[pos]).upper(), ref)):
        rs, as_, _, _ = fetch_seqs(fa, "chr3", pos, r, a, shift=-200)
        for allele, want in ((r, rs), (a, as_)):
            w = fetch_window(fa, "chr3", pos, r, allele, -200)
            assert w == want
            oh = encode_seqs([w])[0]
            c = seq_codes(w)
            assert np.array_equal(oh.argmax(0)[oh.any(0)], c[c < 4])


def test_read_variants_matches_reference_side_outputs(tmp_path):
    from expecto_amd import chromatin
    from expecto_amd.pipeline import shift_order
    vcf = tmp_path / "in.vcf"
    vcf.write_text("##fileformat=VCFv4.1\n" + open(os.path.join(GOLDEN, "chromatin_vcf.txt")).read())
    args = chromatin.build_parser().parse_args([str(vcf), "--output_dir", str(tmp_path)])
    vs = chromatin.read_variants(args)
    assert open(tmp_path / "snps_hg19.vcf").read() == open(os.path.join(GOLDEN, "chromatin_snps_hg19.vcf")).read()
    assert vs.chrom == ["chr1", "chr2", "chr2", "chr3", "chr3", "chr1"]
    assert shift_order(800) == [0, -200, -400, -600, -800, 200, 400, 600, 800]
    assert shift_order(0) == [0]


def test_match_counts_match_reference_stdout(genome):
    from expecto_amd.genome import Fasta
    from expecto_amd.pipeline import VariantSet, match_counts
    rows = [l.split("\t") for l in open(os.path.join(GOLDEN, "chromatin_vcf.txt")).read().splitlines()]
    rows = [r for r in rows if not r[0].startswith("chrUn")]
    vs = VariantSet(["chr" + r[0].replace("chr", "") for r in rows], np.array([int(r[1]) for r in rows]),
                    [r[3] for r in rows], [r[4] for r in rows])
    rm, am = match_counts(Fasta.from_dict(genome), vs)
    lines = open(os.path.join(GOLDEN, "chromatin_stdout.txt")).read().splitlines()
    assert lines[0].endswith(f": {rm.sum()}") and lines[1].endswith(f": {am.sum()}") and lines[2].endswith(f": {len(rm)}")


def test_allele_code_rejects_unknown():
    from expecto_amd.pipeline import _allele_code
    assert [_allele_code(c) for c in "AGCTagctNn-H"] == [0, 1, 2, 3, 0, 1, 2, 3, 4, 4, 4, 4]
    with pytest.raises(KeyError):
        _allele_code("R")


def test_inputsize_other_than_2000_is_rejected(tmp_path):
    from expecto_amd import tss
    with pytest.raises(ValueError):
        tss.replicate_main([str(tmp_path / "a.csv"), "--windowsize", "1000"])


def test_variant_tables_and_decay_table_follow_predict_py():
    """features.variant_tables (the per-batch inputs the variant reduction keeps resident; the
    bench times the kernel on them) on the CPU: dtypes the C-ABI binds and the exp table equal
    to numpy's exp of predict.py:88-107's arguments for every floor(|d|/200) of the batch."""
    import torch
    from expecto_amd.features import DECAY, decay_table, variant_tables
    from expecto_amd.pipeline import shift_order
    rng = np.random.default_rng(8)
    dist = rng.integers(-40000, 40000, 50)
    plus = rng.random(50) < 0.5
    shifts = shift_order(800)
    d, sp, sh, lut = variant_tables(dist, plus, shifts, torch.device("cpu"))
    assert (d.dtype, sp.dtype, sh.dtype, lut.dtype) == (torch.int64, torch.uint8, torch.int32, torch.float64)
    assert d.tolist() == dist.tolist() and sp.tolist() == plus.astype(np.uint8).tolist() and sh.tolist() == shifts
    tab = decay_table(dist, plus, shifts)
    assert np.array_equal(lut.numpy(), tab)
    sgn = np.where(plus, 1, -1)
    fl = np.floor(np.abs(dist[:, None] * sgn[:, None] + np.asarray(shifts)[None] * sgn[:, None]) / 200.0)
    assert tab.shape[1] == int(fl.max()) + 1
    for k, c in enumerate(DECAY):
        np.testing.assert_array_equal(tab[k][fl.astype(int)], np.exp(-c * fl))


def test_beluga_parameter_slots_follow_replaced_modules():
    """Beluga._params caches each parameter's owner module once (host time per forward) and checks
    the cached module links by identity: a replaced submodule, a reassigned parameter and a replica
    with its own module dicts (DataParallel's _replicate_for_data_parallel) all resolve to the
    parameters the module holds now."""
    import torch
    from expecto_amd.beluga import Beluga
    m = Beluga()
    p0 = m._params()
    assert p0[0] is m.model[0][0].weight and p0[-1] is m.model[1][4][1].bias
    m.model[0][0] = torch.nn.Conv2d(4, 320, (1, 8))
    assert m._params()[0] is m.model[0][0].weight and m._params()[0] is not p0[0]
    m.model[0][2].bias = torch.nn.Parameter(torch.zeros(320))
    assert m._params()[3] is m.model[0][2].bias
    r = m._replicate_for_data_parallel()
    r._modules["model"] = m.model._replicate_for_data_parallel()
    r.model._modules["0"] = torch.nn.Sequential(*[c for c in m.model[0]])
    r.model[0]._modules["0"] = torch.nn.Conv2d(4, 320, (1, 8))
    assert r._params()[0] is r.model[0][0].weight and r._params()[0] is not m._params()[0]
    assert m._params()[0] is m.model[0][0].weight
