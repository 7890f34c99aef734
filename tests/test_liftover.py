"""Offline hg38 -> hg19 liftover from a UCSC chain file (expecto_amd/liftover.py), against an
explicit per-base expansion of the chain blocks, and the chromatin CLI's --hg38 path
(chromatin.py:120-135,216-229).  Parity against the `liftover` package itself is unpinned
(neither it nor a UCSC chain file is available offline)."""
import gzip

import numpy as np
import pytest

# chr1: + strand chain, blocks [1000,2000)->[500,1500), gap dt=50, [2050,4050)->[1500,3500),
# gap dq=100, [4050,5000)->[3600,4550).  chr2: - strand chain [10000,10300) -> chr5 (- 2000..2300).
CHAIN = """chain 1000 chr1 100000 + 1000 5000 chr1 90000 + 500 4550 1
1000\t50\t0
2000\t0\t100
950

chain 500 chr2 50000 + 10000 10300 chr5 80000 - 2000 2300 2
300

"""
# a second chain over chr1 [1500, 1600): those positions map twice
CHAIN_DUP = CHAIN + """chain 10 chr1 100000 + 1500 1600 chrX 60000 + 700 800 3
100

"""


def _write(tmp_path, text, name="hg38ToHg19.over.chain.gz"):
    p = tmp_path / name
    with gzip.open(p, "wt") as f:
        f.write(text)
    return str(p)


def _expand(text):
    """position -> list of (chrom, pos, strand), from the chain text block by block."""
    m = {}
    t = q = 0
    hdr = None
    for line in text.splitlines():
        w = line.split()
        if not w:
            continue
        if w[0] == "chain":
            hdr = w
            t, q = int(w[5]), int(w[10])
            continue
        size = int(w[0])
        for k in range(size):
            qp = q + k
            if hdr[9] == "-":
                qp = int(hdr[8]) - 1 - qp
            m.setdefault((hdr[2], t + k), []).append((hdr[7], qp, hdr[9]))
        if len(w) == 3:
            t += size + int(w[1])
            q += size + int(w[2])
    return m


@pytest.mark.parametrize("text", [CHAIN, CHAIN_DUP])
def test_chain_lifter_equals_block_expansion(tmp_path, text):
    from expecto_amd.liftover import ChainLifter
    lf = ChainLifter(_write(tmp_path, text))
    want = _expand(text)
    for chrom, lo, hi in (("chr1", 900, 5100), ("chr2", 9990, 10310), ("chr3", 0, 50)):
        for p in range(lo, hi):
            got = lf.convert_coordinate(chrom, p)
            assert sorted(got) == sorted(want.get((chrom, p), [])), (chrom, p, got)
    # the reference passes contigs with or without the "chr" prefix
    assert lf.convert_coordinate("1", 1234) == lf.convert_coordinate("chr1", 1234) == [("chr1", 734, "+")]
    assert lf.convert_coordinate("chr2", 10000) == [("chr5", 80000 - 1 - 2000, "-")]
    assert len(lf.convert_coordinate("chr1", 1550)) == (2 if text is CHAIN_DUP else 1)


def test_get_lifter_resolution(tmp_path, monkeypatch):
    from expecto_amd import liftover
    path = _write(tmp_path, CHAIN)
    monkeypatch.delenv("EXPECTO_CHAIN_FILE", raising=False)
    assert isinstance(liftover.get_lifter("hg38", "hg19", path), liftover.ChainLifter)
    monkeypatch.setenv("EXPECTO_CHAIN_FILE", path)
    assert liftover.get_lifter("hg38", "hg19").convert_coordinate("chr1", 4999) == [("chr1", 4549, "+")]
    monkeypatch.delenv("EXPECTO_CHAIN_FILE")
    try:
        import liftover as _pkg  # noqa: F401
    except ImportError:
        with pytest.raises(RuntimeError, match="chain file"):
            liftover.get_lifter("hg38", "hg19")
    with pytest.raises(FileNotFoundError):
        liftover.get_lifter("hg38", "hg19", str(tmp_path / "missing.chain"))


def test_chromatin_cli_hg38_liftover(tmp_path, capsys):
    """--hg38 --chain-file: lifted rows go on (snps_hg19.vcf keeps the hg19 coordinates), rows in
    chain gaps or off every chain go to not_lifted.vcf; stdout as chromatin.py:218-225."""
    from expecto_amd import chromatin
    path = _write(tmp_path, CHAIN)
    rows = [("chr1", 1234, "rs1", "A", "G"), ("chr1", 2010, "rs2", "C", "T"),   # 2010: in the dt gap
            ("chr2", 10001, "rs3", "G", "A"), ("chr7", 5, "rs4", "T", "C"), ("1", 4100, "rs5", "A", "C")]
    vcf = tmp_path / "in.vcf"
    vcf.write_text("".join("\t".join(map(str, r)) + "\n" for r in rows))
    out = tmp_path / "out"
    out.mkdir()
    args = chromatin.build_parser().parse_args([str(vcf), "--hg38", "--chain-file", path, "--output_dir", str(out)])
    vs = chromatin.read_variants(args)
    printed = capsys.readouterr().out.splitlines()
    assert printed == ["Lifting over to hg38...", "Failed to lift 2 variants from hg38 to hg19"]
    assert list(vs.chrom) == ["chr1", "chr5", "chr1"]
    assert list(vs.pos) == [734, 80000 - 1 - (2000 + 1), 4100 - 4050 + 3600]
    lifted = [l.split("\t") for l in (out / "snps_hg19.vcf").read_text().splitlines() if not l.startswith("#")]
    assert [(l[0], int(l[1])) for l in lifted] == [("chr1", 734), ("chr5", 77998), ("chr1", 3650)]
    failed = [l.split("\t")[2] for l in (out / "not_lifted.vcf").read_text().splitlines()]
    assert failed == ["rs2", "rs4"]
    assert np.array_equal(vs.pos, np.array([734, 77998, 3650]))
