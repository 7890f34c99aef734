"""CPU: the memory-mapped code-genome cache (expecto_amd.genome; the role of pyfasta's
.flat/.gdx, chromatin.py:44, requirements.txt:20) -- byte-identical to the in-memory reader,
rebuilt when stale, shared by concurrent openers, and keeping encodeSeqs' KeyError on
characters it rejects."""
import os
import subprocess
import sys
import types

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _contigs():
    from expecto_amd import synthetic
    g = synthetic.genome_bytes(n_contigs=3, contig_len=50_000, seed=11)
    g["chr2"] = g["chr2"][:700] + b"R" + g["chr2"][701:1500] + b"y" + g["chr2"][1501:]
    g["chrEmpty"] = b""
    g["chrM"] = b"ACGTNacgtnH-"
    return g


def _write_messy(path, g):
    """FASTA with text before the first header, header descriptions, CRLF line ends, uneven
    line widths and blank lines: what the line reader tolerates."""
    with open(path, "wb") as f:
        f.write(b"; a comment line before the first record\n")
        for k, (name, seq) in enumerate(g.items()):
            f.write(b">" + name.encode() + b" description words\r\n")
            w = 50 + 13 * k
            for i in range(0, len(seq), w):
                f.write(seq[i:i + w] + (b"\r\n" if k % 2 else b"\n"))
                if i == 0:
                    f.write(b"\n")


def _same(fa, mem, g):
    from expecto_amd.genome import CodeGenome
    assert list(fa.keys()) == list(g)
    for c in g:
        assert bytes(fa.raw(c)) == g[c]
    a, b = CodeGenome(fa), CodeGenome(mem)
    assert a.codes_path is not None and b.codes_path is None
    assert np.array_equal(np.asarray(a.codes), b.codes)
    assert a.offsets == b.offsets and a.lengths == b.lengths
    assert np.array_equal(a.invalid_offsets, b.invalid_offsets)
    assert bytes(a.invalid_chars) == bytes(b.invalid_chars) == b"Ry"


def test_cache_round_trip_equals_in_memory_reader(tmp_path):
    from expecto_amd import genome
    g = _contigs()
    p = str(tmp_path / "g.fa")
    _write_messy(p, g)
    fa = genome.Fasta(p)
    assert genome.LAST_OPEN["built"]
    for ext in (".flat", ".codes", ".gdx.npz"):
        assert os.path.exists(p + ".expecto" + ext)
    _same(fa, genome.Fasta.from_dict(g), g)
    for f in ({"chr": "chr2", "start": 690, "stop": 720}, {"chr": "chr1", "start": 1, "stop": 3},
              {"chr": "chrM", "start": 5, "stop": 12}):
        want = g[f["chr"]][f["start"] - 1:f["stop"]].decode("latin-1")
        assert fa.sequence(f) == want == genome.Fasta.from_dict(g).sequence(f)
    fa2 = genome.Fasta(p)                      # warm: mapped, not rebuilt
    assert not genome.LAST_OPEN["built"]
    _same(fa2, genome.Fasta.from_dict(g), g)


def test_stale_cache_is_rebuilt(tmp_path):
    from expecto_amd import genome, synthetic
    g = _contigs()
    p = str(tmp_path / "g.fa")
    synthetic.write_fasta(p, g)
    genome.Fasta(p)
    assert genome.LAST_OPEN["built"]
    g2 = dict(g)
    g2["chr1"] = b"T" * 1000 + g["chr1"][1000:]
    g2["chrNew"] = b"GATTACA" * 100
    synthetic.write_fasta(p, g2)
    st = os.stat(p)
    os.utime(p, ns=(st.st_atime_ns, st.st_mtime_ns + 10_000_000))
    fa = genome.Fasta(p)
    assert genome.LAST_OPEN["built"]
    _same(fa, genome.Fasta.from_dict(g2), g2)
    # a damaged cache (codes file truncated) is rebuilt too
    with open(p + ".expecto.codes", "r+b") as f:
        f.truncate(100)
    fa = genome.Fasta(p)
    assert genome.LAST_OPEN["built"]
    _same(fa, genome.Fasta.from_dict(g2), g2)


def test_invalid_base_still_raises_keyerror(tmp_path):
    """encodeSeqs (chromatin.py:166) raises KeyError on characters outside A/C/G/T/N/H/-: the
    cache records them, so a window touching one raises before any device work."""
    from expecto_amd import genome, synthetic
    from expecto_amd.pipeline import VariantPipeline
    g = _contigs()
    p = str(tmp_path / "g.fa")
    synthetic.write_fasta(p, g)
    cg = genome.CodeGenome(genome.Fasta(p))
    pipe = VariantPipeline.__new__(VariantPipeline)
    pipe.dg = types.SimpleNamespace(host=cg)
    near = np.array([cg.offset("chr2", 701 + 500)], np.int64)      # window reaches position 701 ('R')
    with pytest.raises(KeyError) as e:
        pipe._check_window_chars(near, [0])
    assert e.value.args[0] == "R"
    pipe._check_window_chars(np.array([cg.offset("chr1", 20_000)], np.int64), [0, -800, 800])
    far = np.array([cg.offset("chr2", 1501 + 1300)], np.int64)     # only the -800 shift reaches the 'y'
    pipe._check_window_chars(far, [0])
    with pytest.raises(KeyError):
        pipe._check_window_chars(far, [0, -800])


def test_read_only_directory_uses_cache_dir(tmp_path, monkeypatch):
    from expecto_amd import genome, synthetic
    g = _contigs()
    ro = tmp_path / "ro"
    ro.mkdir()
    p = str(ro / "g.fa")
    synthetic.write_fasta(p, g)
    monkeypatch.setattr(os, "access", lambda d, mode: False if os.path.abspath(d) == str(ro) else True)
    monkeypatch.setenv("EXPECTO_CACHE_DIR", str(tmp_path / "cache"))
    fa = genome.Fasta(p)
    assert fa.cache_prefix.startswith(str(tmp_path / "cache"))
    assert not any("expecto" in f for f in os.listdir(ro))
    _same(fa, genome.Fasta.from_dict(g), g)


def test_concurrent_openers_build_once(tmp_path):
    """Four processes open the same FASTA at once (the ranks of one node): the flock lets one
    build the cache; the others wait and map it."""
    from expecto_amd import synthetic
    g = _contigs()
    p = str(tmp_path / "g.fa")
    synthetic.write_fasta(p, g)
    code = ("import sys; sys.path.insert(0, %r); from expecto_amd import genome; "
            "fa = genome.Fasta(%r); cg = genome.CodeGenome(fa); "
            "print(int(genome.LAST_OPEN['built']), int(cg.codes.sum()))" % (REPO, p))
    procs = [subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, text=True) for _ in range(4)]
    outs = [pr.communicate(timeout=120)[0].split() for pr in procs]
    assert all(pr.returncode == 0 for pr in procs)
    assert sum(int(o[0]) for o in outs) == 1, outs
    assert len({o[1] for o in outs}) == 1
