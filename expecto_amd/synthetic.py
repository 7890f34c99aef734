"""Seeded synthetic genome, variants and genes (SURVEY.md 8d "Synthetic inputs").

There is no network for hg19 or the real VCFs, so benchmarks and tests use:

* a genome of ``n_contigs`` contigs named ``chr1..``: i.i.d. A/C/G/T with 10 %
  lowercase and 1 % N (``numpy.random.default_rng(seed)``), optionally repeat-rich
  (``repeats=True``: about half the sequence in hg19-like low-complexity elements --
  homopolymer runs, di/tri/hexa-nucleotide tandem repeats, tandem copies of 300-bp blocks,
  copies of an interspersed ~300-bp family consensus, long N gaps -- soft-masked);
* biallelic SNVs uniform in ``[margin, len - margin]`` with ref = the genome base
  (upper case) and alt uniform over the other three bases;
* variant->TSS distances uniform over [-20000, 20000] and a random strand.
"""
from __future__ import annotations

import numpy as np

_BASES = np.frombuffer(b"ACGT", np.uint8)


def genome_bytes(n_contigs: int = 24, contig_len: int = 2_000_000, seed: int = 0, repeats: bool = False) -> dict:
    """name -> bytes of the contig sequence (ASCII)."""
    rng = np.random.default_rng(seed)
    out = {}
    for i in range(n_contigs):
        s = _BASES[rng.integers(0, 4, contig_len)]
        low = rng.random(contig_len) < 0.10
        s = np.where(low, s + 32, s).astype(np.uint8)            # lowercase
        nmask = rng.random(contig_len) < 0.01
        s = np.where(nmask, np.uint8(ord("N")), s).astype(np.uint8)
        if repeats:
            add_repeats(s, np.random.default_rng([seed, i, 1]))
        out[f"chr{i + 1}"] = s.tobytes()
    return out


_MOTIFS = [b"A", b"T", b"G", b"C", b"CA", b"TG", b"AT", b"GC", b"CAG", b"CGG", b"GAA", b"CTG", b"GGGGCC", b"TTAGGG"]


def add_repeats(s: np.ndarray, rng, cover: float = 0.5, gap_every: int = 1_000_000) -> np.ndarray:
    """Overwrite about `cover` of the uint8 ASCII sequence `s` in place with low-complexity
    elements (hg19 is ~50 % repeats): homopolymer runs (10-300 bp), di/tri/hexa-nucleotide
    tandem repeats (20-900 bp), 2-5 tandem copies of a 300-bp block of the sequence itself,
    copies of one seeded ~300-bp interspersed family consensus with 10 % point changes, all
    soft-masked (lowercase); plus one N gap (1-20 kb) per `gap_every` bases."""
    n = s.size
    family = _BASES[rng.integers(0, 4, 300)]
    done = 0
    while done < cover * n:
        kind = rng.integers(0, 4)
        p = int(rng.integers(0, n))
        if kind == 0:                                   # tandem repeat of a short motif
            m = np.frombuffer(_MOTIFS[int(rng.integers(0, len(_MOTIFS)))], np.uint8)
            ln = int(rng.integers(10, 300)) if m.size == 1 else int(rng.integers(20, 900))
            el = np.resize(m, ln)
        elif kind == 1:                                 # tandem copies of a 300-bp block
            blk = s[p:p + 300].copy()
            el = np.tile(blk, int(rng.integers(2, 6)))
        else:                                           # interspersed family copy (Alu-like)
            el = family.copy()
            mut = rng.random(el.size) < 0.10
            el[mut] = _BASES[rng.integers(0, 4, int(mut.sum()))]
            el = el[:int(rng.integers(150, 301))]
        el = el[:max(0, n - p)]
        s[p:p + el.size] = np.where(np.isin(el, _BASES), el + 32, el)    # soft-masked
        done += el.size
    for g in range(max(1, n // gap_every)):
        p, ln = int(rng.integers(0, n)), int(rng.integers(1000, 20000))
        s[p:p + ln] = ord("N")
    return s


def write_fasta(path: str, genome: dict, width: int = 60) -> None:
    with open(path, "wb") as f:
        for name, seq in genome.items():
            f.write(b">" + name.encode() + b"\n")
            for i in range(0, len(seq), width):
                f.write(seq[i:i + width] + b"\n")


HG19_LENGTHS = {   # hg19 chr1..chr22, chrX, chrY (3,095,677,412 bp): the size of the real genome
    "chr1": 249250621, "chr2": 243199373, "chr3": 198022430, "chr4": 191154276, "chr5": 180915260,
    "chr6": 171115067, "chr7": 159138663, "chr8": 146364022, "chr9": 141213431, "chr10": 135534747,
    "chr11": 135006516, "chr12": 133851895, "chr13": 115169878, "chr14": 107349540, "chr15": 102531392,
    "chr16": 90354753, "chr17": 81195210, "chr18": 78077248, "chr19": 59128983, "chr20": 63025520,
    "chr21": 48129895, "chr22": 51304566, "chrX": 155270560, "chrY": 59373566}


class TiledGenome:
    """A genome of hg19's size written fast: every contig is a line-aligned rotation of one
    seeded ``block`` of bases (i.i.d. A/C/G/T, 10 % lowercase, 1 % N), so a multi-GB FASTA
    costs one block of random numbers and the file write.  ``base(chrom, pos1)`` gives the
    base at a 1-based position (for SNVs whose ref matches the genome)."""

    def __init__(self, lengths: dict | None = None, block_lines: int = 1 << 18, width: int = 60, seed: int = 0):
        rng = np.random.default_rng(seed)
        nb = block_lines * width
        s = _BASES[rng.integers(0, 4, nb)]
        s = np.where(rng.random(nb) < 0.10, s + 32, s).astype(np.uint8)
        s = np.where(rng.random(nb) < 0.01, np.uint8(ord("N")), s).astype(np.uint8)
        self.block, self.width, self.block_lines = s, width, block_lines
        self.lengths = dict(HG19_LENGTHS if lengths is None else lengths)
        # contig k starts at line (k * 7919) % block_lines of the block
        self.start = {c: (k * 7919) % block_lines for k, c in enumerate(self.lengths)}

    def base(self, chrom: str, pos1: int) -> int:
        return int(self.block[(self.start[chrom] * self.width + pos1 - 1) % self.block.size])

    def write_fasta(self, path: str, lines_per_write: int = 1 << 20) -> int:
        """Write the FASTA; returns its size in bytes."""
        w, nl = self.width, self.block_lines
        lines = np.concatenate([self.block.reshape(nl, w), np.full((nl, 1), ord("\n"), np.uint8)], 1)
        with open(path, "wb") as f:
            for c, ln in self.lengths.items():
                f.write(b">" + c.encode() + b"\n")
                full, tail = divmod(ln, w)
                for a in range(0, full, lines_per_write):
                    idx = (self.start[c] + np.arange(a, min(full, a + lines_per_write))) % nl
                    f.write(lines[idx].tobytes())
                if tail:
                    row = lines[(self.start[c] + full) % nl]
                    f.write(row[:tail].tobytes() + b"\n")
            return f.tell()

    def snvs(self, n: int, seed: int = 1, margin: int = 5000):
        """(chrom, pos, ref, alt) SNVs with ref = the genome base (upper case), as ``snvs``."""
        rng = np.random.default_rng(seed)
        names = list(self.lengths)
        out = []
        while len(out) < n:
            chrom = names[int(rng.integers(0, len(names)))]
            pos = int(rng.integers(margin, self.lengths[chrom] - margin))
            ref = chr(self.base(chrom, pos)).upper()
            if ref not in "ACGT":
                continue
            out.append((chrom, pos, ref, "ACGT".replace(ref, "")[int(rng.integers(0, 3))]))
        return out


def snvs(genome: dict, n: int, seed: int = 1, margin: int = 5000):
    """List of (chrom, pos(1-based), ref, alt) biallelic SNVs."""
    rng = np.random.default_rng(seed)
    names = list(genome)
    out = []
    while len(out) < n:
        chrom = names[int(rng.integers(0, len(names)))]
        seq = genome[chrom]
        pos = int(rng.integers(margin, len(seq) - margin))
        ref = chr(seq[pos - 1]).upper()
        if ref not in "ACGT":
            continue
        alt = "ACGT".replace(ref, "")[int(rng.integers(0, 3))]
        out.append((chrom, pos, ref, alt))
    return out


def tss_dists(n: int, seed: int = 2):
    """Distances pos - TSS uniform over [-20000, 20000] and TSS strands (+/-)."""
    rng = np.random.default_rng(seed)
    return rng.integers(-20000, 20001, n), np.where(rng.random(n) < 0.5, "+", "-")
