"""Seeded synthetic genome, variants and genes (SURVEY.md 8d "Synthetic inputs").

There is no network for hg19 or the real VCFs, so benchmarks and tests use:

* a genome of ``n_contigs`` contigs named ``chr1..``: i.i.d. A/C/G/T with 10 %
  lowercase and 1 % N (``numpy.random.default_rng(seed)``);
* biallelic SNVs uniform in ``[margin, len - margin]`` with ref = the genome base
  (upper case) and alt uniform over the other three bases;
* variant->TSS distances uniform over [-20000, 20000] and a random strand.
"""
from __future__ import annotations

import numpy as np

_BASES = np.frombuffer(b"ACGT", np.uint8)


def genome_bytes(n_contigs: int = 24, contig_len: int = 2_000_000, seed: int = 0) -> dict:
    """name -> bytes of the contig sequence (ASCII)."""
    rng = np.random.default_rng(seed)
    out = {}
    for i in range(n_contigs):
        s = _BASES[rng.integers(0, 4, contig_len)]
        low = rng.random(contig_len) < 0.10
        s = np.where(low, s + 32, s).astype(np.uint8)            # lowercase
        nmask = rng.random(contig_len) < 0.01
        s = np.where(nmask, np.uint8(ord("N")), s).astype(np.uint8)
        out[f"chr{i + 1}"] = s.tobytes()
    return out


def write_fasta(path: str, genome: dict, width: int = 60) -> None:
    with open(path, "wb") as f:
        for name, seq in genome.items():
            f.write(b">" + name.encode() + b"\n")
            for i in range(0, len(seq), width):
                f.write(seq[i:i + width] + b"\n")


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
