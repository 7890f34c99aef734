"""hg38 -> hg19 coordinate liftover from a UCSC chain file, offline.

The reference calls ``liftover.get_lifter('hg38', 'hg19')`` (PyPI ``liftover==1.1.11``,
requirements.txt:11; used at chromatin.py:50,120-135 and compute_expecto_features.py:45-67),
which downloads ``hg38ToHg19.over.chain.gz`` from UCSC on first use and returns an object whose
``convert_coordinate(chrom, pos)`` gives a list of ``(chrom, pos, strand)``.  Neither the
package nor the chain file can be fetched here, so this module restates the chain-file
algorithm and reads a chain file the user supplies (``--chain-file`` of the CLIs, or
``$EXPECTO_CHAIN_FILE``); the installed package is used only when no chain file is given.

Restated algorithm (UCSC chain format: a header ``chain score tName tSize tStrand tStart tEnd
qName qSize qStrand qStart qEnd id`` then ``size dt dq`` lines and a final ``size``; aligned
blocks are ``[t, t+size) <-> [q, q+size)`` with ``t += size + dt``, ``q += size + dq`` between
blocks): a position ``p`` of the target (the old assembly) inside a block maps to
``q + (p - t)`` on a ``+`` query strand and to ``qSize - 1 - (q + (p - t))`` with strand ``-``
on a ``-`` query strand (``q`` counts on the reverse complement there).  Every chain block that
covers ``p`` yields one result; a position in a gap yields none.  ``pos`` is used as given: the
reference passes the VCF / annotation position straight through, and the block arithmetic
preserves it (``p - t + q``).  Chromosome names are matched as given, then with the ``chr``
prefix added or removed; results carry the chain file's query names.

Parity: unpinned (neither ``liftover`` nor a UCSC chain file is available offline); tested on
synthetic chain files against an explicit per-base expansion of their blocks
(tests/test_liftover.py).
"""
from __future__ import annotations

import gzip
import os

import numpy as np


class ChainLifter:
    """``convert_coordinate(chrom, pos)`` over the blocks of one chain file."""

    def __init__(self, path: str):
        opener = gzip.open if path.endswith(".gz") else open
        per_chrom: dict[str, list] = {}
        self.q_names: list[str] = []
        self.q_sizes: list[int] = []
        self.q_minus: list[bool] = []
        t_name = None
        t = q = 0
        chain = -1
        with opener(path, "rt") as f:
            for line in f:
                w = line.split()
                if not w:
                    continue
                if w[0] == "chain":
                    if len(w) < 12:
                        raise ValueError(f"{path}: malformed chain header: {line.strip()}")
                    t_name, t_strand = w[2], w[4]
                    if t_strand != "+":
                        raise ValueError(f"{path}: target strand must be '+' (UCSC chains): {line.strip()}")
                    t, q = int(w[5]), int(w[10])
                    self.q_names.append(w[7])
                    self.q_sizes.append(int(w[8]))
                    self.q_minus.append(w[9] == "-")
                    chain += 1
                    continue
                if t_name is None:
                    raise ValueError(f"{path}: alignment line before any chain header")
                size = int(w[0])
                per_chrom.setdefault(t_name, []).append((t, t + size, q, chain))
                if len(w) >= 3:
                    t += size + int(w[1])
                    q += size + int(w[2])
        self._tab = {}
        for name, blocks in per_chrom.items():
            a = np.array(sorted(blocks), np.int64).reshape(-1, 4)
            self._tab[name] = (a[:, 0], a[:, 1], a[:, 2], a[:, 3], int((a[:, 1] - a[:, 0]).max()))

    def _chrom(self, chrom: str):
        chrom = str(chrom)
        for c in (chrom, "chr" + chrom, chrom[3:] if chrom.startswith("chr") else None):
            if c is not None and c in self._tab:
                return self._tab[c]
        return None

    def convert_coordinate(self, chrom, pos, strand: str = "+"):
        tab = self._chrom(chrom)
        if tab is None:
            return []
        ts, te, qs, ch, maxlen = tab
        p = int(pos)
        out = []
        i = int(np.searchsorted(ts, p, side="right")) - 1
        while i >= 0 and ts[i] > p - maxlen - 1:
            if ts[i] <= p < te[i]:
                c = int(ch[i])
                off = int(qs[i]) + (p - int(ts[i]))
                if self.q_minus[c]:
                    out.append((self.q_names[c], self.q_sizes[c] - 1 - off, "-" if strand == "+" else "+"))
                else:
                    out.append((self.q_names[c], off, strand))
            i -= 1
        return out[::-1]


def get_lifter(target: str = "hg38", query: str = "hg19", chain_file: str | None = None):
    """The reference's ``get_lifter(target, query)``: a chain file given here or in
    $EXPECTO_CHAIN_FILE, else the installed ``liftover`` package (which downloads the UCSC
    chain), else a RuntimeError naming both options."""
    path = chain_file or os.environ.get("EXPECTO_CHAIN_FILE")
    if path:
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        return ChainLifter(path)
    try:
        from liftover import get_lifter as _pkg_get_lifter
    except ImportError as e:
        raise RuntimeError(f"{target} -> {query} liftover needs a UCSC chain file (--chain-file or "
                           f"$EXPECTO_CHAIN_FILE, e.g. {target}To{query.capitalize()}.over.chain.gz) or the "
                           "`liftover` package (it downloads the chain; no network here)") from e
    return _pkg_get_lifter(target, query)
