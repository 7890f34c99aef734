"""Stand-in for Bio.SeqIO.parse(path, 'fasta'): records with .id (first header word) and .seq."""


class _Record:
    def __init__(self, rid, seq):
        self.id, self.seq = rid, seq


def parse(handle, fmt):
    assert fmt == "fasta"
    f = open(handle) if isinstance(handle, str) else handle
    rid, parts = None, []
    for line in f:
        if line.startswith(">"):
            if rid is not None:
                yield _Record(rid, "".join(parts))
            rid, parts = (line[1:].split() or [""])[0], []
        elif rid is not None:
            parts.append(line.strip())
    if rid is not None:
        yield _Record(rid, "".join(parts))
