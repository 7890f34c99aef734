"""Stand-in for pyfasta (absent offline) used ONLY to run the reference scripts when
generating golden vectors.  ``Fasta(path).sequence({'chr','start','stop'})`` returns the
1-based inclusive slice, as pyfasta==0.5.2 does for in-range windows."""


class Fasta:
    def __init__(self, path):
        self._seqs, name, buf = {}, None, []
        with open(path) as f:
            for line in f:
                line = line.rstrip("\n")
                if line.startswith(">"):
                    if name is not None:
                        self._seqs[name] = "".join(buf)
                    name, buf = line[1:].split()[0], []
                else:
                    buf.append(line)
        if name is not None:
            self._seqs[name] = "".join(buf)

    def keys(self):
        return self._seqs.keys()

    def sequence(self, f, one_based=True):
        start = f["start"] - 1 if one_based else f["start"]
        if start < 0:
            raise ValueError("window before contig start (pyfasta edge behaviour is unpinned)")
        return self._seqs[f["chr"]][start:f["stop"]]
