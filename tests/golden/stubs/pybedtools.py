"""Stand-in for pybedtools (absent offline) used ONLY to run the reference scripts for golden
vectors: BedTool from a file or a whitespace-separated string; ``a.intersect(b)`` yields, for
every pair of overlapping intervals (half-open BED), the overlapping part of the a-interval as
(chrom, start, end) string triples -- bedtools intersect's default output."""


class BedTool:
    def __init__(self, src, from_string=False):
        text = src if from_string else open(src).read()
        self.iv = []
        for line in text.splitlines():
            f = line.split()
            if len(f) >= 3 and not line.startswith("#"):
                self.iv.append((f[0], int(f[1]), int(f[2])))

    def intersect(self, other):
        out = []
        for c, s, e in self.iv:
            for c2, s2, e2 in other.iv:
                if c == c2 and s2 < e and e2 > s:
                    out.append((c, str(max(s, s2)), str(min(e, e2))))
        return _Result(out)


class _Result(list):
    pass
