"""Stand-in for liftover (its chain files need the network): no coordinate maps."""


class _Lifter:
    def convert_coordinate(self, chrom, pos):
        return []


def get_lifter(a, b):
    return _Lifter()
