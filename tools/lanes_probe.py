"""Probe: does running two handles on two streams (two variant halves of the headline step
concurrently) fill the partial workgroup rounds of each other's launches?

  python tools/lanes_probe.py [steps]
"""
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from expecto_amd import beluga, synthetic  # noqa: E402
from expecto_amd.genome import DeviceGenome, Fasta  # noqa: E402
from expecto_amd.pipeline import VariantPipeline  # noqa: E402


def timed(fn, steps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda", 0)
    genome = synthetic.genome_bytes(n_contigs=24, contig_len=2_000_000, seed=0)
    fasta = Fasta.from_dict(genome)
    dg = DeviceGenome(fasta, device=dev)
    model = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=bench.MAX_BATCH).cuda()
    params = [p.detach().contiguous() for p in model._params()]
    engs = [beluga.BelugaEngine(params, 0, bench.MAX_BATCH) for _ in range(2)]
    for e in engs:
        e.set_overflow_check(deferred=True)
    pipes = [VariantPipeline(e, fasta, dg) for e in engs]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]

    one96 = bench.Sed200(pipes[0], genome, 96, 202, dev)
    t = timed(one96, steps)
    print(f"1 lane x 96: {t * 1e3:.2f} ms/step  {96 / t:.1f} variants/s", flush=True)
    for n in (48, 96):
        halves = [bench.Sed200(pipes[i], genome, n, 300 + i, dev) for i in range(2)]
        torch.cuda.synchronize()

        def two():
            cur = torch.cuda.current_stream()
            for s, h in zip(streams, halves):
                s.wait_stream(cur)
                with torch.cuda.stream(s):
                    h()
            for s in streams:
                cur.wait_stream(s)

        def seq():
            for h in halves:
                h()

        ts = timed(seq, steps)
        tt = timed(two, steps)
        print(f"2 x {n} sequential: {ts * 1e3:.2f} ms/step {2 * n / ts:.1f} variants/s | "
              f"2 lanes concurrent: {tt * 1e3:.2f} ms/step {2 * n / tt:.1f} variants/s", flush=True)
        # bitwise: concurrent lanes give the sequential outputs
        ya = [h.y.clone() for h in halves]
        seq()
        torch.cuda.synchronize()
        print("  bitwise equal:", all(torch.equal(a, h.y) for a, h in zip(ya, halves)), flush=True)
        del halves
    for e in engs:
        assert not e.overflow_pending()


if __name__ == "__main__":
    main()
