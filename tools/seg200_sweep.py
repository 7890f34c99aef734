"""Sweep handle max_batch and variants per step for the 200-window-per-variant workload
(bench.py extras "variant_200_windows"); prints variants/s per setting."""
import math
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from expecto_amd import beluga, synthetic  # noqa: E402
from expecto_amd.genome import DeviceGenome, Fasta  # noqa: E402
from expecto_amd.pipeline import VariantPipeline  # noqa: E402

dev = torch.device("cuda:0")
genome = synthetic.genome_bytes(n_contigs=24, contig_len=2_000_000, seed=0)
fasta = Fasta.from_dict(genome)
dg = DeviceGenome(fasta, device=dev)
sh200 = list(range(-20000, 20000, 200))
for mb in [int(x) for x in sys.argv[1].split(",")]:
    eng = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=mb).cuda().engine()
    pipe = VariantPipeline(eng, fasta, dg)
    for n in [int(x) for x in sys.argv[2].split(",")]:
        v = bench.make_variants(genome, n, 202)
        p = pipe.prepare(v, sh200)
        el, _ = bench.time_workload(pipe, eng, p, sh200, n, 2, 1, dev, 1)
        print(f"max_batch {mb} variants {n}: {n * 2 / el:.1f} variants/s", flush=True)
    del eng, pipe
    torch.cuda.empty_cache()
