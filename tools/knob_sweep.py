"""A/B sweep of handle knobs (read at handle creation) on the bench workloads, one process.

    python tools/knob_sweep.py EXPECTO_FC2_SPLITS=7,3,9 [EXPECTO_CONV_TILE=0,256] [--steps 5]

For every setting: a fresh handle, the headline 200-window workload (96 variants/step) and
configs[1] (1000 SNVs, shift 0), timed like bench.py (profiling off, per-step release point),
rounds interleaved so clock drift hits every setting alike.  Prints one JSON line per setting.
"""
import itertools
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402
from expecto_amd import beluga, synthetic  # noqa: E402
from expecto_amd.genome import DeviceGenome, Fasta  # noqa: E402
from expecto_amd.pipeline import VariantPipeline, shift_order  # noqa: E402


def main():
    knobs, steps, rounds = [], 5, 3
    args = sys.argv[1:]
    i = 0
    while i < len(args):
        if args[i] == "--steps":
            steps = int(args[i + 1])
            i += 2
            continue
        if args[i] == "--rounds":
            rounds = int(args[i + 1])
            i += 2
            continue
        k, v = args[i].split("=")
        knobs.append([(k, x) for x in v.split(",")])
        i += 1
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    genome = synthetic.genome_bytes(n_contigs=24, contig_len=2_000_000, seed=0, repeats=True)   # = bench.py
    fasta = Fasta.from_dict(genome)
    dg = DeviceGenome(fasta, device=dev)
    settings = list(itertools.product(*knobs)) if knobs else [()]
    res = {s: {"sed200": [], "cfg1": []} for s in settings}
    for r in range(rounds):
        for s in (settings if r % 2 == 0 else settings[::-1]):   # alternate order: drift hits all alike
            for k, v in s:
                os.environ[k] = v
            model = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=bench.MAX_BATCH).cuda()
            eng = model.engine()
            eng.set_overflow_check(True)
            pipe = VariantPipeline(eng, fasta, dg)
            head = bench.Sed200(pipe, genome, bench.N200, 202, dev)
            el, _ = bench.time_steps(head, eng, steps, 1, 1, dev)
            res[s]["sed200"].append(bench.N200 * steps / el)
            c1 = bench.ShiftSweep(pipe, genome, 1000, 1, shift_order(0), dev)
            el, _ = bench.time_steps(c1, eng, steps * 2, 2, 1, dev)
            res[s]["cfg1"].append(1000 * steps * 2 / el)
            del head, c1, pipe, eng, model
            torch.cuda.empty_cache()
            for k, v in s:
                os.environ.pop(k, None)
    for s in settings:
        out = {"setting": dict(s)}
        for w, vals in res[s].items():
            vals = sorted(vals)
            out[w] = {"median": vals[len(vals) // 2], "all": vals}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
