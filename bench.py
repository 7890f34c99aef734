"""Benchmark of the ExPecto hot path on MI355X (contract: see task / DESIGN.md "Measurement").

Workload (BASELINE.json configs[1], per GPU): 1k synthetic biallelic SNVs, shift 0, ref+alt
alleles x fwd+rc strands = 4000 Beluga windows per step.  One step = device window
generation from the HBM-resident genome (expecto_variant_windows) + the Beluga forward over
all 4000 windows (conv1 .. fc2+sigmoid, fp32 in/out) + diff = alt - ref: exactly the device work of
one chromatin.py shift for 1k variants, inputs already resident in HBM.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

N>1: weak scaling, each rank its own 1k SNVs, no collective in the step (variants are
independent; the RCCL gather belongs to file output and is timed after the steps as
"final_gather").  Rank 0 prints ONE JSON line.

The "f16x3" arithmetic computes fp32 products from 22-bit fp16 planes (DTYPES below).
N=1 extras, outside `value`: configs[2] (+-800 sweep), the 200-window variant unit,
configs[4] TSS genes, the other two precisions, the HBM-bound reductions in GB/s, and the
CPU port timed on host cores (16 and 8 threads).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from expecto_amd import beluga, dist as edist, synthetic  # noqa: E402
from expecto_amd.genome import DeviceGenome, Fasta  # noqa: E402
from expecto_amd.pipeline import VariantPipeline, VariantSet  # noqa: E402

METRIC = json.load(open(os.path.join(REPO, "BASELINE.json")))["metric"]
FP32_MFMA_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak
# bf16 dense MFMA peak: 256 CU x 4 SIMD x 1024 FLOP/clk (v_mfma_f32_32x32x16_bf16: 32768 FLOP
# per 32 cycles) x 2.4 GHz = 2516.6 TFLOP/s (MI355X_MICROARCH.md "~2.5 PF dense")
BF16_MFMA_PEAK_TFLOPS = 256 * 4 * 1024 * 2.4e9 / 1e12
HBM_PEAK_GBS = 8000.0             # MI355X_MICROARCH.md: HBM3E ~8 TB/s
BF16X6_PRODUCTS = 6               # bf16 MFMA products per fp32 multiply-add in the bf16x6 kernel
F16X3_PRODUCTS = 3                # fp16 MFMA products per multiply-add in the f16x3 kernel (fp16 peak = bf16 peak)

# per-window dense MACs of each layer, for the roofline of each kernel
LAYER_MACS = {
    "conv1": 1993 * 320 * 32, "conv2": 1986 * 320 * 2560, "conv3": 489 * 480 * 2560,
    "conv4": 482 * 480 * 3840, "conv5": 113 * 640 * 3840, "conv6": 106 * 640 * 5120,
    "fc1": 67840 * 2003, "fc1_reduce": 0, "fc2": 2003 * 2002,
}
GEMM_LAYER_EPI = {"conv2": (2, 1), "conv3": (3, 0), "conv4": (4, 1), "conv5": (5, 0), "conv6": (6, 0),
                  "fc1": (7, 3), "fc2": (8, 3)}


DTYPES = {
    "bf16x6": "fp32 (bf16x6: exact 3-way bf16 split, 6 MFMA products, fp32 accumulate)",
    "f16x3": "fp32 in/out (f16x3: power-of-2-scaled 2-way fp16 split = 22-bit operands, 3 MFMA products, "
             "fp32 accumulate; bf16x6 recompute on fp16 overflow)",
    "fp32": "fp32",
}


def kernel_name(layer: str, precision: str) -> str:
    """rocprofv3 kernel name of a layer's launch (per-window path)."""
    if layer not in GEMM_LAYER_EPI:
        return {"conv1": "beluga_conv1", "fc1_reduce": "fc1_reduce"}[layer]
    l, e = GEMM_LAYER_EPI[layer]
    if precision == "bf16x6":
        return f"beluga_gemm_x6q<{l}, {e}, 0>"
    if precision == "f16x3":
        if l in (7, 8):
            return f"beluga_fc_h3p<{l}, {e}, 0, 3>"
        if l == 2:   # conv2: 384-row tiles (the other conv layers: producer/consumer 256-row tiles)
            return f"beluga_conv_h3r<{l}, {e}, 0>"
        return f"beluga_conv_h3p<{l}, {e}, 0, 3>"
    return f"beluga_gemm<{l}, {e}, 4, 2, 32, 1>"
WINDOW_MACS = sum(LAYER_MACS.values())


def cpu_baseline(sd_cpu, codes: np.ndarray, seconds: float, threads: int, windows_per_variant: int):
    """Oracle torch-CPU forward (the reference's CPU arithmetic) on a bounded sample."""
    from oracle.beluga_np import forward_torch_cpu
    from expecto_amd.encode import codes_to_onehot

    torch.set_num_threads(threads)
    x = torch.from_numpy(codes_to_onehot(codes[:32], with_rc=False).astype(np.float32)).unsqueeze(2)
    forward_torch_cpu(sd_cpu, x[:4])                     # warm-up
    done, t0 = 0, time.perf_counter()
    while True:
        forward_torch_cpu(sd_cpu, x)
        done += x.shape[0]
        el = time.perf_counter() - t0
        if el >= seconds or el >= 30.0:
            break
    wps = done / el
    return {"value": wps / windows_per_variant, "unit": "variants/s", "cores": threads, "kind": "port",
            "windows_per_s": wps,
            "sample": f"{done} windows of the same workload (seeded SNV ref windows), batch 32, "
                      f"oracle/beluga_np.forward_torch_cpu (torch CPU fp32, oneDNN), {el:.1f} s"}


# Handle workspace (windows per launch chunk): 8192 lets the segment path put ~40 variants'
# 200-window segments in one chunk (tools/seg200_sweep.py: 4000 -> 8192 windows and 24 -> 96
# variants per step take the 200-window workload from 799 to 881 variants/s); the headline's
# 4000 windows stay one chunk either way.
MAX_BATCH = 8192
N200 = 96


def hbm_reductions(dev):
    """The metric's "HBM GB/s vs peak": the HBM-bound spatial reductions timed
    with HIP events on synthetic inputs resident in HBM; algorithmic bytes = every input read
    once + every output written once.
      TSS (compute_expecto_features.py:91-124): 1000 genes x 200 shifts x 2002, fwd + rc fp32 ->
        [1000, 20020] fp64 (3.2 MB read + 160 KB written per gene);
      variant (predict.py:87-136): 20000 variants x 9 shifts x 2002 fp32 -> [20000, 20020] fp64
        (write-dominated: "fp64_fill_ceiling" times torch's zero_ of the same output, the
        practical write rate on this box)."""
    from expecto_amd import features
    g = torch.Generator(device=dev).manual_seed(3)
    res = {}
    G, S, F = 1000, 200, 2002
    fwd = torch.rand((G, S, F), device=dev, generator=g)
    rc = torch.rand((G, S, F), device=dev, generator=g)
    w = torch.from_numpy(features.tss_pos_weights()).to(dev)
    out = torch.empty((G, 10 * F), dtype=torch.float64, device=dev)
    n_var, S9 = 20000, 9
    eff = torch.rand((S9, n_var, F), device=dev, generator=g)
    rng = np.random.default_rng(4)
    dist = rng.integers(-20000, 20000, n_var)
    plus = rng.integers(0, 2, n_var).astype(bool)
    from expecto_amd.pipeline import shift_order
    sh = shift_order(800)
    vout = torch.empty((n_var, 10 * F), dtype=torch.float64, device=dev)
    for name, fn, nbytes in (
            ("fp64_fill_ceiling", lambda: vout.zero_(), n_var * 10 * F * 8),   # write-only reference
            ("tss_reduce", lambda: features.tss_reduce(fwd, rc, w, out), 2 * G * S * F * 4 + G * 10 * F * 8),
            ("variant_reduce", lambda: features.variant_features(eff, dist, plus, sh, vout),
             S9 * n_var * F * 4 + n_var * 10 * F * 8)):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        gbs = nbytes / (ms * 1e-3) / 1e9
        res[name] = {"ms": ms, "bytes": nbytes, "GB_per_s": gbs, "peak_GB_per_s": HBM_PEAK_GBS,
                     "frac": gbs / HBM_PEAK_GBS}
    del fwd, rc, eff, out, vout
    torch.cuda.empty_cache()
    return res


def tss_workload(eng, genome, dg, dev, genes=96, steps=2):
    """configs[4]'s per-GPU work (compute_expecto_features.py:88-128): per gene, 200 windows
    x fwd/rc through the segment path, then the 10 x 200 exp-decay reduction to 20020 f64
    features; seeded TSS positions and strands on the synthetic genome."""
    from expecto_amd.tss import TSSPipeline
    rng = np.random.default_rng(55)
    names = sorted(genome)
    chroms = [names[i] for i in rng.integers(0, len(names), genes)]
    tss = [int(rng.integers(30000, len(genome[c]) - 30000)) for c in chroms]
    strands = rng.choice([-1, 1], genes)
    pipe = TSSPipeline(eng, dg)
    pipe.features(chroms, tss, strands)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        pipe.features(chroms, tss, strands)
    e1.record()
    torch.cuda.synchronize()
    el = e0.elapsed_time(e1) * 1e-3
    gps = genes * steps / el
    return {"genes_per_s": gps, "genes_per_step": genes, "windows_per_gene": 400,
            "dense_windows_per_s": gps * 400, "ms_per_step": el / steps * 1e3,
            "projected_20k_genes_s_1gpu": 20000 / gps, "projected_20k_genes_s_8gpu_weak": 20000 / gps / 8}


def time_final_gather(S, n, dev, rank, world):
    """configs[3]'s exchange step, outside the timed steps: one step's outputs of every rank
    (y [2, 2, S, n, 2002] and diff [2, S, n, 2002] fp32) gathered to rank 0 per shift, as the
    chromatin CLI does before rank 0 writes the .diff.h5 files (RCCL gather over xGMI)."""
    y = torch.rand((2, 2, S, n, 2002), device=dev)
    d = torch.rand((2, S, n, 2002), device=dev)
    total = world * n

    def gather():
        for j in range(S):
            edist.gather_rows_to(y[:, :, j:j + 1], 3, total, world, rank)
            edist.gather_rows_to(d[:, j:j + 1], 2, total, world, rank)

    gather()                                   # warm the communicator
    torch.cuda.synchronize()
    torch.distributed.barrier()
    t0 = time.perf_counter()
    gather()
    torch.cuda.synchronize()
    torch.distributed.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if torch.distributed.get_backend() == "nccl":
        el = el.to(dev)
    torch.distributed.all_reduce(el, op=torch.distributed.ReduceOp.MAX)
    nbytes = (world - 1) * (y.numel() + d.numel()) * 4        # bytes arriving at rank 0
    ms = float(el.item()) * 1e3
    return {"ms": ms, "bytes_into_rank0": nbytes, "GB_per_s": nbytes / (ms * 1e-3) / 1e9,
            "what": "one step's y + diff of every rank to rank 0, per shift (not part of value)"}


def make_variants(genome, n, seed):
    snvs = synthetic.snvs(genome, n, seed=seed)
    return VariantSet([v[0] for v in snvs], np.array([v[1] for v in snvs]), [v[2] for v in snvs],
                      [v[3] for v in snvs])


def time_workload(pipe, eng, prep, shifts, n, steps, warmup, dev, world):
    """Time `steps` steps (window generation + forward + diff) with HIP-event layer timing."""
    S = len(shifts)
    y = torch.empty((2, 2, S, n, 2002), dtype=torch.float32, device=dev)

    def step():
        pipe.predict(prep, out=y)
        return pipe.diff(y)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    eng.set_profiling(True)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    el = time.perf_counter() - t0
    layers = eng.layer_times()
    eng.set_profiling(False)
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        el = float(t.item())
    return el, layers


def roofline(layers, precision):
    """MFMA roofline of the dominant GEMM kernel from executed work per launch (library counts)
    and its average launch duration (HIP events on the launch stream)."""
    dom = max((k for k in GEMM_LAYER_EPI), key=lambda k: layers[k][0])
    ms, calls, macs = layers[dom]
    fp32_flops_launch = 2.0 * macs / calls
    fp32_tflops = fp32_flops_launch / (ms / calls / 1e3) / 1e12
    if precision == "bf16x6":
        mult, peak = BF16X6_PRODUCTS, BF16_MFMA_PEAK_TFLOPS
    elif precision == "f16x3":
        mult, peak = F16X3_PRODUCTS, BF16_MFMA_PEAK_TFLOPS
    else:
        mult, peak = 1, FP32_MFMA_PEAK_TFLOPS
    achieved = mult * fp32_tflops
    return {"bound": "mfma", "kernel": kernel_name(dom, precision), "layer": dom, "achieved": achieved,
            "peak": peak, "unit": "TFLOP/s", "frac": achieved / peak, "traffic": None,
            "avg_launch_ms": ms / calls, "launches": calls, "mfma_flops_per_launch": mult * fp32_flops_launch,
            "fp32_flops_per_launch": fp32_flops_launch, "fp32_tflops": fp32_tflops, "precision": precision}


def pmc_traffic(key, kernel):
    """HBM bytes per launch of ``kernel`` from the newest committed rocprofv3 --pmc summary
    (profiles/<tag>/traffic.json, written by tools/collect_profiles.py from FETCH_SIZE and
    WRITE_SIZE passes of this same bench command).  None unless that profile was taken on the
    same workload key (variants, shifts, precision, max_batch): PMC counters cannot be read
    live next to the HIP-event timing."""
    import glob
    for path in sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r*",
                                              "traffic.json")), reverse=True):
        try:
            t = json.load(open(path))
        except (OSError, ValueError):
            continue
        if t.get("profile_key") != key:
            continue
        for name, v in t["kernels"].items():
            if kernel in name:
                return v["hbm_bytes"], t["source"]
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--variants", type=int, default=1000, help="SNVs per GPU per step")
    ap.add_argument("--maxshift", type=int, default=0, help="0 = configs[1] (shift 0 only)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the cfg3 / 200-window extra workloads")
    ap.add_argument("--precision", default=None, help="GEMM arithmetic (default: the engine default)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) for the scaling runs; gloo to "
                    "rehearse several ranks on one GPU")
    args = ap.parse_args()

    rank, world, local = edist.init(args.dist_backend)
    # one rank per GPU; a rehearsal on fewer GPUs than ranks (--dist-backend gloo) shares them
    local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    from expecto_amd.pipeline import shift_order
    shifts = shift_order(args.maxshift)
    S, n = len(shifts), args.variants
    rows = 4 * S * n

    genome = synthetic.genome_bytes(n_contigs=24, contig_len=2_000_000, seed=0)
    fasta = Fasta.from_dict(genome)
    vs = make_variants(genome, n, 1 + rank)
    model = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=MAX_BATCH)
    sd_cpu = {k: v.detach().clone() for k, v in model.state_dict().items()} if (rank == 0 and world == 1) else None
    model = model.cuda()
    eng = model.engine()
    if args.precision:
        eng.set_precision(args.precision)
    pipe = VariantPipeline(eng, fasta, DeviceGenome(fasta, device=dev))
    prep = pipe.prepare(vs, shifts)                          # variant table resident in HBM

    el, layers = time_workload(pipe, eng, prep, shifts, n, args.steps, args.warmup, dev, world)
    total_rows = rows * args.steps
    value = world * n * args.steps / el
    exec_macs = sum(m for _, _, m in layers.values())
    key = {"variants": n, "shifts": shifts, "precision": eng.precision, "max_batch": MAX_BATCH}
    roof = roofline(layers, eng.precision)
    roof["traffic"], src = pmc_traffic(key, roof["kernel"])
    if roof["traffic"] is not None:
        roof["traffic_unit"] = "bytes/launch (HBM read+write)"
        roof["traffic_source"] = src
    rec = {
        "metric": METRIC, "value": value, "unit": "variants/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None,
        "dtype": DTYPES[eng.precision],
        "data": "synthetic: seeded genome (24 x 2 Mbp), seeded SNVs, seeded Beluga weights x sqrt(6)",
        "config": {"workload": f"configs[1]: {n} SNVs/GPU, shifts {shifts}, ref+alt x fwd+rc = "
                               f"{rows} Beluga windows/step/GPU (window gen + forward + diff)",
                   "variants_per_gpu": n, "windows_per_variant": 4 * S, "parallelism": f"dp{world} (variant shards)"},
        "windows_per_s": world * total_rows / el,
        "dense_equivalent_tflops": 2.0 * WINDOW_MACS * world * total_rows / el / 1e12,
        "executed_fp32_tflops": 2.0 * exec_macs * world / el / 1e12,
        "roofline": roof,
        "layer_ms_per_step": {k: ms / args.steps for k, (ms, c, m) in layers.items()},
        "layer_tflops": {k: 2.0 * m / (ms * 1e-3) / 1e12 for k, (ms, c, m) in layers.items() if ms > 0},
        "profile_key": key,
        "reuse": "alt-cone (SNV alt windows recompute <=20 of 106 conv6 rows; bit-identical)" if S == 1 else
                 "segments (trunk shared across shifts; bit-identical)",
    }
    if eng.precision == "f16x3":
        fb, sx = eng.f16_state()
        rec["f16x3"] = {"fallback_calls": fb, "activation_scale_exp": sx}
    if world == 1 and not args.no_extras:
        extras = {}
        # configs[2]: the +-800 shift sweep (9 shifts) -- segment path (trunk shared across shifts)
        sh9 = shift_order(800)
        v3 = make_variants(genome, 400, 101)
        p3 = pipe.prepare(v3, sh9)
        el3, l3 = time_workload(pipe, eng, p3, sh9, 400, 2, 1, dev, 1)
        extras["cfg3_shift_sweep_800"] = {
            "variants_per_s": 400 * 2 / el3, "windows_per_variant": 36, "dense_windows_per_s": 400 * 36 * 2 / el3,
            "executed_fp32_tflops": 2.0 * sum(m for _, _, m in l3.values()) / el3 / 1e12,
            "layer_ms_per_step": {k: ms / 2 for k, (ms, c, m) in l3.items()},
            "layer_tflops": {k: 2.0 * m / (ms * 1e-3) / 1e12 for k, (ms, c, m) in l3.items() if ms > 0},
            "roofline": roofline(l3, eng.precision)}
        # the metric's literal unit: a variant scored with 200 windows (+-20 kb, stride 200) x ref/alt x fwd/rc
        sh200 = list(range(-20000, 20000, 200))
        v200 = make_variants(genome, N200, 202)
        p200 = pipe.prepare(v200, sh200)
        el2, l2 = time_workload(pipe, eng, p200, sh200, N200, 2, 1, dev, 1)
        extras["variant_200_windows"] = {
            "variants_per_s": N200 * 2 / el2, "variants_per_step": N200, "windows_per_variant": 800,
            "dense_windows_per_s": N200 * 800 * 2 / el2,
            "executed_fp32_tflops": 2.0 * sum(m for _, _, m in l2.values()) / el2 / 1e12,
            "layer_ms_per_step": {k: ms / 2 for k, (ms, c, m) in l2.items()},
            "layer_tflops": {k: 2.0 * m / (ms * 1e-3) / 1e12 for k, (ms, c, m) in l2.items() if ms > 0},
            "roofline": roofline(l2, eng.precision)}
        # the same headline workload under the other two arithmetics (all three pass the same
        # parity bar; DESIGN.md accuracy table): exact fp32 MFMA and fp32-faithful bf16x6
        alt_prec = {}
        for prec in ("bf16x6", "fp32"):
            if prec == eng.precision:
                continue
            base = eng.precision
            eng.set_precision(prec)
            elp, lp = time_workload(pipe, eng, prep, shifts, n, 3, 1, dev, 1)
            eng.set_precision(base)
            rp = roofline(lp, prec)
            alt_prec[prec] = {"variants_per_s": n * 3 / elp, "ms_per_step": elp / 3 * 1e3,
                              "dominant": {k: rp[k] for k in ("kernel", "layer", "achieved", "peak", "frac")}}
        extras["headline_other_precisions"] = alt_prec
        extras["cfg5_tss_features"] = tss_workload(eng, genome, pipe.dg, dev)
        extras["hbm_reductions"] = hbm_reductions(dev)
        rec["extra_workloads"] = extras
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from expecto_amd.encode import seqs_to_codes
        g1 = genome["chr1"]
        rng = np.random.default_rng(5)
        sample = [g1[p - 1000:p + 1000] for p in rng.integers(5000, len(g1) - 5000, 32)]
        rec["cpu_baseline"] = cpu_baseline(sd_cpu, seqs_to_codes(sample), args.cpu_seconds,
                                           min(args.cpu_threads, os.cpu_count() or 1), 4 * S)
        rec["speedup_vs_cpu_baseline"] = value / rec["cpu_baseline"]["value"]
        if args.cpu_threads != 8:
            # SURVEY.md 8(d) asks for P = 8 beside the box's full share (a shorter sample)
            p8 = cpu_baseline(sd_cpu, seqs_to_codes(sample), args.cpu_seconds / 2, 8, 4 * S)
            rec["cpu_baseline_8_threads"] = {k: p8[k] for k in ("value", "unit", "cores", "windows_per_s", "sample")}
    if world > 1:
        rec["final_gather"] = time_final_gather(S, n, dev, rank, world)
    if rank == 0:
        print(json.dumps(rec))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
