"""Benchmark of the ExPecto hot path on MI355X (contract: see task / DESIGN.md "Measurement").

Headline workload = BASELINE.json's metric unit, the "200-window variant" (per GPU and step):
96 seeded SNVs, each scored with 200 windows (shifts -20000..19800 step 200,
geuvadis_sed_for_top_eqtls.py:61) x ref/alt allele x fwd/rc strand = 800 Beluga windows per
variant.  One step = window generation from the HBM-resident genome + the Beluga forward of
all 76,800 windows (segment path: conv trunk shared across the shifts, alt allele through
its SNV cone, bit-identical to per-window forwards) + the float64 fwd/rc mean and 10 x 200
exp-decay reduction to 20030 features per allele (geuvadis_sed_for_top_eqtls.py:83-121).
`value` is timed with layer profiling OFF; the f16x3 overflow flag is checked at the end of
every step (the release point of a batch) and a flagged step is recomputed in bf16x6 inside
the timed region.  Layer times and the roofline come from a separate profiled pass.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

N>1: weak scaling, each rank its own 96 variants per step, no collective in the step (variants
are independent).  N>1 extra, outside `value`: configs[3]'s per-rank shape (100k SNVs over 8
ranks = 12.5k SNVs x 9 shifts per rank) computed once and its outputs gathered to rank 0 per
shift over RCCL (the file-output exchange), both timed.  Rank 0 prints ONE JSON line.

N=1 extras, outside `value`: the headline in bf16x6 (fp32-faithful split), configs[1]
(1k SNVs, shift 0), configs[2] (+-800 sweep), configs[4] TSS genes, the chromatin CLI end to
end (streamed batches vs one batch: compute overlapped with the .diff.h5 writes), the HBM-bound
reductions in GB/s, and the CPU port timed on host cores (P = this job's CPU share and 8, batch 32 and 512).
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
from expecto_amd.pipeline import VariantPipeline, VariantSet, shift_order  # noqa: E402

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
WINDOW_MACS = sum(LAYER_MACS.values())

SHIFTS_200 = list(range(-20000, 20000, 200))     # geuvadis_sed_for_top_eqtls.py:61, compute_expecto_features.py:88
N200 = 96                                        # 200-window variants per GPU and step
WIN_PER_VARIANT_200 = 2 * 2 * len(SHIFTS_200)    # ref/alt x fwd/rc x 200 shifts = 800
SNV_MARGIN_200 = 25_000                          # every window of the +-20 kb sweep inside its contig
CFG3_PER_RANK = 12_500                           # configs[3]: 100k SNVs over 8 ranks
CFG4_PER_RANK = 2_500                            # configs[4]: 20k genes over 8 ranks

DTYPES = {
    "bf16x6": "fp32 (bf16x6: exact 3-way bf16 split, 6 MFMA products, fp32 accumulate)",
    "f16x3": "fp32 in/out (f16x3: power-of-2-scaled 2-way fp16 split = 22-bit operands, 3 MFMA products, "
             "fp32 accumulate; bf16x6 recompute on fp16 overflow)",
    "fp32": "fp32",
}


def conv2_table_on(precision: str = "f16x3") -> bool:
    """conv1 + conv2 + pool1 from the k-mer table (the library default for f16x3 and bf16x6 forwards
    from codes; EXPECTO_CONV2_TABLE=0 runs them on the MFMAs)."""
    return precision in ("f16x3", "bf16x6") and os.environ.get("EXPECTO_CONV2_TABLE", "1") != "0"


def fc1_karatsuba_on(precision: str = "f16x3") -> bool:
    """FC1 as the block-Karatsuba convolution (the library default for f16x3; EXPECTO_FC1_KARATSUBA=0
    runs the direct split-K FC1): 9 block products per 4 windows instead of 16 on the headline."""
    return precision == "f16x3" and os.environ.get("EXPECTO_FC1_KARATSUBA", "1") != "0"


# 200-window segment (41,800 bp): pooled conv2 rows per segment, and the k-mer gather's algorithmic
# bytes per pooled row (4 conv2 rows x 2 quad-table rows of 320 fp32 read, 320 fp16 hi + lo planes
# written; a conv2 half whose 11-mer holds an N reads 2 pair-table rows instead of 1)
SEG200_POOL1_ROWS = ((2000 + 199 * 200 - 7) - 7) // 4
KMER_BYTES_PER_POOLED_ROW = 8 * 320 * 4 + 320 * 4


def conv2_table_roofline(layers, n):
    """HBM roofline of the k-mer gather (conv2_kmer_pool) of the headline: algorithmic bytes per
    strand launch over its average launch time (HIP events on the launch stream)."""
    ms, calls, _ = layers["conv2"]
    if not calls:
        return None
    b = n * SEG200_POOL1_ROWS * KMER_BYTES_PER_POOLED_ROW
    gbs = b / (ms / calls * 1e-3) / 1e9
    return {"bound": "hbm", "kernel": "conv2_kmer_pool", "achieved": gbs, "peak": 8000.0, "unit": "GB/s",
            "frac": gbs / 8000.0, "bytes_per_launch": b, "avg_launch_ms": ms / calls, "launches": calls,
            "what": f"{n} segments x {SEG200_POOL1_ROWS} pooled rows x (8 quad-table rows x 1,280 B read + 1,280 B "
                    f"written); table hits in L2 / Infinity Cache (repeated k-mers) count as HBM bytes here"}


def kernel_name(layer: str, precision: str, segments: bool = True) -> str:
    """rocprofv3 kernel name of a layer's launch.  On the segment path (the headline, configs[2]
    and [4]) conv4 writes the pool2 phase blocks from its epilogue (f16x3; else it runs unpooled and
    its pool2 is a separate per-phase kernel)."""
    if layer not in GEMM_LAYER_EPI:
        return {"conv1": "beluga_conv1", "fc1_reduce": "fc1_reduce"}[layer]
    l, e = GEMM_LAYER_EPI[layer]
    if segments and layer == "conv4":
        # unpooled, its pool2 a separate pass; f16x3 with the pool2 phases in the epilogue: EPI 4
        e = 4 if precision == "f16x3" and os.environ.get("EXPECTO_POOL_FUSED", "1") != "0" else 0
    if layer == "conv2" and conv2_table_on(precision):
        return "conv2_kmer_pool"                           # conv1 + conv2 + pool1 gathered from the k-mer table
    if precision == "bf16x6":
        return f"beluga_gemm_x6q<{l}, {e}, 0>"
    if precision == "f16x3":
        if l == 7 and fc1_karatsuba_on(precision):
            return "beluga_fc_h3k"                         # FC1 products + tail: one grouped launch
        if l in (7, 8):   # split-K FC GEMMs on 336-column tiles (beluga_fc_h3w)
            return f"beluga_fc_h3w<{l}, {e}, 0>"
        ea = 64 if os.environ.get("EXPECTO_CONV_EA", "1") != "0" else 0   # early next-stage reads (TM bit 64)
        if layer == "conv2" and os.environ.get("EXPECTO_FUSE_CONV1", "1") != "0":
            return f"beluga_conv_h3p<{l}, {e}, {16640 + ea}, 4>"   # conv1 fused into the producers (256 | 16384)
        return f"beluga_conv_h3p<{l}, {e}, {256 + ea}, 4>"   # producer / consumer 256-row tiles (every conv layer)
    return f"beluga_gemm<{l}, {e}, 4, 2, 32, 1>"


# ---- CPU baseline ---------------------------------------------------------------------------
def host_cpu_share():
    """CPUs this job may use: the affinity mask (os.sched_getaffinity) and the cgroup v2 / v1
    CPU quota (cpu.max, cfs_quota_us / cfs_period_us), whichever is smaller.  os.cpu_count()
    reports the whole machine (256 on the GPU box), not this job's share."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    share = aff if quota is None else max(1, min(aff, int(math.ceil(quota))))
    return {"affinity_cpus": aff, "cgroup_cpus": quota, "host_cpu_count": os.cpu_count(), "share": share}


def cpu_baseline(sd_cpu, codes: np.ndarray, seconds: float, windows_per_variant: int):
    """Oracle torch-CPU forward (the reference's CPU arithmetic, oneDNN fp32) on a bounded sample
    of the headline's windows, at P = this job's CPU share (affinity mask and cgroup quota,
    host_cpu_share; SURVEY.md 8(d) "P = all physical cores" of what the job may use) and P = 8,
    batch 32 and 512.  Per window the cost is linear, so windows/s extrapolates; variants/s =
    windows/s / 800 (the reference forwards every window of a 200-window variant,
    geuvadis_sed_for_top_eqtls.py:80-98).  `value` is the best setting; `cores` its thread count."""
    from oracle.beluga_np import forward_torch_cpu
    from expecto_amd.encode import codes_to_onehot

    share = host_cpu_share()
    x_all = torch.from_numpy(codes_to_onehot(codes, with_rc=False).astype(np.float32)).unsqueeze(2)
    runs = {}
    for threads in sorted({share["share"], 8}, reverse=True):
        torch.set_num_threads(threads)
        forward_torch_cpu(sd_cpu, x_all[:4])                     # warm-up
        for batch in (32, 512):
            x = x_all[:batch]
            done, t0 = 0, time.perf_counter()
            while True:
                forward_torch_cpu(sd_cpu, x)
                done += x.shape[0]
                el = time.perf_counter() - t0
                if el >= seconds:
                    break
            runs[f"p{threads}_b{batch}"] = {"windows_per_s": done / el, "windows": done, "s": el,
                                            "threads": threads, "batch": batch}
    best_k = max(runs, key=lambda k: runs[k]["windows_per_s"])
    best = runs[best_k]
    return {"value": best["windows_per_s"] / windows_per_variant, "unit": "variants/s", "cores": best["threads"],
            "kind": "port", "windows_per_s": best["windows_per_s"], **share,
            "per_setting": {k: dict(v, variants_per_s=v["windows_per_s"] / windows_per_variant)
                            for k, v in runs.items()},
            "sample": f"seeded SNV ref windows of the headline workload; oracle/beluga_np.forward_torch_cpu "
                      f"(torch CPU fp32, oneDNN) at P = {share['share']} (this job's CPU share: affinity "
                      f"{share['affinity_cpus']}, cgroup quota {share['cgroup_cpus']}) and 8 threads x batch 32 "
                      f"and 512, ~{seconds:.0f} s each; value = best setting ({best_k}) / {windows_per_variant} "
                      f"windows per variant"}


# ---- HBM-bound reductions -----------------------------------------------------------------
def hbm_reductions(dev):
    """The metric's "HBM GB/s vs peak": the HBM-bound spatial reductions timed
    with HIP events on synthetic inputs resident in HBM; algorithmic bytes = every input read
    once + every output written once.
      TSS (compute_expecto_features.py:91-124): 1000 genes x 200 shifts x 2002, fwd + rc fp32 ->
        [1000, 20020] fp64 (3.2 MB read + 160 KB written per gene);
      variant (predict.py:87-136): 20000 variants x 9 shifts x 2002 fp32 -> [20000, 20020] fp64
        (write-dominated: "fp64_fill_ceiling" times torch's zero_ of the same output, the
        practical write rate on this box);
      sed (geuvadis_sed_for_top_eqtls.py:83-121): the headline step's per-allele reduction, 96
        variants x 200 shifts x fwd/rc -> [96, 20030] fp64 (a small grid: 3 waves per SIMD)."""
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
    sh = shift_order(800)
    vout = torch.empty((n_var, 10 * F), dtype=torch.float64, device=dev)
    vtab = features.variant_tables(dist, plus, sh, dev)   # inputs resident: not part of the timing
    # the headline step's own reduction (geuvadis_sed_for_top_eqtls.py:83-121): one allele of
    # the 96-variant step, float64 fwd/rc mean, legacy 20030 layout
    from expecto_amd import _lib
    lib, NS = _lib.load(), 96
    sfwd, src = fwd[:NS], rc[:NS]
    sout = torch.empty((NS, 10 * (F + 1)), dtype=torch.float64, device=dev)
    def sed_reduce():
        _lib.check(lib.expecto_shift_reduce(_lib.dptr(sfwd), _lib.dptr(src), _lib.dptr(w), NS, S, F, 3,
                                            _lib.dptr(sout), _lib.stream_ptr()), "shift_reduce")
    for name, fn, nbytes in (
            ("fp64_fill_ceiling", lambda: vout.zero_(), n_var * 10 * F * 8),   # write-only reference
            ("tss_reduce", lambda: features.tss_reduce(fwd, rc, w, out), 2 * G * S * F * 4 + G * 10 * F * 8),
            ("variant_reduce", lambda: features.variant_reduce(eff, vtab, vout),
             S9 * n_var * F * 4 + n_var * 10 * F * 8),
            ("sed_shift_reduce_96", sed_reduce, 2 * NS * S * F * 4 + NS * 10 * (F + 1) * 8)):
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
    del fwd, rc, eff, out, vout, sfwd, src, sout, vtab
    torch.cuda.empty_cache()
    return res


# ---- workloads ------------------------------------------------------------------------------
def make_variants(genome, n, seed, margin=5000):
    snvs = synthetic.snvs(genome, n, seed=seed, margin=margin)
    return VariantSet([v[0] for v in snvs], np.array([v[1] for v in snvs]), [v[2] for v in snvs],
                      [v[3] for v in snvs])


class Sed200:
    """The headline step: 200-window variants (geuvadis_sed_for_top_eqtls.py:61-121).  Two output
    slots, so step k+1 can be enqueued before step k is released (time_steps)."""

    def __init__(self, pipe, genome, n, seed, dev):
        from expecto_amd.features import tss_pos_weights
        self.pipe, self.n = pipe, n
        self.vs = make_variants(genome, n, seed, margin=SNV_MARGIN_200)
        self.prep = pipe.prepare(self.vs, SHIFTS_200, rows="variant")
        S = len(SHIFTS_200)
        self.y = [torch.empty((2, 2, n, S, 2002), dtype=torch.float32, device=dev) for _ in range(2)]
        self.w = torch.from_numpy(tss_pos_weights(np.asarray(SHIFTS_200))).to(dev)
        self.feat = [torch.empty((2, n, 20030), dtype=torch.float64, device=dev) for _ in range(2)]

    def __call__(self, slot=0):
        self.pipe.predict(self.prep, out=self.y[slot])
        self.pipe.sed_features(self.y[slot], self.w, out=self.feat[slot])

    def recover(self, slot):
        """The step's f16x3 overflow flag fired: recompute only the flagged variant slices in
        bf16x6 (VariantPipeline.recompute_overflowed), then the features."""
        n = self.pipe.recompute_overflowed(self.vs, SHIFTS_200, self.y[slot], rows="variant")
        self.pipe.sed_features(self.y[slot], self.w, out=self.feat[slot])
        return n


class ShiftSweep:
    """chromatin.py's device work for one variant batch: every shift's ref/alt x fwd/rc windows
    + diff = alt - ref (configs[1]: shift 0; configs[2]/[3]: +-800)."""

    def __init__(self, pipe, genome, n, seed, shifts, dev):
        self.pipe, self.n, self.S = pipe, n, len(shifts)
        self.prep = pipe.prepare(make_variants(genome, n, seed), shifts)
        self.ys = [torch.empty((2, 2, self.S, n, 2002), dtype=torch.float32, device=dev) for _ in range(2)]
        self.y = self.ys[0]
        self.d = None

    def __call__(self, slot=0):
        self.y = self.ys[slot]
        self.pipe.predict(self.prep, out=self.y)
        self.d = self.pipe.diff(self.y)


def time_steps(step, eng, steps, warmup, world, dev):
    """Wall time of `steps` steps between barriers + syncs (max over ranks), profiling off.
    Every step is released inside the timed region, as the streamed chromatin CLI releases its
    batches: step k's f16x3 overflow flag is copied to pinned memory behind its kernels
    (overflow_take), step k+1 is enqueued (into the other output slot), then step k's event is
    waited for and its flag read; a flagged step is recomputed in bf16x6 before moving on.  So
    the host work that prepares a step overlaps the previous step's kernels instead of idling
    the GPU at every release (0.7 ms of 97 on the headline)."""
    fallbacks = 0
    f16 = eng.precision == "f16x3"
    flags = [torch.zeros(1, dtype=torch.int32, pin_memory=True) for _ in range(2)]
    events = [torch.cuda.Event() for _ in range(2)]
    state = {"k": 0, "pending": None}

    def release(slot):
        nonlocal fallbacks
        events[slot].synchronize()
        if f16 and int(flags[slot][0]):
            fallbacks += 1
            if hasattr(step, "recover"):     # only the flagged variant slices in bf16x6
                step.recover(slot)
            else:
                eng.count_fallback()
                with eng.precision_override("bf16x6"):
                    step(slot)
            torch.cuda.synchronize()

    def one():
        slot = state["k"] % 2
        step(slot)
        if f16:
            eng.overflow_take(flags[slot])
        events[slot].record()
        if state["pending"] is not None:
            release(state["pending"])
        state["pending"] = slot
        state["k"] += 1

    def drain():
        if state["pending"] is not None:
            release(state["pending"])
            state["pending"] = None

    for _ in range(warmup):
        one()
    drain()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
    drain()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        el = float(t.item())
    return el, fallbacks


def profile_layers(step, eng, steps):
    """Per-layer HIP-event times / launches / executed MACs over `steps` profiled steps (a pass
    apart from the timed one)."""
    torch.cuda.synchronize()
    eng.set_profiling(True)
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    layers = eng.layer_times()
    eng.set_profiling(False)
    eng.overflow_pending()
    return layers


def products_and_peak(precision):
    if precision == "bf16x6":
        return BF16X6_PRODUCTS, BF16_MFMA_PEAK_TFLOPS
    if precision == "f16x3":
        return F16X3_PRODUCTS, BF16_MFMA_PEAK_TFLOPS
    return 1, FP32_MFMA_PEAK_TFLOPS


CONV_LAYERS = ("conv2", "conv3", "conv4", "conv5", "conv6")


def main_launches(eng):
    """{conv layer: (rows, ms, launches, MACs)} of its full-size GEMM launches alone, timed while
    profiling (include/expecto_hip.h expecto_beluga_main_launches)."""
    return {k: eng.main_launches(k) for k in CONV_LAYERS}


def roofline(layers, precision, segments=True, main=None):
    """MFMA roofline of the dominant GEMM kernel from executed work per launch (library counts)
    over its average launch duration (HIP events on the launch stream).  For a conv layer the
    figure is taken over its FULL-SIZE launches alone (`main`: the GEMM launch without the pool2
    pass that shares conv4's slot, nor the small alt-delta launches; the rocprofv3 launch_groups.csv
    row of the largest grid times the same launches); the slot's all-launch figure stands beside it."""
    gemm = [k for k in GEMM_LAYER_EPI if not (k == "conv2" and conv2_table_on(precision))]
    dom = max(gemm, key=lambda k: layers[k][0])   # (the f16x3 conv2 is a gather: conv2_table_roofline)
    ms, calls, macs = layers[dom]
    mult, peak = products_and_peak(precision)
    all_tflops = 2.0 * macs / calls / (ms / calls / 1e3) / 1e12
    all_launches = {"avg_launch_ms": ms / calls, "launches": calls, "fp32_tflops": all_tflops,
                    "frac": mult * all_tflops / peak,
                    "what": "every launch of the layer slot, HIP events around the layer (conv4: + its pool2 pass)"}
    rows = 0
    if main and dom in main and main[dom][2] > 0:
        rows, ms, calls, macs = main[dom]
    fp32_flops_launch = 2.0 * macs / calls
    fp32_tflops = fp32_flops_launch / (ms / calls / 1e3) / 1e12
    achieved = mult * fp32_tflops
    return {"bound": "mfma", "kernel": kernel_name(dom, precision, segments), "layer": dom, "achieved": achieved,
            "peak": peak, "unit": "TFLOP/s", "frac": achieved / peak, "traffic": None,
            "avg_launch_ms": ms / calls, "launches": calls, "rows_per_launch": rows or None,
            "timed": "full-size launches alone" if rows else "every launch of the slot",
            "mfma_flops_per_launch": mult * fp32_flops_launch,
            "fp32_flops_per_launch": fp32_flops_launch, "fp32_tflops": fp32_tflops, "precision": precision,
            "all_launches": all_launches}


def profile_key(n=None, precision="f16x3"):
    """Workload key a committed rocprofv3 profile (profiles/<tag>/traffic.json) must carry for
    its PMC numbers to be attached to this bench line."""
    return {"workload": "sed200", "variants": N200 if n is None else n, "precision": precision,
            "max_batch": MAX_BATCH, "genome": "repeat-rich",
            "fc1": "karatsuba" if fc1_karatsuba_on(precision) else "direct"}


def pmc_traffic(key, kernel):
    """HBM bytes per launch of ``kernel`` from the newest committed rocprofv3 --pmc summary
    (profiles/<tag>/traffic.json, written by tools/collect_profiles.py from FETCH_SIZE and
    WRITE_SIZE passes of this same bench command).  None unless that profile was taken on the
    same workload key: PMC counters cannot be read live next to the HIP-event timing."""
    import glob
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "r*", "traffic.json")), reverse=True):
        try:
            t = json.load(open(path))
        except (OSError, ValueError):
            continue
        if t.get("profile_key") != key:
            continue
        for name, v in t["kernels"].items():
            if kernel in name:   # the layer's full launches (the alt-delta launches share the kernel)
                return v.get("main_hbm_bytes", v["hbm_bytes"]), t["source"]
    return None, None


def pmc_held_clock(key, kernel):
    """MFMA-busy fraction and held clock of ``kernel`` from the same committed profile as
    pmc_traffic (profiles/<tag>/pmc_sq.csv + kernel_stats.csv of this bench command):
    busy = SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8 XCDs), clock =
    GRBM_GUI_ACTIVE / 8 / average duration.  The nominal peak assumes 2.4 GHz; under this load
    the chip holds a lower clock (MI355X_MICROARCH.md "DVFS give-back"), so frac's ceiling is
    clock / 2.4 GHz."""
    import csv
    import glob
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "r*", "traffic.json")), reverse=True):
        d = os.path.dirname(path)
        try:
            if json.load(open(path)).get("profile_key") != key:
                continue
            sq = [r for r in csv.DictReader(open(os.path.join(d, "pmc_sq.csv"))) if kernel in r["kernel"]]
            lg = os.path.join(d, "launch_groups.csv")
            if os.path.exists(lg):   # the full-size launches (largest grid) of the kernel
                st = sorted((r for r in csv.DictReader(open(lg)) if kernel in r["kernel"]),
                            key=lambda r: -int(r["grid_size"]))[:1]
                ns = float(st[0]["avg_ns"]) if st else None
            else:
                st = [r for r in csv.DictReader(open(os.path.join(d, "kernel_stats.csv"))) if kernel in r["Name"]]
                ns = float(st[0]["AverageNs"]) if st else None
        except (OSError, ValueError, KeyError):
            continue
        if not sq or not ns:
            continue
        g = float(sq[0]["GRBM_GUI_ACTIVE"]) / 8
        busy = float(sq[0]["SQ_VALU_MFMA_BUSY_CYCLES"]) / 1024 / g
        clock = g / (ns * 1e-9) / 1e9
        return {"mfma_busy": busy, "held_clock_ghz": clock, "frac_ceiling_at_held_clock": clock / 2.4,
                "avg_launch_ns_rocprof": ns, "source": os.path.relpath(os.path.join(d, "pmc_sq.csv"), REPO)}
    return None


def layer_summary(layers, el_steps):
    return ({k: ms / el_steps for k, (ms, c, m) in layers.items()},
            {k: 2.0 * m / (ms * 1e-3) / 1e12 for k, (ms, c, m) in layers.items() if ms > 0})


def measure(step, eng, n_units, steps, warmup, world, dev, prof_steps=2, segments=True):
    """(units/s, ms/step, fallbacks, layers, roofline, executed MACs per step)."""
    el, fb = time_steps(step, eng, steps, warmup, world, dev)
    layers = profile_layers(step, eng, prof_steps)
    main = main_launches(eng)
    exec_macs = sum(m for _, _, m in layers.values()) / prof_steps
    return {"units_per_s": world * n_units * steps / el, "ms_per_step": el / steps * 1e3, "fallbacks": fb,
            "layers": layers, "roofline": roofline(layers, eng.precision, segments, main), "exec_macs_step": exec_macs,
            "prof_steps": prof_steps}


def extra_record(m, unit, n_units, windows_per_unit, precision):
    ms_l, tf_l = layer_summary(m["layers"], m["prof_steps"])
    mult, peak = products_and_peak(precision)
    step_s = m["ms_per_step"] * 1e-3
    return {unit: m["units_per_s"], f"{unit.split('_')[0]}_per_step": n_units, "ms_per_step": m["ms_per_step"],
            "windows_per_unit": windows_per_unit, "dense_windows_per_s": m["units_per_s"] * windows_per_unit,
            "executed_fp32_tflops": 2.0 * m["exec_macs_step"] / step_s / 1e12,
            "step_mfma_frac": mult * 2.0 * m["exec_macs_step"] / step_s / 1e12 / peak,
            "f16_fallback_steps": m["fallbacks"], "layer_ms_per_step": ms_l, "layer_tflops": tf_l,
            "roofline": m["roofline"], "precision": precision}


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
    step = lambda slot=0: pipe.features(chroms, tss, strands)   # noqa: E731
    el, fb = time_steps(step, eng, steps, 1, 1, dev)
    gps = genes * steps / el
    return {"genes_per_s": gps, "genes_per_step": genes, "windows_per_gene": 400, "f16_fallback_steps": fb,
            "dense_windows_per_s": gps * 400, "ms_per_step": el / steps * 1e3,
            "projected_20k_genes_s_1gpu": 20000 / gps, "projected_20k_genes_s_8gpu_weak": 20000 / gps / 8}


def _cli_run(d, fa, vcf, name, vb, runs=2):
    """chromatin.run over `vcf` into d/name (stdout swallowed: bench prints one JSON line); the
    fastest of `runs` runs' LAST_RUN timings (the first also pays pinned-buffer allocation)."""
    import contextlib
    import io
    from expecto_amd import chromatin
    args = chromatin.build_parser().parse_args(
        [vcf, "--genome", fa, "--synthetic-weights", "0", "--output_dir", os.path.join(d, name), "--variant-batch",
         str(vb), "--max-batch", str(MAX_BATCH)])
    out = []
    for _ in range(runs):
        with contextlib.redirect_stdout(io.StringIO()):
            chromatin.run(args)
        out.append(dict(chromatin.LAST_RUN))
    return min(out, key=lambda r: r["loop_s"])


def cli_streamed(genome, n=8192):
    """The chromatin CLI end to end (chromatin.py:243-286) on configs[2]'s +-800 sweep of n
    seeded SNVs: device forward + diff + D2H into pinned buffers + the .diff.h5 row writes of
    every shift, streamed in batches of n/4 (batch k+1 computes while batch k is written, the
    overflow flag read at the release point) against one batch (no overlap).  Batch-loop wall
    time (model / genome setup excluded); variants on chr23/chr24 are filtered as chromatin.py
    does (CHRS).  Files go to a temporary directory, removed afterwards.
    `cfg3_rank`: the same CLI at configs[3]'s per-rank shape (12,500 SNVs x 9 shifts = 1/8 of
    100k), streamed in the default 4,096-variant batches, once: under --output-mode rank every
    rank of an 8-GPU run does exactly this (its own rows into the shared files, no collective),
    so its loop time is the 8-GPU CLI's; write_share = host row-write seconds / loop seconds."""
    import shutil
    import tempfile
    d = tempfile.mkdtemp(prefix="expecto_cli_")
    try:
        fa = os.path.join(d, "genome.fa")
        synthetic.write_fasta(fa, genome)
        vcf = os.path.join(d, "snvs.vcf")
        with open(vcf, "w") as f:
            for c, p, r, a in synthetic.snvs(genome, n, seed=77):
                f.write(f"{c}\t{p}\t.\t{r}\t{a}\n")
        out = {}
        for name, vb in (("streamed", n // 4), ("one_batch", n)):
            st = _cli_run(d, fa, vcf, name, vb)
            out[name] = {"loop_s": st["loop_s"], "variants_per_s": st["variants"] / st["loop_s"],
                         "batches": st["batches"], "host_launch_s": st["launch_s"], "host_wait_s": st["wait_s"],
                         "host_write_s": st["write_s"]}
            shutil.rmtree(os.path.join(d, name), ignore_errors=True)
        nv = st["variants"]
        out["variants"] = nv
        out["h5_bytes_written"] = 9 * 3 * 2 * nv * 2002 * 4
        out["what"] = ("chromatin CLI batch loop, +-800 sweep: forward + diff + D2H + snps.shift_*.diff.h5 rows; "
                       "streamed = 4 batches overlapping compute with the previous batch's writes")
        vcf3 = os.path.join(d, "cfg3.vcf")
        with open(vcf3, "w") as f:
            for c, p, r, a in synthetic.snvs(genome, CFG3_PER_RANK, seed=78):
                f.write(f"{c}\t{p}\t.\t{r}\t{a}\n")
        st = _cli_run(d, fa, vcf3, "cfg3", 4096, runs=1)
        out["cfg3_rank"] = {"variants": st["variants"], "shifts": st["shifts"], "batches": st["batches"],
                            "loop_s": st["loop_s"], "variants_per_s": st["variants"] / st["loop_s"],
                            "host_launch_s": st["launch_s"], "host_wait_s": st["wait_s"],
                            "host_write_s": st["write_s"], "write_share": st["write_s"] / st["loop_s"],
                            "h5_bytes_written": 9 * 3 * 2 * st["variants"] * 2002 * 4,
                            "what": "configs[3] per-rank shape through the CLI (1 GPU, --output-mode rank: what each "
                                    "of 8 ranks does in parallel; unmeasured on 8 GPUs)"}
        return out
    finally:
        shutil.rmtree(d, ignore_errors=True)


def replicate_rank(genome, genes=CFG4_PER_RANK):
    """configs[4]'s named path per rank (replicate_expecto_features.py:65-86; 20k genes over 8
    GPUs = 2,500 per rank): the streamed `tss replicate` CLI run in-process on seeded TSSs of the
    bench genome, writing one (200, 2002) float32 .npy per gene (4 GB) into a temporary
    directory: setup (genome open, model, HBM genome), batch loop (forward + fwd/rc mean + D2H +
    the .npy writes of the previous batch), host write seconds, genes/s of the loop."""
    import contextlib
    import io
    import shutil
    import tempfile
    from expecto_amd import tss
    d = tempfile.mkdtemp(prefix="expecto_rep_", dir=os.environ.get("EXPECTO_BENCH_TMP"))
    try:
        fa = os.path.join(d, "genome.fa")
        synthetic.write_fasta(fa, genome)
        rng = np.random.default_rng(56)
        names = sorted(genome)
        anno = os.path.join(d, "anno.csv")
        with open(anno, "w") as f:
            f.write("id,symbol,seqnames,strand,TSS,CAGE_representative_TSS,type\n")
            for k in range(genes):
                c = names[int(rng.integers(0, len(names)))]
                t = int(rng.integers(30000, len(genome[c]) - 30000))
                f.write(f"G{k:06d},S{k},{c},{'+' if rng.random() < 0.5 else '-'},{t},{t},protein_coding\n")
        out = os.path.join(d, "out")
        with contextlib.redirect_stdout(io.StringIO()):
            r = tss.replicate_main([anno, "-o", out, "--genome", fa, "--synthetic-weights", "0",
                                    "--max-batch", str(MAX_BATCH)])
        files = len(os.listdir(out))
        return {"genes": r["genes"], "files": files, "gene_batch": r["gene_batch"], "batches": r["batches"],
                "setup_s": r["setup_s"], "loop_s": r["loop_s"], "total_s": r["total_s"],
                "host_write_s": r["write_s"], "host_wait_s": r["wait_s"], "write_share": r["write_s"] / r["loop_s"],
                "genes_per_s": r["genes"] / r["loop_s"], "npy_bytes_written": files * (200 * 2002 * 4 + 128),
                "recomputed_batches": r["recomputed_batches"],
                "projected_20k_genes_8gpu_s": r["setup_s"] + r["loop_s"] * 20000 / 8 / r["genes"],
                "what": "configs[4] per-rank shape through the streamed `tss replicate` CLI (1 GPU; each of 8 ranks "
                        "does this in parallel with no collective; unmeasured on 8 GPUs)"}
    finally:
        shutil.rmtree(d, ignore_errors=True)


def cli_e2e(n=CFG3_PER_RANK, tmp_root=None):
    """configs[3]'s per-rank shape through the chromatin CLI as a user runs it, setup included
    (VERDICT r03 item 1): a synthetic genome of hg19's size (24 contigs, 3.096 Gbp, written as a
    60-column FASTA), 12,500 SNVs x 9 shifts, `python -m expecto_amd.chromatin` as a child
    process, twice:
      cold = no code cache yet: the first open flattens + encodes the FASTA into the memory-mapped
             cache (expecto_amd.genome; pyfasta's .flat/.gdx role, chromatin.py:44);
      warm = the cache exists (every later run, every rank of a node).
    Per run: the process wall time (Python + torch import, GPU init included) and the CLI's own
    record (EXPECTO_TIMING_JSON): setup_s (genome open, VCF, model, HBM genome upload, engine and
    pinned buffers), loop_s (batch loop incl. .diff.h5 writes), total_s.  The files were just
    written, so the cold run reads the FASTA from the page cache (no root to drop it)."""
    import shutil
    import subprocess
    import tempfile
    root = tmp_root or os.environ.get("EXPECTO_BENCH_TMP") or tempfile.gettempdir()
    need = 17 << 30                                        # FASTA + cache + one run's outputs
    free = shutil.disk_usage(root).free
    if free < need:
        return {"skipped": f"{free / 2**30:.1f} GiB free under {root}, need ~{need / 2**30:.0f}"}
    d = tempfile.mkdtemp(prefix="expecto_e2e_", dir=root)
    try:
        tg = synthetic.TiledGenome()
        fa = os.path.join(d, "hg19.fa")
        t0 = time.perf_counter()
        fa_bytes = tg.write_fasta(fa)
        gen_s = time.perf_counter() - t0
        vcf = os.path.join(d, "cfg3.vcf")
        with open(vcf, "w") as f:
            for c, p, r, a in tg.snvs(n, seed=78):
                f.write(f"{c}\t{p}\t.\t{r}\t{a}\n")
        out = {"genome_bp": int(sum(tg.lengths.values())), "fasta_bytes": fa_bytes, "fasta_write_s": gen_s,
               "snvs": n, "shifts": 9}
        for name in ("cold", "warm"):
            od = os.path.join(d, f"out_{name}")
            tj = os.path.join(d, f"timing_{name}.json")
            env = dict(os.environ, EXPECTO_TIMING_JSON=tj)
            t0 = time.perf_counter()
            r = subprocess.run([sys.executable, "-m", "expecto_amd.chromatin", vcf, "--genome", fa,
                                "--synthetic-weights", "0", "--output_dir", od, "--max-batch", str(MAX_BATCH)],
                               cwd=REPO, env=env, capture_output=True, text=True, timeout=600)
            wall = time.perf_counter() - t0
            if r.returncode != 0:
                out[name] = {"error": r.stderr[-2000:]}
                break
            t = json.load(open(tj))
            out[name] = {"process_s": wall, "setup_s": t["setup_s"], "loop_s": t["loop_s"], "total_s": t["total_s"],
                         "setup": t["setup"], "host_write_s": t["write_s"], "variants": t["variants"],
                         "interpreter_and_imports_s": wall - t["total_s"]}
            shutil.rmtree(od, ignore_errors=True)
        out["what"] = ("chromatin CLI at configs[3]'s per-rank shape on an hg19-sized synthetic genome, as a child "
                       "process: cold = first open builds the memory-mapped code cache, warm = later runs / ranks")
        return out
    finally:
        shutil.rmtree(d, ignore_errors=True)


def operator_api(model, genome, dev, seconds=2.0):
    """The reference's own call of the operator: `input =
    torch.from_numpy(encoded[i*B:(i+1)*B]).unsqueeze(2).cuda(); model.forward(input).cpu().numpy()`
    (chromatin.py:266-279, batch 32 = chromatin.py:37-38; compute_expecto_features.py:115-122,
    batch 200; scripts/sed_immune_atlas, batch 512) on host one-hot float32 windows (pageable, as
    the reference's numpy arrays), H2D and D2H included.  `device_only`: the same forward on an
    input already resident in HBM.  `mfma_conv2`: a handle with EXPECTO_ONEHOT_CODES=0 (one-hot
    floats through conv1 / conv2 on the MFMAs, round 4's path) for comparison; same weights."""
    from expecto_amd.encode import encodeSeqs
    rng = np.random.default_rng(9)
    names = sorted(genome)
    seqs = []
    for _ in range(512):
        c = names[int(rng.integers(0, len(names)))]
        p = int(rng.integers(30000, len(genome[c]) - 30000))
        seqs.append(genome[c][p - 1000:p + 1000].decode())
    enc = encodeSeqs(seqs).astype(np.float32)[:512]           # [512, 4, 2000] fwd windows
    os.environ["EXPECTO_ONEHOT_CODES"] = "0"
    try:
        alt_model = beluga.Beluga(max_batch=MAX_BATCH)
        alt_model.load_state_dict(model.state_dict())
        alt_model = alt_model.cuda()
        alt_model.engine()
    finally:
        del os.environ["EXPECTO_ONEHOT_CODES"]

    def rate(fn, batch):
        fn()
        torch.cuda.synchronize()
        done, t0 = 0, time.perf_counter()
        while True:
            fn()
            done += batch
            el = time.perf_counter() - t0
            if el >= seconds:
                break
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        return done / el

    eng = model.engine()
    eng.set_overflow_check(deferred=False)       # the drop-in's default: outputs final when forward returns
    out = {"table_active": eng.conv2_table_active}
    for batch in (32, 200, 512):
        host = enc[:batch]
        xd = torch.from_numpy(host).unsqueeze(2).to(dev)
        rec = {}
        for name, m in (("k_mer", model), ("mfma_conv2", alt_model)):
            def api(m=m):
                inp = torch.from_numpy(host).unsqueeze(2).cuda(dev)
                return m.forward(inp).cpu().detach().numpy()

            def device_only(m=m):
                return m.forward(xd)
            rec[name] = {"windows_per_s": rate(api, batch), "device_only_windows_per_s": rate(device_only, batch)}
        rec["speedup_k_mer_vs_mfma"] = rec["k_mer"]["windows_per_s"] / rec["mfma_conv2"]["windows_per_s"]
        out[f"batch_{batch}"] = rec
    del alt_model
    torch.cuda.empty_cache()
    eng.set_overflow_check(deferred=True)
    out["what"] = ("Beluga.forward drop-in (expecto_beluga_forward_onehot) on host one-hot float32 batches: H2D + "
                   "forward + D2H per batch, windows/s; k_mer = exact one-hot converted to codes on the device and "
                   "gathered from the k-mer tables (default), mfma_conv2 = the MFMA conv1 / conv2 path")
    return out


def cfg3_rank_shard(pipe, eng, genome, rank, world, dev):
    """configs[3] per rank (100k SNVs over 8 GPUs = 12.5k SNVs x 9 shifts, +-800), computed once
    (timed, max over ranks), then its y + diff gathered to rank 0 one shift at a time (RCCL gather
    over xGMI, as the chromatin CLI does before rank 0 writes each .diff.h5).  Not part of value."""
    sh9 = shift_order(800)
    work = ShiftSweep(pipe, genome, CFG3_PER_RANK, 1000 + rank, sh9, dev)
    el, fb = time_steps(work, eng, 1, 1, world, dev)
    y, d, n, total = work.y, work.d, CFG3_PER_RANK, world * CFG3_PER_RANK

    def gather():
        for j in range(len(sh9)):
            edist.gather_rows_to(y[:, :, j:j + 1], 3, total, world, rank)
            edist.gather_rows_to(d[:, j:j + 1], 2, total, world, rank)

    gather()                                   # warm the communicator
    torch.cuda.synchronize()
    torch.distributed.barrier()
    t0 = time.perf_counter()
    gather()
    torch.cuda.synchronize()
    torch.distributed.barrier()
    gl = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if torch.distributed.get_backend() == "nccl":
        gl = gl.to(dev)
    torch.distributed.all_reduce(gl, op=torch.distributed.ReduceOp.MAX)
    nbytes = (world - 1) * (y.numel() + d.numel()) * 4        # bytes arriving at rank 0
    gms = float(gl.item()) * 1e3
    return {"snvs_per_rank": n, "shifts": sh9, "compute_s": el, "variants_per_s": world * n / el,
            "f16_fallback_steps": fb,
            "gather": {"ms": gms, "bytes_into_rank0": nbytes, "GB_per_s": nbytes / (gms * 1e-3) / 1e9,
                       "what": f"every rank's y + diff to rank 0, one shift at a time "
                               f"({'RCCL' if torch.distributed.get_backend() == 'nccl' else 'gloo'} gather)"}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--variants", type=int, default=N200, help="200-window variants per GPU per step")
    ap.add_argument("--cpu-seconds", type=float, default=7.0, help="per CPU-baseline setting (4 settings)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the extra workloads")
    ap.add_argument("--no-e2e", action="store_true", help="skip the hg19-sized CLI end-to-end extra")
    ap.add_argument("--extras", default="all", help="comma-separated extra workloads to run (default all): "
                    "headline_other,cfg1,cfg2,cfg4,operator_api,cli_streamed,replicate_rank,cli_e2e,hbm")
    ap.add_argument("--precision", default=None, help="GEMM arithmetic (default: the engine default)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) for the scaling runs; gloo to "
                    "rehearse several ranks on one GPU")
    args = ap.parse_args()

    rank, world, local = edist.init(args.dist_backend)
    # one rank per GPU; a rehearsal on fewer GPUs than ranks (--dist-backend gloo) shares them
    local = edist.local_device(local)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    n = args.variants

    # repeat-rich (hg19-like: ~half low-complexity elements, N gaps), so the f16x3 range safety and
    # the operand bit statistics of the headline are those of realistic sequence
    genome = synthetic.genome_bytes(n_contigs=24, contig_len=2_000_000, seed=0, repeats=True)
    fasta = Fasta.from_dict(genome)
    model = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=MAX_BATCH)
    sd_cpu = {k: v.detach().clone() for k, v in model.state_dict().items()} if (rank == 0 and world == 1) else None
    model = model.cuda()
    eng = model.engine()
    if args.precision:
        eng.set_precision(args.precision)
    eng.set_overflow_check(deferred=True)              # checked at each step's release point
    pipe = VariantPipeline(eng, fasta, DeviceGenome(fasta, device=dev))
    head = Sed200(pipe, genome, n, 202 + rank, dev)    # variant tables resident in HBM

    m = measure(head, eng, n, args.steps, args.warmup, world, dev)
    ms_l, tf_l = layer_summary(m["layers"], m["prof_steps"])
    mult, peak = products_and_peak(eng.precision)
    step_s = m["ms_per_step"] * 1e-3
    key = profile_key(n, eng.precision)
    roof = m["roofline"]
    roof["traffic"], src = pmc_traffic(key, roof["kernel"])
    if roof["traffic"] is not None:
        roof["traffic_unit"] = "bytes/launch (HBM read+write)"
        roof["traffic_source"] = src
    held = pmc_held_clock(key, roof["kernel"])
    if held is not None:
        roof["pmc"] = held
    rec = {
        "metric": METRIC, "value": m["units_per_s"], "unit": "variants/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": m["ms_per_step"], "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None,
        "dtype": DTYPES[eng.precision],
        "data": "synthetic: seeded repeat-rich genome (24 x 2 Mbp: ~45 % soft-masked homopolymer / tandem / "
                "block / interspersed repeats, N gaps), seeded SNVs, seeded Beluga weights x sqrt(6)",
        "config": {"workload": f"200-window variants (BASELINE metric unit): {n} SNVs/GPU/step x 200 shifts "
                               f"(-20000..19800 step 200) x ref/alt x fwd/rc = {n * WIN_PER_VARIANT_200} Beluga "
                               f"windows/step/GPU; window gen + forward + float64 fwd/rc mean + 10x200 exp-decay "
                               f"reduction to 20030 features per allele (geuvadis_sed_for_top_eqtls.py:61-121)",
                   "variants_per_gpu_step": n, "windows_per_variant": WIN_PER_VARIANT_200,
                   "parallelism": f"dp{world} (variant shards)"},
        "windows_per_s": m["units_per_s"] * WIN_PER_VARIANT_200,
        "dense_equivalent_tflops": 2.0 * WINDOW_MACS * m["units_per_s"] * WIN_PER_VARIANT_200 / 1e12,
        "executed_fp32_tflops": 2.0 * m["exec_macs_step"] * world / step_s / 1e12,
        "step_mfma_frac": mult * 2.0 * m["exec_macs_step"] / step_s / 1e12 / peak,
        "roofline": roof,
        "conv2_table_gather": (conv2_table_roofline(m["layers"], n)
                               if conv2_table_on(eng.precision) else None),
        "layer_ms_per_step": ms_l,
        "layer_tflops": tf_l,
        "layer_timing": f"separate profiled pass of {m['prof_steps']} steps (HIP events per launch); the "
                        f"*_delta slots run on the second stream beside the ref launches (upper bounds)",
        "f16_fallback_steps": m["fallbacks"],
        "conv2_table": dict(zip(("active", "state"), eng.conv2_table_state())),
        "profile_key": key,
        "reuse": "segments (conv trunk shared by the 200 shifts) + alt-cone (the alt allele recomputes only the "
                 "rows its SNV changes; windows without it copy the ref row); bit-identical to per-window forwards",
    }
    if eng.precision == "f16x3":
        fb, sx = eng.f16_state()
        rec["f16x3"] = {"fallback_calls": fb, "activation_scale_exp": sx}
    if world == 1 and not args.no_extras:
        extras = {}
        want = set(args.extras.split(",")) if args.extras != "all" else None
        run = lambda name: want is None or name in want   # noqa: E731
        if run("headline_other"):   # the same headline workload in the fp32-faithful bf16x6 split
            other = "bf16x6" if eng.precision != "bf16x6" else "f16x3"
            with eng.precision_override(other):
                mo = measure(head, eng, n, 3, 1, 1, dev)
            extras[f"headline_{other}"] = extra_record(mo, "variants_per_s", n, WIN_PER_VARIANT_200, other)
        if run("cfg1"):   # configs[1]: 1k SNVs, shift 0 (per-window pair path)
            c1 = ShiftSweep(pipe, genome, 1000, 1, shift_order(0), dev)
            extras["cfg1_1k_snv_shift0"] = extra_record(measure(c1, eng, 1000, 10, 3, 1, dev, segments=False),
                                                        "variants_per_s", 1000, 4, eng.precision)
            del c1
        if run("cfg2"):   # configs[2]: +-800 sweep (9 shifts, segment path)
            c2 = ShiftSweep(pipe, genome, 400, 101, shift_order(800), dev)
            extras["cfg2_shift_sweep_800"] = extra_record(measure(c2, eng, 400, 2, 1, 1, dev), "variants_per_s",
                                                          400, 36, eng.precision)
            del c2
        if run("cfg4"):
            extras["cfg4_tss_features"] = tss_workload(eng, genome, pipe.dg, dev)
        if run("operator_api"):
            extras["operator_api"] = operator_api(model, genome, dev)
        if run("cli_streamed"):
            extras["cli_streamed"] = cli_streamed(genome)
        if run("replicate_rank"):
            extras["replicate_rank"] = replicate_rank(genome)
        if run("cli_e2e") and not args.no_e2e:
            extras["cli_e2e"] = cli_e2e()
        if run("hbm"):
            extras["hbm_reductions"] = hbm_reductions(dev)
        rec["extra_workloads"] = extras
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from expecto_amd.encode import seqs_to_codes
        rng = np.random.default_rng(5)
        sample = []
        for _ in range(512):
            c = sorted(genome)[int(rng.integers(0, len(genome)))]
            p = int(rng.integers(30000, len(genome[c]) - 30000)) + int(rng.choice(SHIFTS_200))
            sample.append(genome[c][p - 1000:p + 1000].decode())
        rec["cpu_baseline"] = cpu_baseline(sd_cpu, seqs_to_codes(sample), args.cpu_seconds, WIN_PER_VARIANT_200)
        rec["speedup_vs_cpu_baseline"] = rec["value"] / rec["cpu_baseline"]["value"]
    if world > 1:
        rec["cfg3_rank_shard"] = cfg3_rank_shard(pipe, eng, genome, rank, world, dev)
    if rank == 0:
        print(json.dumps(rec))
    if world > 1:
        torch.distributed.destroy_process_group()


# Handle workspace (windows per per-window chunk and per FC slice of the segment path; round 1:
# 4000 -> 8192 windows and 24 -> 96 variants per step took the 200-window workload from 799 to
# 881 variants/s).  Round 2: the 96 variants' segments of a strand run as one chunk.
MAX_BATCH = 8192

if __name__ == "__main__":
    main()
