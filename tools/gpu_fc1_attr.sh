#!/bin/bash
# FC1 read attribution: gemm_bench fc1 timing probes (A L2-hot vs B L2-hot)
# on dense and segment-like (Toeplitz, overlapping) A rows, then TCC hit/miss and FETCH_SIZE
# passes of one round (per-dispatch counters; dispatch order = variant order, two per variant).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
NB=${NB:-8192}
for s in fc1 fc1t; do
  timeout -k 10 180 tools/gemm_bench $NB 5 $s 8 > gpurun_out/fc1attr_$s.log 2>&1 || exit $?
done
for s in fc1 fc1t; do
  timeout -k 10 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv \
    -d gpurun_out/fc1attr_tcc_$s -o run -- tools/gemm_bench $NB 1 $s 8 > gpurun_out/fc1attr_tcc_$s.log 2>&1 || exit $?
  timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv \
    -d gpurun_out/fc1attr_fetch_$s -o run -- tools/gemm_bench $NB 1 $s 8 > gpurun_out/fc1attr_fetch_$s.log 2>&1 || exit $?
done
echo done > gpurun_out/fc1attr.done
