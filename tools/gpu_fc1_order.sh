#!/bin/bash
# FC1 dispatch orders (gemm_bench fc1): N tiles fastest per XCD vs grouped M tiles (m_fastest 3),
# plus FETCH_SIZE of one round (dispatch order = variant order, two per variant).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for nb in 8192 2816; do
  timeout -k 10 180 tools/gemm_bench $nb 7 fc1t 8 > gpurun_out/fc1order_$nb.log 2>&1 || exit $?
done
timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv \
  -d gpurun_out/fc1order_fetch -o run -- tools/gemm_bench 8192 1 fc1t 8 > gpurun_out/fc1order_fetch.log 2>&1 || exit $?
echo done > gpurun_out/fc1order.done
