#!/bin/bash
# Same-box power / clock during 200 headline steps, conv2 on the MFMAs (EXPECTO_CONV2_TABLE=0) vs
# the k-mer gather (1), alternating: gpurun_out/power_ab_<i>_table<t>.{smi,bench}.log
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
i=0
for t in 0 1 0 1; do
  i=$((i+1))
  ( for k in $(seq 1 40); do rocm-smi --showpower --showclocks 2>/dev/null | grep -E "Power|sclk"; echo "---"; sleep 0.5; done ) \
    > gpurun_out/power_ab_${i}_table$t.smi.log 2>&1 &
  S=$!
  EXPECTO_CONV2_TABLE=$t timeout -k 10 300 python3 bench.py --no-extras --no-cpu-baseline --steps 200 --warmup 3 \
    > gpurun_out/power_ab_${i}_table$t.bench.log 2>&1 || exit $?
  kill $S 2>/dev/null
done
