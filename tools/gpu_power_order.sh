#!/bin/bash
# MFMA operand-order power probe: rotating A and B vs B stable over 4 MFMAs (16x16x32), dense
# random and half-zero operands, board power sampled (tools/mfma_power_run.sh)
set -o pipefail
mkdir -p gpurun_out
bash tools/mfma_power_run.sh 3000000 0.0 || exit $?
mv gpurun_out/mfma_probe.jsonl gpurun_out/order_z0.jsonl; mv gpurun_out/mfma_power.log gpurun_out/order_z0_power.log
bash tools/mfma_power_run.sh 3000000 0.5 || exit $?
mv gpurun_out/mfma_probe.jsonl gpurun_out/order_z5.jsonl; mv gpurun_out/mfma_power.log gpurun_out/order_z5_power.log
