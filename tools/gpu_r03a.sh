#!/bin/bash
# round-3 kernel experiments in one box session: FC1 dispatch orders, persistent conv kernel
set -o pipefail
bash tools/gpu_fc1_order.sh || exit $?
bash tools/gpu_conv_pp.sh || exit $?
