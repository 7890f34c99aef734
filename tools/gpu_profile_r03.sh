#!/bin/bash
# Round-3 evidence on one box: full bench line (extras + CPU baseline), then the rocprofv3
# kernel-trace / FETCH / WRITE / SQ passes of the headline command (tools/profile_round.sh), then
# board power during 200 headline steps.  Stops at the first failure.
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
TAG=${1:-r03}
mkdir -p $OUT
cd $REPO
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || exit $?
bash tools/profile_round.sh $TAG || exit $?
bash tools/power_probe.sh || exit $?
echo done > $OUT/profile_all.done
