#!/bin/bash
# rocprofv3 evidence for the bench headline (the same command as the roofline line):
#   kernel-trace stats, then FETCH_SIZE, WRITE_SIZE and SQ counters in separate PMC passes.
# Each pass runs the program itself after `--` under its own time limit; stops at the first failure.
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
TAG=${1:-r02}
shift
EXTRA="$@"
mkdir -p $OUT
export TMPDIR=/tmp
cd $REPO
set -o pipefail
B="python3 $REPO/bench.py --no-extras --no-cpu-baseline $EXTRA"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- \
  $B --steps 5 --warmup 2 > $OUT/prof_$TAG.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch_$TAG -o run -- \
  $B --steps 1 --warmup 1 > $OUT/pmc_fetch_$TAG.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write_$TAG -o run -- \
  $B --steps 1 --warmup 1 > $OUT/pmc_write_$TAG.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace \
  --output-format csv -d $OUT/pmc_sq_$TAG -o run -- $B --steps 1 --warmup 1 > $OUT/pmc_sq_$TAG.log 2>&1 || exit $?
echo done > $OUT/profile_$TAG.done
