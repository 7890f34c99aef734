#!/bin/bash
# rocprofv3 evidence for the bench headline (same command as the roofline line):
#   kernel-trace stats, then FETCH_SIZE and WRITE_SIZE in separate PMC passes.
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
TAG=${1:-r01}
mkdir -p $OUT
export TMPDIR=/tmp
cd $REPO
set -o pipefail
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- \
  python3 $REPO/bench.py --steps 10 --warmup 3 --no-extras --no-cpu-baseline > $OUT/prof_$TAG.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch_$TAG -o run -- \
  python3 $REPO/bench.py --steps 2 --warmup 1 --no-extras --no-cpu-baseline > $OUT/pmc_fetch_$TAG.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write_$TAG -o run -- \
  python3 $REPO/bench.py --steps 2 --warmup 1 --no-extras --no-cpu-baseline > $OUT/pmc_write_$TAG.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace \
  --output-format csv -d $OUT/pmc_sq_$TAG -o run -- \
  python3 $REPO/bench.py --steps 2 --warmup 1 --no-extras --no-cpu-baseline > $OUT/pmc_sq_$TAG.log 2>&1 || exit $?
echo done > $OUT/profile_$TAG.done
