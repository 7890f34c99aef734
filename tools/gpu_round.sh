#!/bin/bash
# One GPU-box session: gpu tests, smoke, bench, rocprofv3 kernel stats + PMC traffic passes.
# Stops at the first step that ends by a signal/timeout/fault (exit >= 124); test failures (1)
# do not stop the later measurement steps.
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p $OUT
TAG=${1:-r01}
STEPS=${STEPS:-tests,smoke,bench,accuracy,prof,pmc}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" >> $OUT/steps.log
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ge 124 ]; then echo "stopping after $name (rc=$rc)" >> $OUT/steps.log; exit $rc; fi
  return 0
}
cd $REPO
[[ $STEPS == *tests* ]] && run gpu_tests 900 python -m pytest tests -m gpu -x -q
[[ $STEPS == *smoke* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *bench* ]] && run bench 600 python bench.py --steps 10 --warmup 3
[[ $STEPS == *accuracy* ]] && run accuracy 300 python tools/accuracy_gpu.py 24
export TMPDIR=/tmp
if [[ $STEPS == *prof* ]]; then
  run prof_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- python3 $REPO/bench.py --steps 5 --warmup 2 --no-cpu-baseline
fi
if [[ $STEPS == *pmc* ]]; then
  run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch_$TAG -o run -- python3 $REPO/bench.py --steps 2 --warmup 1 --no-cpu-baseline
  run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write_$TAG -o run -- python3 $REPO/bench.py --steps 2 --warmup 1 --no-cpu-baseline
fi
echo "=== done" >> $OUT/steps.log
