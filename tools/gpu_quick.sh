# tests + one bench line (used while iterating)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/gpu_tests.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 600 python bench.py --steps 10 --warmup 3 ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bench.log 2>&1
