# iterate: GPU tests of the forward / pipelines / precision, then one headline bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_forward.py tests/test_gpu_pipelines.py tests/test_gpu_precision.py} > gpurun_out/t1.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-extras --no-cpu-baseline > gpurun_out/b1.log 2>&1
