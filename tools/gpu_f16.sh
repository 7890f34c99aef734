set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 tools/gemm_bench 1000 5 conv2 > gpurun_out/gb_conv2.log 2>&1 &&
timeout -k 10 120 tools/gemm_bench 1000 5 conv3 > gpurun_out/gb_conv3.log 2>&1 &&
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 ;
rc=$?; echo "tests rc=$rc" >> gpurun_out/gpu_tests.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --precision f16x3 --no-cpu-baseline > gpurun_out/bench_f16.log 2>&1
timeout -k 10 300 python tools/accuracy_gpu.py 24 > gpurun_out/accuracy.log 2>&1
