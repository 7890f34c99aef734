set -o pipefail
mkdir -p gpurun_out
for s in ${SHAPES:-conv2 conv3}; do
  timeout -k 10 120 tools/gemm_bench 1000 5 $s > gpurun_out/gb_$s.log 2>&1 || exit $?
done
