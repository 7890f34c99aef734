mkdir -p gpurun_out
for sp in 10 20 40 10; do
  EXPECTO_FC1_SPLITS=$sp timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-extras --no-cpu-baseline > gpurun_out/b_$sp.log 2>&1 || exit $?
  python -c "import json; r=json.loads(open('gpurun_out/b_$sp.log').read().strip().splitlines()[-1]); print($sp, r['value'], r['ms_per_step'], r['layer_ms_per_step']['fc1'], r['layer_ms_per_step']['fc1_reduce'])" >> gpurun_out/splits.txt
done
