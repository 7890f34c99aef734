mkdir -p gpurun_out
: > gpurun_out/vsweep.jsonl
for r in 1 2; do
  for v in 96 192 144; do
    timeout -k 10 240 python -u bench.py --steps 6 --warmup 2 --no-extras --no-cpu-baseline --variants $v > gpurun_out/vs_$v.json 2> gpurun_out/vs_err.log || exit $?
    python -c "
import json; s=open('gpurun_out/vs_$v.json').read(); d=json.loads(s[s.index('{\"metric'):].split(chr(10))[0])
print(json.dumps({'variants': $v, 'round': $r, 'value': round(d['value'],1), 'ms': round(d['ms_per_step'],2), 'fb': d['f16_fallback_steps']}))" >> gpurun_out/vsweep.jsonl
  done
done
