# Same-box A/B of the HBM-bound reductions (bench.hbm_reductions): _ab/old (a worktree of an
# earlier commit, built in place) vs this tree, alternating rounds; one JSON line per run in
# gpurun_out/hbm_ab.jsonl
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/hbm_ab.jsonl
for r in ${ROUNDS:-1 2 3}; do
  for t in old new; do
    d=$([ $t = old ] && echo _ab/old || echo .)
    (cd $d && timeout -k 10 200 python -u -c "
import json, torch, bench
res = bench.hbm_reductions(torch.device('cuda'))
print(json.dumps({'tree': '$t', **{k: {'ms': round(v['ms'], 4), 'frac': round(v['frac'], 3)} for k, v in res.items()}}))
") >> gpurun_out/hbm_ab.jsonl 2> gpurun_out/hbm_ab_err.log || exit $?
  done
done
