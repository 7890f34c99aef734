# Same-box A/B of the headline: _ab/old (a worktree of an earlier commit, built in place; OLD_DIR=.
# for this tree) vs this tree, alternating rounds, with OLD_ENV / NEW_ENV (VAR=value ...) set for
# each side; one JSON summary line per run in gpurun_out/ab.log
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab.log
for r in ${ROUNDS:-1 2 3}; do
  for t in old new; do
    d=$([ $t = old ] && echo "${OLD_DIR:-_ab/old}" || echo .)
    e=$([ $t = old ] && echo "${OLD_ENV:-}" || echo "${NEW_ENV:-}")
    (cd $d && env $e timeout -k 10 300 python -u bench.py --steps ${STEPS:-8} --warmup 2 --no-extras --no-cpu-baseline) > gpurun_out/ab_$t.json 2> gpurun_out/ab_err.log || exit $?
    python - $t >> gpurun_out/ab.log <<'PY'
import json, sys
t = sys.argv[1]
s = open(f"gpurun_out/ab_{t}.json").read()
d = json.loads(s[s.index('{"metric'):].split("\n")[0])
print(json.dumps({"tree": t, "value": round(d["value"], 1), "ms": round(d["ms_per_step"], 2),
                  "layers": {k: round(v, 2) for k, v in d["layer_ms_per_step"].items() if "delta" not in k}}))
PY
  done
done
