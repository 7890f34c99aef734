# tools/mfma_power_probe under a rocm-smi power/clock sampler (GPU box)
mkdir -p gpurun_out
( for i in $(seq 1 40); do rocm-smi --showpower --showclocks 2>/dev/null | grep -E "Power|sclk" ; echo "--- $(date +%s.%N)"; sleep 0.25; done ) > gpurun_out/mfma_power.log 2>&1 &
SAMPLER=$!
timeout -k 10 120 ./tools/mfma_power_probe "$@" > gpurun_out/mfma_probe.jsonl 2> gpurun_out/mfma_probe.err
rc=$?
kill $SAMPLER 2>/dev/null
exit $rc
