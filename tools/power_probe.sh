# Sample board power / clocks while the headline bench runs (is the chip power-limited?)
mkdir -p gpurun_out
( for i in $(seq 1 60); do rocm-smi --showpower --showclocks --showtemp 2>/dev/null | grep -E "Power|sclk|Temperature|fclk|mclk" ; echo "---"; sleep 0.5; done ) > gpurun_out/power.log 2>&1 &
SAMPLER=$!
timeout -k 10 300 python -u bench.py --steps 200 --warmup 3 --no-extras --no-cpu-baseline > gpurun_out/power_bench.log 2>&1
rc=$?
kill $SAMPLER 2>/dev/null
rocm-smi --showmaxpower 2>/dev/null | grep -i power >> gpurun_out/power.log
exit $rc
