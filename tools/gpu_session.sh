#!/bin/bash
# One GPU-box session, the steps named in $STEPS (comma-separated, run in this order):
#
#   tests    pytest -m gpu (one process, per-test time limit)
#   smoke    __graft_entry__.smoke()
#   bench    python bench.py (default K/W; extras + cpu_baseline)           -> gpurun_out/bench.log
#   prof     rocprofv3 --kernel-trace --stats of the headline               -> gpurun_out/prof_$TAG/
#   pmc      FETCH_SIZE, WRITE_SIZE and SQ busy counters, one --pmc pass each (same command)
#   power    rocm-smi power / clock samples during 200 headline steps       -> gpurun_out/power.log
#   gb       tools/gemm_bench $GB_ARGS (e.g. "8192 5 fc1 8")                -> gpurun_out/gb.log
#   gbpmc    SQ stall counter sets of gemm_bench $GB_ARGS, VARIANT=$V
#   ckstamp  tools/ck_bench per conv layer with the stamp build (barrier / vmcnt / epilogue shares) -> ck_<layer>.log
#   convpmc  SQ stall counter sets of the headline's conv kernels (beluga_conv_h3p only)  -> convpmc_<i>_$TAG/
#   sb       tools/small_batch_probe.py: batch 32 / 200 / 512 Beluga.forward, device-resident and the
#            reference's H2D + forward + D2H pattern; then a kernel trace of it -> sb.log, sbt/
#   writes   tools/write_probe.py, 8 writers at configs[3]'s full size: plain, staggered, staggered with 4 threads
#
#   STEPS=tests,bench TAG=r04 /usr/local/graft/bin/gpurun -- bash tools/gpu_session.sh
#
# Every step runs under its own time limit; the session stops at the first step that ends by a
# signal / time limit / fault (exit >= 124), so nothing more touches the GPU after a fault.
# Test failures (exit 1) do not stop the later measurement steps.  `tools/collect_profiles.py
# gpurun_out $TAG` turns the prof/pmc outputs into profiles/$TAG/.
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p $OUT
TAG=${TAG:-r04}
STEPS=${STEPS:-tests,smoke,bench}
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" >> $OUT/steps.log
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> $OUT/steps.log
  if [ $rc -ge 124 ]; then echo "stopping after $name (rc=$rc)" >> $OUT/steps.log; exit $rc; fi
  return 0
}
has() { [[ ",$STEPS," == *",$1,"* ]]; }
cd $REPO
B="python3 $REPO/bench.py --no-extras --no-cpu-baseline"
has tests && run gpu_tests 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
has smoke && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
has bench && run bench 900 python -u bench.py
if has prof; then
  run prof_$TAG 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- $B --steps 5 --warmup 2
fi
if has pmc; then
  run pmc_fetch_$TAG 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch_$TAG -o run -- $B --steps 1 --warmup 1
  run pmc_write_$TAG 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write_$TAG -o run -- $B --steps 1 --warmup 1
  run pmc_sq_$TAG 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace \
    --output-format csv -d $OUT/pmc_sq_$TAG -o run -- $B --steps 1 --warmup 1
fi
if has power; then
  ( for i in $(seq 1 60); do rocm-smi --showpower --showclocks --showtemp 2>/dev/null | grep -E "Power|sclk|Temperature"; echo "---"; sleep 0.5; done ) > $OUT/power.log 2>&1 &
  SAMPLER=$!
  run power_bench 300 $B --steps 200 --warmup 3
  kill $SAMPLER 2>/dev/null
fi
has gb && run gb 300 tools/gemm_bench ${GB_ARGS:-2000 5 conv2}
if has gbpmc; then
  export VARIANT=${V:-}
  i=0
  for ctrs in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
              "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
              "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS" \
              "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU"; do
    i=$((i+1))
    run gbpmc_$i 180 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $OUT/gbpmc_$i -o run -- \
      tools/gemm_bench ${GB_ARGS:-1000 2 conv2}
  done
fi
if has ckstamp; then
  run ck_conv3 200 tools/ck_bench 2000 3 conv3
  run ck_conv4 200 tools/ck_bench 2000 3 conv4
  run ck_conv5 200 tools/ck_bench 16000 3 conv5
  run ck_conv6 200 tools/ck_bench 16000 3 conv6
fi
if has convpmc; then
  i=0
  for ctrs in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE" \
              "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
              "SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_VMEM SQ_WAVES GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    run convpmc_${i}_$TAG 300 rocprofv3 --pmc $ctrs --kernel-include-regex beluga_conv_h3p --kernel-trace \
      --output-format csv -d $OUT/convpmc_${i}_$TAG -o run -- $B --steps 1 --warmup 1
  done
fi
if has sb; then
  run sb 300 python -u tools/small_batch_probe.py
  run sbt 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/sbt -o run -- python3 $REPO/tools/small_batch_probe.py --trace
fi
if has writes; then
  run writes_plain 600 python -u tools/write_probe.py --ranks 8 --variants 100000 --dir /tmp/wp
  run writes_stagger 600 python -u tools/write_probe.py --ranks 8 --variants 100000 --dir /tmp/wp --stagger
  run writes_stagger_t4 600 python -u tools/write_probe.py --ranks 8 --variants 100000 --dir /tmp/wp --stagger --threads 4
fi
echo "=== done" >> $OUT/steps.log
