#!/bin/bash
# GPU tests on the round-3 kernels, then the pipeline A/B of the new defaults, then gemm_bench fc1
# with the wide-tile FC kernel.  Stops at the first step that ends by a signal / timeout / fault.
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p $OUT
cd $REPO
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" >> $OUT/steps_b.log
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> $OUT/steps_b.log
  if [ $rc -ge 124 ]; then echo "stopping after $name (rc=$rc)" >> $OUT/steps_b.log; exit $rc; fi
  return 0
}
[[ ${STEPS:-tests,sweep,fcw} == *tests* ]] && run gpu_tests 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
[[ ${STEPS:-tests,sweep,fcw} == *fcw* ]] && run fcw 240 tools/gemm_bench 8192 5 fc1t 8
[[ ${STEPS:-tests,sweep,fcw} == *fcw* ]] && run stagger3 240 env VARIANT=h3c,h3p4_pf,h3pp,h3pp_stagger,h3p4_pf_noepi tools/gemm_bench 2000 5 conv3
[[ ${STEPS:-tests,sweep,fcw} == *fcw* ]] && run stagger6 240 env VARIANT=h3c,h3p4_pf,h3pp,h3pp_stagger,h3p4_pf_noepi tools/gemm_bench 2000 5 conv6
[[ ${STEPS:-tests,sweep,fcw} == *sweep* ]] && run sweep 600 python -u tools/knob_sweep.py ${SWEEP:-EXPECTO_FC_WIDE=0,1 EXPECTO_CONV_TILE=0,256} --steps 5 --rounds 3
echo done >> $OUT/steps_b.log
