#!/bin/bash
# batched epilogue factor loads (gemm_bench, bitwise vs h3c), GPU tests, pipeline A/B sweep
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p $OUT
cd $REPO
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" >> $OUT/steps_d.log
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> $OUT/steps_d.log
  if [ $rc -ge 124 ]; then echo "stopping after $name (rc=$rc)" >> $OUT/steps_d.log; exit $rc; fi
  return 0
}
for s in conv3 conv6 conv2 conv5 conv4; do
  run epi_$s 240 env VARIANT=h3c,h3r,h3r_oldepi,h3p4_pf,h3p4_pf_oldepi,h3p4_pf_noepi tools/gemm_bench 2000 5 $s
done
run gpu_tests 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run sweep 600 python -u tools/knob_sweep.py ${SWEEP:-EXPECTO_FC_WIDE=0,1 EXPECTO_CONV_TILE=0,256} --steps 5 --rounds 3
echo done >> $OUT/steps_d.log
