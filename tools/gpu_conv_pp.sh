#!/bin/bash
# Persistent producer / consumer conv kernel (beluga_conv_h3pp) against the per-tile one
# (beluga_conv_h3p<.., 256, 4>) and the 384-row h3r, bitwise-checked against h3c, conv2..conv6.
set -o pipefail
mkdir -p gpurun_out
for s in ${SHAPES:-conv3 conv4 conv5 conv6 conv2}; do
  VARIANT=${VARIANTS:-h3c,h3r,h3p4_pf,h3pp,h3p4_pf_noepi,h3pp_noepi,h3pp_stagger} timeout -k 10 240 tools/gemm_bench ${NB:-2000} 5 $s \
    > gpurun_out/convpp_$s.log 2>&1 || exit $?
done
echo done > gpurun_out/convpp.done
