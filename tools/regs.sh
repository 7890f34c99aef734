# compile gemm_bench keeping the temps, print register / scratch use of the conv kernels
set -e
cd "$(dirname "$0")"
hipcc -O3 --offload-arch=gfx950 -std=c++17 gemm_bench.hip -o gemm_bench -save-temps=obj 2>&1 | grep -v warning | grep -i -A3 error || true
python3 - <<'PY'
import re
s=open('gemm_bench-hip-amdgcn-amd-amdhsa-gfx950.s').read()
for blk in s.split('.end_amdhsa_kernel')[:-1]:
    nm=re.search(r'\.amdhsa_kernel (\S+)',blk)
    if not nm or 'conv_h3' not in nm.group(1): continue
    v=re.search(r'\.amdhsa_next_free_vgpr (\d+)',blk).group(1)
    sp=re.search(r'\.amdhsa_private_segment_fixed_size (\d+)',blk).group(1)
    print(nm.group(1)[14:60], 'vgpr',v,'scratch',sp)
PY
cp gemm_bench-hip-amdgcn-amd-amdhsa-gfx950.s /tmp/gb.s
rm -f gemm_bench-hip-* gemm_bench-host-* gemm_bench.hip-hip-*
