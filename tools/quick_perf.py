"""Dev probe: time the HIP Beluga forward and print per-layer device times."""
import sys, time
import torch
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__file__)))
from expecto_amd import beluga
from oracle.beluga_np import macs_per_window

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
mb = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
m = beluga.seeded(0, max_batch=mb).cuda()
codes = torch.randint(0, 4, (n, 2000), dtype=torch.uint8, device="cuda")
eng = m.engine()
out = eng.forward_codes(codes, 0)
torch.cuda.synchronize()
t = time.time(); out = eng.forward_codes(codes, 0); torch.cuda.synchronize(); dt = time.time() - t
print(f"n={n} max_batch={mb}: {dt*1e3:.1f} ms, {n/dt:.1f} windows/s, {2*macs_per_window()*n/dt/1e12:.1f} TFLOP/s")
eng.set_profiling(True)
out = eng.forward_codes(codes, 0)
torch.cuda.synchronize()
for k, (ms, c, _m) in eng.layer_times().items():
    print(f"  {k:11s} {ms:9.2f} ms  ({c} launches)")
