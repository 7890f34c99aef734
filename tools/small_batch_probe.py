"""Beluga.forward at the reference's per-window batch sizes (chromatin.py:37-38 batch 32,
compute_expecto_features.py:115-122 batch 200, 512): wall time per device-resident forward, and
per call of the reference's own pattern (host one-hot -> .cuda() -> forward -> .cpu()).
    python tools/small_batch_probe.py            (plain timing)
    rocprofv3 --kernel-trace ... -- python tools/small_batch_probe.py --trace
      (then tools/small_batch_trace.py <kernel_trace.csv>: kernels of the 23rd forward per batch)"""
import os, sys; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import math, time, torch, numpy as np
from expecto_amd import beluga
trace = "--trace" in sys.argv
m = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=512).cuda()
eng = m.engine(); eng.set_overflow_check(deferred=False)
rng = np.random.default_rng(0)
for B in (32, 200, 512):
    codes = rng.integers(0, 4, (B, 2000))
    x = torch.zeros(B, 4, 1, 2000); x[torch.arange(B)[:, None], torch.from_numpy(codes), 0, torch.arange(2000)[None]] = 1
    xd = x.cuda()
    host = x.numpy().copy()
    for _ in range(3): m.forward(xd)
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(20): m.forward(xd)
    torch.cuda.synchronize(); dev = (time.perf_counter() - t) / 20 * 1e3
    if trace:
        print(B, "ms/forward", dev, flush=True)
        continue
    def api():
        return m.forward(torch.from_numpy(host).cuda()).cpu().numpy()
    for _ in range(3): api()
    t = time.perf_counter()
    for _ in range(40): api()
    el = (time.perf_counter() - t) / 40
    print(B, f"ms/forward {dev:.3f}  api (H2D+forward+D2H) {el * 1e3:.3f} ms = {B / el:.0f} windows/s", flush=True)
