import os, sys; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import math, time, torch, numpy as np
from expecto_amd import beluga
m = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=512).cuda()
eng = m.engine(); eng.set_overflow_check(deferred=False)
rng = np.random.default_rng(0)
for B in (32, 200, 512):
    codes = rng.integers(0, 4, (B, 2000))
    x = torch.zeros(B, 4, 1, 2000); x[torch.arange(B)[:, None], torch.from_numpy(codes), 0, torch.arange(2000)[None]] = 1
    xd = x.cuda()
    for _ in range(3): m.forward(xd)
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(20): m.forward(xd)
    torch.cuda.synchronize(); print(B, "ms/forward", (time.perf_counter() - t) / 20 * 1e3, flush=True)
