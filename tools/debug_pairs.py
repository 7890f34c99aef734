import sys, os, math
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from expecto_amd import beluga
eng = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=300).cuda().engine()
eng.set_precision("fp32")
rng = np.random.default_rng(7)
pos = np.array([0, 5, 100, 308, 309, 310, 500, 998, 999, 1000, 1500, 1690, 1700, 1701, 1990, 1999], np.int32)
n = pos.size
ref = torch.from_numpy(rng.integers(0, 5, (n, 2000)).astype(np.uint8)).cuda()
for label, alt in (("alt==ref", ref.clone()), ("snv", None)):
    if alt is None:
        alt = ref.clone()
        nb = torch.from_numpy(((ref.cpu().numpy()[np.arange(n), pos] + 1) % 4).astype(np.uint8)).cuda()
        alt[torch.arange(n), torch.from_numpy(pos).long()] = nb
    for mode in (0, 2):
        S = 2 if mode == 2 else 1
        y = torch.empty((S, 2, n, 2002), device="cuda")
        yv = y.view(S * 2 * n, 2002)
        eng.forward_pairs(ref, alt, pos, yv[0:], yv[n:], 2 * n, mode)
        want_alt = eng.forward_codes(alt, mode).view(S, n, 2002)
        want_ref = eng.forward_codes(ref, mode).view(S, n, 2002)
        d = (y[:, 1] - want_alt).abs().amax(-1).cpu().numpy()
        dr = (y[:, 0] - want_ref).abs().amax(-1).cpu().numpy()
        print(label, "mode", mode, "ref max", dr.max(), "alt per window:", np.array2string(d, precision=2, max_line_width=200))
