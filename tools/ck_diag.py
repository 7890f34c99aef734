"""Diagnostic: segment-pair alt patches with the pair Karatsuba conv3 / conv4 on and off, against
per-window forwards in the matching conv role (which SNV positions / layers differ)."""
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from expecto_amd import beluga  # noqa: E402


def run(env_off):
    os.environ["EXPECTO_CONV_KARATSUBA"] = "0" if env_off else "1"
    m = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=300).cuda()
    eng = m.engine()
    rng = np.random.default_rng(43)
    L = 2000 + 1600
    q = np.array([0, 3, 7, 30, 31, 500, 1234, 1799, 1800, 2001, 3000, L - 40, L - 9, L - 2, L - 1], np.int32)
    n = q.size
    ref = torch.from_numpy(rng.integers(0, 5, (n, L)).astype(np.uint8)).cuda()
    alt_code = torch.from_numpy(((ref.cpu().numpy()[np.arange(n), q] + 1 + rng.integers(0, 3, n)) % 4).astype(np.uint8)).cuda()
    alt = ref.clone()
    alt[torch.arange(n), torch.from_numpy(q).long()] = alt_code
    offs = np.array([0, 8, 200, 792, 800, 1000, 1592, 1600], np.int32)
    S = offs.size
    v_i, j_i = np.meshgrid(np.arange(n), np.arange(S), indexing="ij")
    win_seg, win_off, win_row = v_i.ravel().astype(np.int32), offs[j_i.ravel()], (j_i * n + v_i).ravel().astype(np.int32)
    y = torch.full((2, 2, S * n, 2002), float("nan"), device="cuda")
    yf = y.view(4 * S * n, 2002)
    eng.forward_segment_pairs(ref, L, q, alt_code, win_seg, win_off, win_row, yf[0:], yf[S * n:], 2 * S * n)
    from expecto_amd.pipeline import fc1_role
    n_alt = int(sum(((o <= q) & (q < o + 2000)).sum() for o in offs))
    print("n_alt", n_alt, "of", S * n, "-> fc1 role 4" if 3 * n_alt > S * n else "")
    wins = torch.stack([alt[:, o:o + 2000] for o in offs], 0).reshape(S * n, 2000).contiguous()
    for r in range(5):
        eng.set_fc1_role(r)
        yw = eng.forward_codes(wins, 2).view(2, S, n, 2002).clone()
        if r == 0:
            ys = {0: yw}
        ys[r] = yw
    eng.set_fc1_role(0)
    role = (lambda o, sd: 4) if 3 * n_alt > S * n else (lambda o, sd: fc1_role(int(o), L, sd == 1))
    want = torch.stack([torch.stack([ys[role(o, sd)][sd, j] for j, o in enumerate(offs)]) for sd in range(2)]).view(2, S * n, 2002)
    d = (y[:, 1] - want).abs().amax(-1).view(2, S, n).cpu().numpy()
    print("karatsuba off" if env_off else "karatsuba on", "bad (strand, offset idx, q):",
          [(s, j, int(q[v])) for s, j, v in zip(*np.nonzero(d))][:40])


run(True)
run(False)
