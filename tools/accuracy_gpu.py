"""Accuracy of each GEMM precision against a float64 forward (GPU, dev tool).

    python tools/accuracy_gpu.py [n_pairs=24]

Seeded SNV ref/alt window pairs (golden-vector weights, x sqrt(6)); prints, per precision and
for the reference's own fp32 CPU forward (oneDNN), the max error against float64 on outputs
and on alt-ref diffs, as a fraction of the parity bound |d| <= 1e-4|y| + 1e-5 (conftest.py).
"""
import json
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from expecto_amd import beluga, synthetic  # noqa: E402
from expecto_amd.encode import codes_to_onehot, seqs_to_codes  # noqa: E402
from oracle import weights  # noqa: E402
from oracle.beluga_np import forward_torch_cpu  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
torch.set_num_threads(min(16, os.cpu_count() or 1))
sd = weights.seeded_state_dict(0)
g = synthetic.genome_bytes(n_contigs=1, contig_len=400000, seed=3)["chr1"].decode()
rng = np.random.default_rng(0)
refs, alts = [], []
for p in rng.integers(2000, 390000, n):
    s = g[p - 1000:p + 1000]
    base = s[999].upper()
    alt = "ACGT".replace(base, "")[rng.integers(0, 3)] if base in "ACGT" else "A"
    refs.append(s)
    alts.append(s[:999] + alt + s[1000:])
codes = seqs_to_codes(refs + alts)
x = torch.from_numpy(codes_to_onehot(codes, with_rc=False).astype(np.float32)).unsqueeze(2)
y64 = forward_torch_cpu({k: v.double() for k, v in sd.items()}, x.double()).numpy()
d64 = y64[n:] - y64[:n]


def ratios(y):
    y = y.astype(np.float64)
    d = y[n:] - y[:n]
    ry = np.max(np.abs(y - y64) / (1e-4 * np.abs(y64) + 1e-5))
    rd = np.max(np.abs(d - d64) / (1e-4 * np.abs(d64) + 1e-5))
    return {"ratio_y": float(ry), "ratio_diff": float(rd), "max_abs_err_y": float(np.abs(y - y64).max()),
            "max_abs_err_diff": float(np.abs(d - d64).max())}


out = {"pairs": n, "cpu_fp32_onednn": ratios(forward_torch_cpu(sd, x).numpy())}
m = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=2 * n).cuda()
xc = x.cuda()
for prec in ("fp32", "bf16x6", "f16x3"):
    m.engine().set_precision(prec)
    out[prec] = ratios(m.forward(xc).cpu().numpy())
print(json.dumps(out, indent=1))
