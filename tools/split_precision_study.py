"""Dev study: does split-bf16 (bf16x3) arithmetic meet the parity bar on Beluga?

Emulates an MFMA bf16 GEMM with fp32 accumulation: each operand x = hi + lo with
hi = bf16(x), lo = bf16(x - hi); products of bf16 values are exact in fp32.
Reports max |delta| / (1e-4|y| + 1e-5) on outputs and on alt-ref diffs (must be < 1).
"""
import math, sys, os
import numpy as np, torch, torch.nn.functional as F
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import weights
from oracle.beluga_np import CONV_KEYS, FC1_KEY, FC2_KEY
from expecto_amd import synthetic
from expecto_amd.encode import seqs_to_codes, codes_to_onehot

def split(t):
    hi = t.to(torch.bfloat16).float()
    lo = (t - hi).to(torch.bfloat16).float()
    return hi, lo

def split3(t):
    a = t.to(torch.bfloat16).float()
    b = (t - a).to(torch.bfloat16).float()
    c = (t - a - b).to(torch.bfloat16).float()
    return a, b, c

def op3(f, x, w, terms):
    if terms == 6:   # 3-way split, products of combined order <= 2 (x0y0 x0y1 x1y0 x0y2 x1y1 x2y0)
        x0, x1, x2 = split3(x); w0, w1, w2 = split3(w)
        return f(x0, w0) + (f(x0, w1) + f(x1, w0)) + (f(x0, w2) + f(x1, w1) + f(x2, w0))
    xh, xl = split(x); wh, wl = split(w)
    out = f(xh, wh)
    if terms >= 3:
        out = out + f(xh, wl) + f(xl, wh)
    if terms >= 4:
        out = out + f(xl, wl)
    return out

def forward(sd, x, mode):
    h = x
    for i, key in enumerate(CONV_KEYS):
        w, b = sd[key + ".weight"], sd[key + ".bias"]
        if i == 0 or mode == "fp32":
            z = F.conv2d(h, w)
        else:
            z = op3(F.conv2d, h, w, mode)
        h = F.relu(z + b.view(1, -1, 1, 1))
        if i in (1, 3):
            h = F.max_pool2d(h, (1, 4), (1, 4))
    h = h.reshape(h.shape[0], -1)
    fc = lambda a, w: F.linear(a, w)
    lin = (lambda a, w: fc(a, w)) if mode == "fp32" else (lambda a, w: op3(fc, a, w, mode))
    h = F.relu(lin(h, sd[FC1_KEY + ".weight"]) + sd[FC1_KEY + ".bias"])
    h = lin(h, sd[FC2_KEY + ".weight"]) + sd[FC2_KEY + ".bias"]
    return torch.sigmoid(h)

torch.set_num_threads(8)
sd = weights.seeded_state_dict(0)
g = synthetic.genome_bytes(n_contigs=1, contig_len=200000, seed=3)["chr1"].decode()
rng = np.random.default_rng(0)
refs, alts = [], []
for p in rng.integers(2000, 190000, 12):
    s = g[p - 1000:p + 1000]
    base = s[999].upper()
    alt = "ACGT".replace(base, "")[0] if base in "ACGT" else "A"
    refs.append(s); alts.append(s[:999] + alt + s[1000:])
codes = seqs_to_codes(refs + alts)
x = torch.from_numpy(codes_to_onehot(codes, with_rc=False).astype(np.float32)).unsqueeze(2)
with torch.no_grad():
    y64 = None
    base = forward({k: v.double() for k, v in sd.items()}, x.double(), "fp32")
    for mode in ("fp32", 3, 6):
        y = forward(sd, x, mode).double()
        n = len(refs)
        d_ref = base[n:] - base[:n]
        d = y[n:] - y[:n]
        r1 = ((y - base).abs() / (1e-4 * base.abs() + 1e-5)).max().item()
        r2 = ((d - d_ref).abs() / (1e-4 * d_ref.abs() + 1e-5)).max().item()
        print(f"mode={mode}: max|dy|={float((y-base).abs().max()):.3g} ratio_y={r1:.3f}  max|ddiff|={float((d-d_ref).abs().max()):.3g} ratio_diff={r2:.3f}")
