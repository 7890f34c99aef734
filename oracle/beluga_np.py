"""CPU restatement of the Beluga forward -- TEST INFRASTRUCTURE (oracle) ONLY.

Reference: ``Beluga.py:18-51`` (identical copies at ``chromatin.py:67-100``,
``compute_expecto_features.py:148-181``, ``replicate_expecto_features.py:112-145``).

    Conv(4->320,k8)-ReLU-Conv(320->320,k8)-ReLU-Drop-MaxPool(4,4)
    -Conv(320->480,k8)-ReLU-Conv(480->480,k8)-ReLU-Drop-MaxPool(4,4)
    -Conv(480->640,k8)-ReLU-Conv(640->640,k8)-ReLU-Drop-Flatten(c*106+t)
    -Linear(67840->2003)-ReLU-Linear(2003->2002)-Sigmoid

Dropout is the identity in eval mode (``chromatin.py:104``).  Convolutions are
``Conv2d`` with kernel ``(1,8)``, stride 1, no padding (``Beluga.py:23-37``);
pools are ``MaxPool2d((1,4),(1,4))`` in floor mode (``Beluga.py:28,34``).

Two restatements:

* ``forward_numpy``     -- plain numpy fp32 (im2col + sgemm), independent of torch.
* ``forward_torch_cpu`` -- the same graph in ``torch.nn.functional`` on the CPU
                           (oneDNN), i.e. the arithmetic the reference's CPU path
                           runs; used as ``bench.py``'s timed ``cpu_baseline``.
"""
from __future__ import annotations

import numpy as np

CONV_KEYS = ("model.0.0", "model.0.2", "model.0.6", "model.0.8", "model.0.12", "model.0.14")
FC1_KEY = "model.1.2.1"
FC2_KEY = "model.1.4.1"
INPUT_LEN = 2000
N_FEATURES = 2002


def _conv_k8_np(x: np.ndarray, w: np.ndarray, b: np.ndarray) -> np.ndarray:
    """x [B,Cin,L] f32, w [Cout,Cin,1,8] -> [B,Cout,L-7] (Beluga.py:23 Conv2d (1,8))."""
    B, cin, L = x.shape
    cout = w.shape[0]
    lo = L - 7
    w2 = w.reshape(cout, cin * 8).astype(np.float32)          # index ci*8+k
    out = np.empty((B, cout, lo), np.float32)
    for bi in range(B):
        # im2col [lo, cin*8] with index ci*8+k  <- x[ci, t+k]
        cols = np.lib.stride_tricks.sliding_window_view(x[bi], 8, axis=1)  # [cin, lo, 8]
        cols = np.ascontiguousarray(cols.transpose(1, 0, 2)).reshape(lo, cin * 8)
        out[bi] = (cols @ w2.T).T + b.astype(np.float32)[:, None]
    return out


def _maxpool4_np(x: np.ndarray) -> np.ndarray:
    """MaxPool2d((1,4),(1,4)) floor mode (Beluga.py:28,34)."""
    B, C, L = x.shape
    lo = L // 4
    return x[:, :, : lo * 4].reshape(B, C, lo, 4).max(axis=3)


def _relu(x):
    return np.maximum(x, np.float32(0))


def forward_numpy(sd: dict, x: np.ndarray) -> np.ndarray:
    """Beluga.forward (Beluga.py:50-51) for x [B,4,2000] or [B,4,1,2000] f32."""
    x = np.asarray(x, np.float32)
    if x.ndim == 4:
        x = x[:, :, 0, :]
    g = lambda k: np.asarray(sd[k], np.float32)
    h = x
    for i, key in enumerate(CONV_KEYS):
        h = _relu(_conv_k8_np(h, g(key + ".weight"), g(key + ".bias")))
        if i in (1, 3):
            h = _maxpool4_np(h)
    flat = h.reshape(h.shape[0], -1)                            # c*106 + t (Beluga.py:42)
    h = _relu(flat @ g(FC1_KEY + ".weight").T + g(FC1_KEY + ".bias"))
    h = h @ g(FC2_KEY + ".weight").T + g(FC2_KEY + ".bias")
    return (1.0 / (1.0 + np.exp(-h.astype(np.float64)))).astype(np.float32)


def forward_torch_cpu(sd: dict, x, threads: int | None = None):
    """Functional torch-CPU restatement of Beluga.forward (oneDNN arithmetic).

    ``sd`` holds torch tensors (the reference state-dict keys).
    """
    import torch
    import torch.nn.functional as F

    if threads is not None:
        torch.set_num_threads(threads)
    x = torch.as_tensor(x, dtype=sd[CONV_KEYS[0] + ".weight"].dtype)
    if x.dim() == 3:
        x = x.unsqueeze(2)
    with torch.no_grad():
        h = x
        for i, key in enumerate(CONV_KEYS):
            h = F.relu(F.conv2d(h, sd[key + ".weight"], sd[key + ".bias"]))
            if i in (1, 3):
                h = F.max_pool2d(h, (1, 4), (1, 4))
        h = h.reshape(h.shape[0], -1)
        h = F.relu(F.linear(h, sd[FC1_KEY + ".weight"], sd[FC1_KEY + ".bias"]))
        h = F.linear(h, sd[FC2_KEY + ".weight"], sd[FC2_KEY + ".bias"])
        return torch.sigmoid(h)


def macs_per_window() -> int:
    """Dense multiply-accumulates of one 2000 bp window."""
    total, L, cin = 0, INPUT_LEN, 4
    for i, cout in enumerate((320, 320, 480, 480, 640, 640)):
        L -= 7
        total += L * cout * cin * 8
        cin = cout
        if i in (1, 3):
            L //= 4
    total += 67840 * 2003 + 2003 * 2002
    return total
