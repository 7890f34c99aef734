"""Seeded synthetic Beluga weights for golden vectors -- TEST INFRASTRUCTURE (oracle) ONLY.

The real ``resources/deepsea.beluga.pth`` is not available offline.
Golden vectors use ``torch.manual_seed(seed); Beluga()`` (default PyTorch init of the
layers declared at ``Beluga.py:23-45``, in declaration order) with every ``*.weight``
multiplied by ``gain`` (sqrt(6) by default, which spreads the sigmoid outputs over
[0.005, 0.993] like the real model's).

The layers are constructed here in the same order as the reference so the torch RNG
stream -- and therefore the weights -- are identical without importing the reference.
``tests/golden/weights_checksum.json`` pins them.
"""
from __future__ import annotations

import math

SHAPES = [
    ("model.0.0", "conv", 4, 320), ("model.0.2", "conv", 320, 320),
    ("model.0.6", "conv", 320, 480), ("model.0.8", "conv", 480, 480),
    ("model.0.12", "conv", 480, 640), ("model.0.14", "conv", 640, 640),
    ("model.1.2.1", "fc", 67840, 2003), ("model.1.4.1", "fc", 2003, 2002),
]


def seeded_state_dict(seed: int = 0, gain: float = math.sqrt(6.0)) -> dict:
    import torch
    from torch import nn

    torch.manual_seed(seed)
    sd = {}
    for key, kind, cin, cout in SHAPES:
        m = nn.Conv2d(cin, cout, (1, 8)) if kind == "conv" else nn.Linear(cin, cout)
        with torch.no_grad():
            m.weight.mul_(gain)
        sd[key + ".weight"] = m.weight.detach()
        sd[key + ".bias"] = m.bias.detach()
    return sd


def checksum(sd: dict) -> dict:
    import torch

    out = {}
    for k, v in sd.items():
        v64 = v.detach().double()
        out[k] = [float(v64.sum()), float((v64 * v64).sum()), float(v64.flatten()[: 97].sum())]
    return out
