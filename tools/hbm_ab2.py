"""Same-process A/B of the HBM-bound reductions of two builds of the library (e.g. the HEAD
build against an older one copied to _abtmp/): bench.hbm_reductions' three workloads through
each library's C-ABI in alternating rounds, outputs compared bit for bit.

    python tools/hbm_ab2.py _abtmp/libexpecto_hip_old.so [rounds]
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from expecto_amd import _lib, features  # noqa: E402
from expecto_amd.pipeline import shift_order  # noqa: E402


def bind(path):
    lib = ctypes.CDLL(path)
    for name, (res, args) in _lib.SIGNATURES.items():
        if hasattr(lib, name):
            f = getattr(lib, name)
            f.restype, f.argtypes = res, args
    return lib


def main():
    old_path = sys.argv[1]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    libs = {"new": bind(os.path.join(REPO, "expecto_amd", "libexpecto_hip.so")), "old": bind(old_path)}
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    G, S, F = 1000, 200, 2002
    fwd = torch.rand((G, S, F), device=dev, generator=g)
    rc = torch.rand((G, S, F), device=dev, generator=g)
    w = torch.from_numpy(features.tss_pos_weights()).to(dev)
    n_var, S9 = 20000, 9
    eff = torch.rand((S9, n_var, F), device=dev, generator=g)
    rng = np.random.default_rng(4)
    dist = torch.from_numpy(rng.integers(-20000, 20000, n_var).astype(np.int64)).to(dev)
    plus = torch.from_numpy(rng.integers(0, 2, n_var).astype(np.uint8)).to(dev)
    sh = torch.tensor(shift_order(800), dtype=torch.int32, device=dev)
    lut = torch.from_numpy(features.decay_table(dist.cpu().numpy(), plus.cpu().numpy().astype(bool),
                                                shift_order(800))).to(dev)
    NS = 96
    outs = {t: {"tss": torch.empty((G, 10 * F), dtype=torch.float64, device=dev),
                "variant": torch.empty((n_var, 10 * F), dtype=torch.float64, device=dev),
                "sed": torch.empty((NS, 10 * (F + 1)), dtype=torch.float64, device=dev)} for t in libs}
    st = _lib.stream_ptr()

    def run(t, k):
        lib, o = libs[t], outs[t][k]
        if k == "tss":
            r = lib.expecto_tss_reduce(_lib.dptr(fwd), _lib.dptr(rc), _lib.dptr(w), G, S, F, _lib.dptr(o), st)
        elif k == "variant":
            r = lib.expecto_variant_reduce_lut(_lib.dptr(eff), _lib.dptr(dist), _lib.dptr(plus), _lib.dptr(sh), S9,
                                               n_var, F, _lib.dptr(lut), lut.shape[1], _lib.dptr(o), st)
        else:
            r = lib.expecto_shift_reduce(_lib.dptr(fwd[:NS]), _lib.dptr(rc[:NS]), _lib.dptr(w), NS, S, F, 3,
                                         _lib.dptr(o), st)
        assert r == 0, (t, k, r)

    nbytes = {"tss": 2 * G * S * F * 4 + G * 10 * F * 8, "variant": S9 * n_var * F * 4 + n_var * 10 * F * 8,
              "sed": 2 * NS * S * F * 4 + NS * 10 * (F + 1) * 8}
    res = {t: {k: [] for k in nbytes} for t in libs}
    for r in range(rounds):
        for t in (("old", "new") if r % 2 == 0 else ("new", "old")):
            for k in nbytes:
                run(t, k)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    run(t, k)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / 5
                res[t][k].append(nbytes[k] / (ms * 1e-3) / 8e12)
    same = {k: bool(torch.equal(outs["old"][k], outs["new"][k])) for k in nbytes}
    print(json.dumps({"frac_of_8TBps": {t: {k: [round(x, 3) for x in v] for k, v in d.items()} for t, d in res.items()},
                      "bitwise_equal": same}))


if __name__ == "__main__":
    main()
