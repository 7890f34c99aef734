import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


# Parity criterion (BASELINE.json north_star: within 1e-4 relative fp32):
# |got - want| <= RTOL*|want| + ATOL element-wise, and max|diff| / max|want| <= RTOL.
RTOL = 1e-4
ATOL = 1e-5


def assert_close(got, want, rtol=RTOL, atol=ATOL, what=""):
    import numpy as np
    got = np.asarray(got, np.float64)
    want = np.asarray(want, np.float64)
    assert got.shape == want.shape, (what, got.shape, want.shape)
    err = np.abs(got - want)
    bound = rtol * np.abs(want) + atol
    bad = err > bound
    assert not bad.any(), f"{what}: {bad.sum()} elements out of tolerance, max err {err.max():.3g}"
    if want.size and np.abs(want).max() > 0:
        assert err.max() / np.abs(want).max() <= rtol, f"{what}: max err ratio {err.max() / np.abs(want).max():.3g}"


def run_in_roles(eng, fn):
    """{role: fn()} with the engine's per-window forwards in each block-Karatsuba FC1 role 0..3 and
    the direct FC1 (role 4, the default; include/expecto_hip.h expecto_beluga_set_fc1_role); reset
    to 4 after."""
    ys = {}
    try:
        for r in range(5):
            eng.set_fc1_role(r)
            ys[r] = fn().clone()
    finally:
        eng.set_fc1_role(4)
    return ys


def sweep_in_roles(eng, fn, shifts, pairs=True):
    """Per-window sweep predictions y[2 strands, 2 alleles, S, n, 2002] (fn() with rows="shift")
    with window (strand, shift j) taken in the FC1 role the segment path (segment pairs if `pairs`)
    gives it (pipeline.sweep_roles): what the segment path must equal bit for bit."""
    from expecto_amd.pipeline import sweep_roles
    ys = run_in_roles(eng, fn)
    roles = sweep_roles(shifts, pairs)
    out = ys[0].clone()
    for s in range(2):
        for j in range(len(shifts)):
            out[s, :, j] = ys[int(roles[s, j])][s, :, j]
    return out
