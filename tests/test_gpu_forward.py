"""HIP Beluga forward vs the reference golden vectors and the CPU oracle (gfx950 only)."""
import math
import os

import numpy as np
import pytest

from conftest import GOLDEN, assert_close

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=["bf16x6", "fp32"])
def model(request):
    import torch
    from expecto_amd import beluga
    m = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=96).cuda()
    m.engine().set_precision(request.param)
    yield m
    torch.cuda.synchronize()


@pytest.fixture(scope="module")
def cpu_sd():
    from oracle import weights
    return weights.seeded_state_dict(0)


def _golden_forward():
    z = np.load(os.path.join(GOLDEN, "forward.npz"))
    return [s.decode() for s in z["seqs"]], z["y"]


def test_forward_onehot_matches_reference_golden(model):
    import torch
    from expecto_amd.encode import encodeSeqs
    seqs, y = _golden_forward()
    x = torch.from_numpy(encodeSeqs(seqs).astype(np.float32)).unsqueeze(2).cuda()
    out = model.forward(x).cpu().numpy()
    assert_close(out, y, what="forward_onehot vs reference Beluga.forward")


def test_forward_codes_both_strands_matches_golden(model):
    import torch
    from expecto_amd.encode import seqs_to_codes
    seqs, y = _golden_forward()
    codes = torch.from_numpy(seqs_to_codes(seqs)).cuda()
    out = model.forward_codes(codes, strand_mode=2).cpu().numpy()
    assert_close(out, y, what="forward_codes(BOTH) vs reference")
    fwd = model.forward_codes(codes, strand_mode=0).cpu().numpy()
    rc = model.forward_codes(codes, strand_mode=1).cpu().numpy()
    assert_close(fwd, y[:3], what="fwd only")
    assert_close(rc, y[3:], what="rc only")


@pytest.mark.parametrize("n", [1, 7, 97, 250])
def test_forward_random_onehot_vs_cpu_oracle(model, cpu_sd, n):
    """Chunking (max_batch=96), odd batch sizes and M tails against the torch-CPU oracle."""
    import torch
    from oracle.beluga_np import forward_torch_cpu
    rng = np.random.default_rng(n)
    codes = rng.integers(0, 5, (n, 2000)).astype(np.uint8)
    from expecto_amd.encode import codes_to_onehot
    x = codes_to_onehot(codes, with_rc=False).astype(np.float32)
    got = model.forward(torch.from_numpy(x).unsqueeze(2).cuda()).cpu().numpy()
    idx = np.unique(np.r_[0, n - 1, rng.integers(0, n, min(n, 12))])
    want = forward_torch_cpu(cpu_sd, torch.from_numpy(x[idx]).unsqueeze(2)).numpy()
    assert_close(got[idx], want, what=f"random one-hot n={n}")


def test_forward_dense_float_input_vs_cpu_oracle(model, cpu_sd):
    """forward() accepts arbitrary fp32 input like the reference (not only one-hot)."""
    import torch
    from oracle.beluga_np import forward_torch_cpu
    rng = np.random.default_rng(11)
    x = rng.uniform(-1, 1, (3, 4, 1, 2000)).astype(np.float32)
    got = model.forward(torch.from_numpy(x).cuda()).cpu().numpy()
    want = forward_torch_cpu(cpu_sd, torch.from_numpy(x)).numpy()
    assert_close(got, want, what="dense input")


def test_accuracy_vs_float64(model, cpu_sd):
    """Both GEMM precisions are fp32-accurate: error vs a float64 forward within 3x the
    reference's own fp32 (oneDNN) error, on 9 random windows."""
    import torch
    from oracle.beluga_np import forward_torch_cpu
    from expecto_amd.encode import codes_to_onehot
    rng = np.random.default_rng(42)
    x = codes_to_onehot(rng.integers(0, 5, (9, 2000)).astype(np.uint8), with_rc=False).astype(np.float32)
    xt = torch.from_numpy(x).unsqueeze(2)
    y64 = forward_torch_cpu({k: v.double() for k, v in cpu_sd.items()}, xt.double()).numpy()
    y32 = forward_torch_cpu(cpu_sd, xt).numpy()
    got = model.forward(xt.cuda()).cpu().numpy()
    e_ref = np.abs(y32 - y64).max()
    e_got = np.abs(got - y64).max()
    assert e_got <= 3 * e_ref + 1e-6, (e_got, e_ref)


def test_empty_batch_and_errors(model):
    import torch
    out = model.forward(torch.zeros((0, 4, 1, 2000), device="cuda"))
    assert out.shape == (0, 2002)
    with pytest.raises(RuntimeError):
        model.forward(torch.zeros((2, 4, 1, 1999), device="cuda"))
    with pytest.raises(RuntimeError):
        model.forward(torch.zeros((2, 4, 1, 2000)))  # CPU tensor: no CPU path
    x = torch.zeros((2, 4, 1, 4000), device="cuda")[..., ::2]
    assert not x.is_contiguous()
    with pytest.raises(RuntimeError):
        model.forward(x)  # non-contiguous, like the reference's view() failure


def test_load_state_dict_rebuilds_engine(model):
    import torch
    from expecto_amd import beluga
    m2 = beluga.seeded(1, max_batch=16).cuda()
    x = torch.zeros((2, 4, 1, 2000), device="cuda")
    a = m2.forward(x).clone()
    m2.load_state_dict(model.state_dict())
    b = m2.forward(x)
    c = model.forward(x)
    assert not torch.allclose(a, b)
    assert torch.allclose(b, c, atol=1e-6)
