"""HIP Beluga forward vs the reference golden vectors and the CPU oracle (gfx950 only)."""
import math
import os

import numpy as np
import pytest

from conftest import GOLDEN, assert_close

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=["bf16x6", "f16x3", "fp32"])
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
    """Every GEMM precision is fp32-accurate: error vs a float64 forward within 3x the
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
    assert_close(b.cpu().numpy(), c.cpu().numpy(), what="rebuilt engine (default precision) vs fixture")


def _f16_pair():
    """An f16x3 engine and a bf16x6 engine on the same seeded weights."""
    from expecto_amd import beluga
    a = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=64).cuda()
    b = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=64).cuda()
    a.engine().set_precision("f16x3")
    b.engine().set_precision("bf16x6")
    return a, b


def test_f16x3_calibration_and_no_fallback_on_genomic_windows():
    """Calibrated scales keep ordinary windows inside fp16 (no fallback), and the f16x3 result
    stays within the parity bar of the bf16x6 one."""
    import torch
    a, b = _f16_pair()
    n0, sx = a.engine().f16_state()
    assert len(sx) == 7 and all(-40 <= s <= 40 for s in sx), sx
    rng = np.random.default_rng(5)
    codes = torch.from_numpy(rng.integers(0, 5, (40, 2000)).astype(np.uint8)).cuda()
    ya = a.forward_codes(codes, 2).cpu().numpy()
    yb = b.forward_codes(codes, 2).cpu().numpy()
    assert a.engine().f16_state()[0] == n0
    assert_close(ya, yb, what="f16x3 vs bf16x6")


def test_f16x3_overflow_recomputes_with_bf16x6():
    """An activation that does not fit fp16 after scaling (here: inputs x 3e4 on the dense
    one-hot path, then a calibration target that puts every layer at the edge) makes the call
    fall back to bf16x6: the output equals the bf16x6 engine's bit for bit."""
    import torch
    a, b = _f16_pair()
    rng = np.random.default_rng(6)
    x = torch.from_numpy(rng.uniform(0, 3e4, (5, 4, 1, 2000)).astype(np.float32)).cuda()
    n0 = a.engine().f16_state()[0]
    ya = a.forward(x).cpu()
    yb = b.forward(x).cpu()
    assert a.engine().f16_state()[0] == n0 + 1
    assert torch.equal(ya, yb)
    a.engine().set_f16_target(20)
    codes = torch.from_numpy(rng.integers(0, 4, (8, 2000)).astype(np.uint8)).cuda()
    ya = a.forward_codes(codes, 0).cpu()
    yb = b.forward_codes(codes, 0).cpu()
    assert a.engine().f16_state()[0] == n0 + 2
    assert torch.equal(ya, yb)
    a.engine().set_f16_target(10)
    ya = a.forward_codes(codes, 0).cpu()
    assert a.engine().f16_state()[0] == n0 + 2
    assert_close(ya.numpy(), yb.numpy(), what="f16x3 after re-calibration")


def test_conv_tile_choice_is_bitwise(monkeypatch):
    """The f16x3 conv kernels of every tile shape (384-row: 4-wave pool / 8-wave ReLU; 256-row:
    4-wave pool / 8-wave ReLU) produce the same bits, so the per-launch choice (auto: by CU
    rounds) never changes a result: auto, all-256 and all-384 handles agree exactly."""
    import torch
    from expecto_amd import beluga
    rng = np.random.default_rng(11)
    codes = torch.from_numpy(rng.integers(0, 5, (150, 2000)).astype(np.uint8)).cuda()
    out = {}
    for tile in ("0", "256", "384"):
        monkeypatch.setenv("EXPECTO_CONV_TILE", tile)
        m = beluga.seeded(0, gain=math.sqrt(6.0), max_batch=300).cuda()
        m.engine().set_precision("f16x3")
        out[tile] = m.forward_codes(codes, 2).cpu()
        del m
    assert torch.equal(out["0"], out["256"])
    assert torch.equal(out["0"], out["384"])


def test_forward_into_4byte_aligned_output_equals_aligned(model):
    """A caller-owned output that is 4- but not 8-byte aligned takes fc2_reduce's one-value
    kernel instead of the 2-wide one (expecto_beluga_forward_* write straight into `out`):
    the same bits either way."""
    import torch
    from expecto_amd.encode import seqs_to_codes
    seqs, _ = _golden_forward()
    codes = torch.from_numpy(seqs_to_codes(seqs)).cuda()
    eng = model.engine()
    want = eng.forward_codes(codes).cpu().numpy()
    rows = want.shape[0]
    buf = torch.full((rows * 2002 + 1,), float("nan"), dtype=torch.float32, device="cuda")
    out = buf[1:].view(rows, 2002)
    assert out.data_ptr() % 8 == 4
    eng.forward_codes(codes, out=out)
    np.testing.assert_array_equal(out.cpu().numpy(), want)
