"""The operator API (Beluga.forward, the reference's own call: chromatin.py:266-279,
compute_expecto_features.py:115-122, Beluga.py:50-51) through the k-mer gather, and the k-mer
table state:

* exact one-hot floats (encodeSeqs' output) give forward_codes' bits, fwd and rc, across chunks;
* any other float input (a 0.5, a -0.0) keeps conv1 / conv2 on the MFMAs for the whole call;
* forward_codes after load_state_dict runs on tables rebuilt for the new weights (oracle parity);
* base codes >= 5 read as the zero column (code 4), as conv1 reads them, on every table path;
* a handle that cannot hold the tables says so (conv2_table_state, one stderr line) and stays at
  the parity bar; shared tables count once in device_bytes.
"""
import math
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, assert_close

pytestmark = pytest.mark.gpu


def _model(seed=0, max_batch=64, precision="f16x3", env=None, monkeypatch=None):
    from expecto_amd import beluga
    for k, v in (env or {}).items():
        monkeypatch.setenv(k, v)
    m = beluga.seeded(seed, gain=math.sqrt(6.0), max_batch=max_batch).cuda()
    m.engine().set_precision(precision)
    for k in (env or {}):
        monkeypatch.delenv(k)
    return m


def _codes(n, seed):
    rng = np.random.default_rng(seed)
    c = rng.integers(0, 4, (n, 2000)).astype(np.uint8)
    c[1, 300:700] = 4                      # an N run
    c[min(4, n - 1), ::53] = 4             # scattered N
    return c


def _onehot(codes):
    from expecto_amd.encode import codes_to_onehot
    return torch.from_numpy(codes_to_onehot(codes, with_rc=False).astype(np.float32)).unsqueeze(2).cuda()


@pytest.mark.parametrize("precision", ["f16x3", "bf16x6"])
def test_onehot_forward_equals_forward_codes_bitwise(precision):
    """150 windows over max_batch 64 (3 chunks): forward(one-hot) == forward_codes(FWD) and
    forward(rc one-hot, x[:, ::-1, :, ::-1]) == forward_codes(RC), bit for bit; and the oracle's
    values at the parity bar."""
    from oracle import weights
    from oracle.beluga_np import forward_torch_cpu
    m = _model(precision=precision)
    assert m.engine().conv2_table_state() == (True, "held")
    codes_np = _codes(150, 1)
    codes = torch.from_numpy(codes_np).cuda()
    x = _onehot(codes_np)
    y = m.forward(x)
    assert torch.equal(y, m.forward_codes(codes, 0))
    xr = torch.flip(x, dims=[1, 3]).contiguous()         # the reference's rc input (compute_expecto_features.py:116)
    assert torch.equal(m.forward(xr), m.forward_codes(codes, 1))
    idx = [0, 1, 4, 77, 149]
    want = forward_torch_cpu(weights.seeded_state_dict(0), x[idx].cpu()).numpy()
    assert_close(y[idx].cpu().numpy(), want, what=f"one-hot forward ({precision}) vs oracle")


@pytest.mark.parametrize("deferred", [False, True])
def test_non_onehot_input_keeps_the_mfma_path(monkeypatch, deferred):
    """A batch with one non-one-hot value (0.5, or a -0.0) runs conv1 / conv2 on the MFMAs for the
    whole call: the same bits as a handle with EXPECTO_ONEHOT_CODES=0; an exact one-hot batch
    differs from that handle (it takes the gather) and equals forward_codes.  Both overflow-check
    modes: per call (the codes path runs first, its one-hot flag read with the overflow flag: a
    rerun on the MFMA path) and deferred (a check pass first)."""
    m = _model()
    mm = _model(env={"EXPECTO_ONEHOT_CODES": "0"}, monkeypatch=monkeypatch)
    for e in (m.engine(), mm.engine()):
        e.set_overflow_check(deferred=deferred)
    codes = _codes(20, 2)
    x = _onehot(codes)
    assert torch.equal(m.forward(x), m.forward_codes(torch.from_numpy(codes).cuda(), 0))
    assert not torch.equal(m.forward(x), mm.forward(x))
    for bad in (0.5, -0.0):
        xb = x.clone()
        xb[7, 2, 0, 1000] = bad
        assert torch.equal(m.forward(xb), mm.forward(xb)), bad
    xb = x.clone()
    xb[3, :, 0, 10] = 1.0                                    # two ones in a column: not one-hot
    assert torch.equal(m.forward(xb), mm.forward(xb))


def test_forward_codes_after_load_state_dict_vs_oracle():
    """load_state_dict rebuilds the engine, and with it the k-mer tables of the new conv1 / conv2
    weights: forward_codes of the rebuilt model against the oracle of the loaded weights."""
    from expecto_amd import beluga
    from expecto_amd.encode import codes_to_onehot, seqs_to_codes
    from oracle import weights
    from oracle.beluga_np import forward_torch_cpu
    z = np.load(os.path.join(GOLDEN, "forward.npz"))
    seqs = [s.decode() for s in z["seqs"]]
    codes = torch.from_numpy(seqs_to_codes(seqs)).cuda()
    m2 = beluga.seeded(1, max_batch=16).cuda()
    before = m2.forward_codes(codes, 2).clone()
    m2.load_state_dict(beluga.seeded(0, gain=math.sqrt(6.0)).state_dict())
    got = m2.forward_codes(codes, 2)
    assert m2.engine().conv2_table_state() == (True, "held")
    assert not torch.allclose(before, got)
    x = torch.from_numpy(codes_to_onehot(seqs_to_codes(seqs)).astype(np.float32)).unsqueeze(2)
    want = forward_torch_cpu(weights.seeded_state_dict(0), x).numpy()
    assert_close(got.cpu().numpy(), want, what="forward_codes after load_state_dict vs oracle")
    assert_close(got.cpu().numpy(), z["y"], what="forward_codes after load_state_dict vs reference golden")


@pytest.mark.parametrize("precision", ["f16x3", "bf16x6"])
def test_codes_above_4_read_as_the_zero_column(precision):
    """a code byte >= 5 (5, 200, 255) reads as code 4 (the zero one-hot column, as
    conv1 reads it) in the k-mer gather: forward_codes (fwd + rc) and forward_pairs (the alt conv2
    patch from the alt codes) equal the runs with those bytes set to 4, bit for bit."""
    m = _model(precision=precision)
    eng = m.engine()
    c4 = _codes(12, 3)
    c4[2, 990:1010] = 4
    odd = c4.copy()
    rng = np.random.default_rng(4)
    pos = rng.integers(0, 2000, 120)
    odd[rng.integers(0, 12, 120), pos] = 255
    odd[2, 990:1010] = np.array([5, 200, 255, 6] * 5, np.uint8)
    c4 = np.where(odd > 4, 4, odd).astype(np.uint8)
    a, b = torch.from_numpy(odd).cuda(), torch.from_numpy(c4).cuda()
    assert torch.equal(m.forward_codes(a, 2), m.forward_codes(b, 2))
    var_pos = np.full(12, 1000, np.int32)
    alt_base = torch.from_numpy((c4[:, 1000] + 1) % 4).cuda()   # the same alt allele for both runs
    outs = []
    for ref in (a, b):
        alt = ref.clone()
        alt[:, 1000] = alt_base
        yr = torch.empty((24, 2002), device="cuda")
        ya = torch.empty((24, 2002), device="cuda")
        eng.forward_pairs(ref, alt, var_pos, yr, ya, 12)
        outs.append((yr, ya))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


def test_no_room_for_the_tables_is_reported_and_stays_at_parity(monkeypatch, capfd):
    """EXPECTO_KMER_MAX_BYTES below the tables' 20.7 GB: the handle holds no tables, says so
    (conv2_table_state, one line on stderr) and runs conv1 / conv2 on the MFMAs, inside the parity
    bar of the reference golden; EXPECTO_CONV2_TABLE=0 reports "off"."""
    from expecto_amd.encode import encodeSeqs, seqs_to_codes
    z = np.load(os.path.join(GOLDEN, "forward.npz"))
    seqs = [s.decode() for s in z["seqs"]]
    capfd.readouterr()
    m = _model(env={"EXPECTO_KMER_MAX_BYTES": str(10 << 30)}, monkeypatch=monkeypatch)
    assert m.engine().conv2_table_state() == (False, "no room")
    assert "no k-mer tables" in capfd.readouterr().err
    codes = torch.from_numpy(seqs_to_codes(seqs)).cuda()
    assert_close(m.forward_codes(codes, 2).cpu().numpy(), z["y"], what="no tables: forward_codes vs golden")
    x = torch.from_numpy(encodeSeqs(seqs).astype(np.float32)).unsqueeze(2).cuda()
    assert_close(m.forward(x).cpu().numpy(), z["y"], what="no tables: forward vs golden")
    off = _model(env={"EXPECTO_CONV2_TABLE": "0"}, monkeypatch=monkeypatch)
    assert off.engine().conv2_table_state() == (False, "off (EXPECTO_CONV2_TABLE=0)")


def test_shared_tables_count_once_in_device_bytes():
    """Two handles sharing one set of tables: the first holder reports the 20.7 GB, the second
    not; when the first goes, the second reports them."""
    import gc
    table = (4 * 5 ** 9 + 2 * 4 ** 11) * 320 * 4
    a = _model(seed=4343)
    b = _model(seed=4343)
    ea, eb = a.engine(), b.engine()
    assert ea.device_bytes() >= table > eb.device_bytes()
    own_b = eb.device_bytes()
    del ea, a
    gc.collect()
    assert eb.device_bytes() == own_b + table
