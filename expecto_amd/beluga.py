"""Drop-in ``Beluga`` module backed by the gfx950 HIP kernels.

Mirrors the reference operator API (``Beluga.py:18-51``): the same ``nn.Module`` tree,
so ``state_dict()`` keys are exactly ``model.0.{0,2,6,8,12,14}.{weight,bias}``,
``model.1.2.1.{weight,bias}``, ``model.1.4.1.{weight,bias}`` and a strict
``load_state_dict(torch.load(pth))`` of the reference checkpoint works unchanged
(``chromatin.py:102-106``).  Constructing the layers in the reference order also
reproduces the reference's default initialisation bit for bit under the same seed.

``forward(x)`` takes ``x`` = ``[B,4,1,2000]`` (or ``[B,4,2000]``) fp32 on the GPU and
returns ``[B,2002]`` sigmoid outputs, computed by ``libexpecto_hip.so``.  There is no
CPU path: a CPU tensor, or a missing library, raises ``RuntimeError``.  One-hot input as
``encodeSeqs`` writes it (``chromatin.py:138-172``) runs through the k-mer gather, the same
bits as ``forward_codes``; any other fp32 input keeps conv1 / conv2 on the MFMAs.
"""
from __future__ import annotations

import ctypes

import torch
from torch import nn

from . import _lib

PARAM_KEYS = (
    "model.0.0.weight", "model.0.0.bias", "model.0.2.weight", "model.0.2.bias",
    "model.0.6.weight", "model.0.6.bias", "model.0.8.weight", "model.0.8.bias",
    "model.0.12.weight", "model.0.12.bias", "model.0.14.weight", "model.0.14.bias",
    "model.1.2.1.weight", "model.1.2.1.bias", "model.1.4.1.weight", "model.1.4.1.bias",
)
INPUT_LEN = 2000
N_FEATURES = 2002


class _Flatten(nn.Module):
    """Stands where the reference has ``Lambda(lambda x: x.view(...))`` (no parameters)."""

    def forward(self, x):
        return x.reshape(x.size(0), -1)


class BelugaEngine:
    """Owns one ``expecto_beluga_t`` handle (weights repacked on the device + workspace)."""

    def __init__(self, params: list, device: int, max_batch: int = 1024, stream=None):
        self.lib = _lib.load()
        if len(params) != len(PARAM_KEYS):
            raise RuntimeError("Beluga needs 16 parameter tensors")
        ptrs = (ctypes.c_void_p * len(params))()
        for i, p in enumerate(params):
            if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()):
                raise RuntimeError(f"parameter {PARAM_KEYS[i]} must be a contiguous fp32 device tensor")
            ptrs[i] = p.data_ptr()
        h = ctypes.c_void_p()
        with torch.cuda.device(device):
            _lib.check(self.lib.expecto_beluga_create(device, ptrs, int(max_batch), _lib.stream_ptr(stream),
                                                      ctypes.byref(h)), "expecto_beluga_create")
        self.handle = h
        self.device = device
        self.max_batch = max_batch
        import os
        self.set_precision(os.environ.get("EXPECTO_PRECISION", "f16x3"))

    def set_precision(self, precision: str):
        """GEMM arithmetic (include/expecto_hip.h): 'f16x3' (default: scaled split-fp16, half the
        MFMA work of bf16x6, bf16x6 recompute on fp16 overflow), 'bf16x6' (split-bf16 over fp32's
        whole range) or 'fp32' (exact fp32 MFMA).  All three are within the parity bar of the
        float64 forward with the same margin as the exact-fp32 kernel (tools/accuracy_gpu.py)."""
        if precision not in _lib.PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(_lib.PRECISIONS)}")
        with torch.cuda.device(self.device):
            _lib.check(self.lib.expecto_beluga_set_precision(self.handle, _lib.PRECISIONS[precision]),
                       "set_precision")
        self.precision = precision

    def set_fc1_role(self, role: int):
        """FC1 role of this engine's per-window forwards (include/expecto_hip.h
        expecto_beluga_set_fc1_role): 4 = the direct FC1 (default, the form of +-800 sweeps), 0..3 =
        block-Karatsuba roles; a segment-path window of role r equals a per-window forward in role r
        bit for bit (pipeline.fc1_role / sweep_roles give a segment window's role)."""
        _lib.check(self.lib.expecto_beluga_set_fc1_role(self.handle, int(role)), "set_fc1_role")

    def set_f16_target(self, target_log2: int):
        """f16x3 calibration target: the largest calibration activation maps to 2^target_log2."""
        with torch.cuda.device(self.device):
            _lib.check(self.lib.expecto_beluga_set_f16_target(self.handle, int(target_log2)), "set_f16_target")

    def f16_state(self):
        """(calls recomputed with bf16x6 after an fp16 overflow, activation scale exponents [7])."""
        sx = (ctypes.c_int * 7)()
        n = self.lib.expecto_beluga_f16_fallbacks(self.handle, sx)
        if n < 0:
            _lib.check(int(n), "f16_fallbacks")
        return int(n), list(sx)

    def set_overflow_check(self, deferred: bool):
        """f16x3 overflow check: per call (default; one stream sync per forward call) or deferred
        to ``overflow_pending()`` at the caller's release point (no sync inside a forward)."""
        _lib.check(self.lib.expecto_beluga_set_overflow_check(self.handle, int(bool(deferred))), "set_overflow_check")
        self.deferred = bool(deferred)

    def overflow_pending(self, stream=None) -> bool:
        """Deferred mode: sync the stream; True if an f16x3 activation overflowed since the last
        check (the flag is cleared; recompute those calls under ``precision_override('bf16x6')``)."""
        with torch.cuda.device(self.device):
            r = self.lib.expecto_beluga_overflow_pending(self.handle, _lib.stream_ptr(stream))
        if r < 0:
            _lib.check(int(r), "overflow_pending")
        return bool(r)

    def overflow_take(self, dst: torch.Tensor, stream=None):
        """Deferred mode: enqueue a copy of the overflow flag into ``dst`` (an int32 tensor of one
        element, pinned host or device) and reset the flag, with no host sync."""
        if dst.dtype != torch.int32 or dst.numel() != 1 or not (dst.is_cuda or dst.is_pinned()):
            raise RuntimeError("overflow_take: dst must be a pinned-host or device int32 tensor of one element")
        with torch.cuda.device(self.device):
            _lib.check(self.lib.expecto_beluga_overflow_take(self.handle, ctypes.c_void_p(dst.data_ptr()),
                                                             _lib.stream_ptr(stream)), "overflow_take")

    def count_fallback(self):
        """Deferred mode: record that a batch flagged through ``overflow_take`` was recomputed in
        bf16x6 (``f16_state()`` reports the count)."""
        _lib.check(self.lib.expecto_beluga_count_fallback(self.handle), "count_fallback")

    def precision_override(self, precision: str):
        """Context manager: run the enclosed calls in another arithmetic, then restore."""
        import contextlib

        @contextlib.contextmanager
        def cm():
            base = self.precision
            self.set_precision(precision)
            try:
                yield self
            finally:
                self.set_precision(base)
        return cm()

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            self.lib.expecto_beluga_destroy(h)
            self.handle = None

    def forward_onehot(self, x: torch.Tensor, out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
        if x.dim() == 4:
            if x.shape[2] != 1:
                raise RuntimeError("expected input [B,4,1,2000]")
            x3 = x
        elif x.dim() == 3:
            x3 = x
        else:
            raise RuntimeError("expected input [B,4,1,2000] or [B,4,2000]")
        if x3.shape[1] != 4 or x3.shape[-1] != INPUT_LEN:
            raise RuntimeError(f"expected 4 channels x {INPUT_LEN} positions, got {tuple(x.shape)}")
        if x3.dtype != torch.float32:
            raise RuntimeError("input must be float32")
        if not x3.is_contiguous():
            # the reference fails on non-contiguous input at x.view (Beluga.py:42)
            raise RuntimeError("view size is not compatible with input tensor's size and stride "
                               "(input must be contiguous)")
        n = x3.shape[0]
        if out is None:
            out = torch.empty((n, N_FEATURES), device=x3.device, dtype=torch.float32)
        _lib.check(self.lib.expecto_beluga_forward_onehot(self.handle, _lib.dptr(x3), n, _lib.dptr(out),
                                                          _lib.stream_ptr(stream)), "forward_onehot")
        return out

    def forward_codes(self, codes: torch.Tensor, strand_mode: int = _lib.STRAND_BOTH,
                      out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
        if codes.dtype != torch.uint8 or codes.dim() != 2 or codes.shape[1] < INPUT_LEN:
            raise RuntimeError("codes must be uint8 [n, >=2000]")
        if codes.stride(1) != 1:
            raise RuntimeError("codes rows must be contiguous")
        n = codes.shape[0]
        rows = 2 * n if strand_mode == _lib.STRAND_BOTH else n
        if out is None:
            out = torch.empty((rows, N_FEATURES), device=codes.device, dtype=torch.float32)
        _lib.check(self.lib.expecto_beluga_forward_codes(self.handle, _lib.dptr(codes), n, codes.stride(0),
                                                         int(strand_mode), _lib.dptr(out),
                                                         _lib.stream_ptr(stream)), "forward_codes")
        return out

    def forward_segments(self, codes: torch.Tensor, seg_len: int, win_seg, win_off, win_row=None,
                         strand_mode: int = _lib.STRAND_BOTH, out: torch.Tensor | None = None, stream=None):
        """Windows that are slices of longer sequences (shared trunk, bit-identical outputs).

        codes: uint8 [n_seg, >=seg_len] device; win_seg/win_off/win_row: host int arrays
        (sorted by segment; offsets multiples of 4).  Returns [n_win or 2*n_win, 2002]."""
        import numpy as np

        if codes.dtype != torch.uint8 or codes.dim() != 2 or codes.shape[1] < seg_len or codes.stride(1) != 1:
            raise RuntimeError("codes must be uint8 [n_seg, >=seg_len] with contiguous rows")
        ws = np.ascontiguousarray(win_seg, np.int32)
        wo = np.ascontiguousarray(win_off, np.int32)
        wr = None if win_row is None else np.ascontiguousarray(win_row, np.int32)
        n_win = int(ws.size)
        rows = 2 * n_win if strand_mode == _lib.STRAND_BOTH else n_win
        if out is None:
            out = torch.empty((rows, N_FEATURES), device=codes.device, dtype=torch.float32)
        if out.shape != (rows, N_FEATURES) or not out.is_contiguous():
            raise RuntimeError("out must be contiguous [rows, 2002]")
        _lib.check(self.lib.expecto_beluga_forward_segments(
            self.handle, _lib.dptr(codes), codes.shape[0], int(seg_len), codes.stride(0), int(strand_mode),
            ws.ctypes.data, wo.ctypes.data, None if wr is None else wr.ctypes.data, n_win, _lib.dptr(out),
            _lib.stream_ptr(stream)), "forward_segments")
        return out

    def forward_segment_pairs(self, codes: torch.Tensor, seg_len: int, var_pos, alt_code: torch.Tensor,
                              win_seg, win_off, win_row, y_ref: torch.Tensor, y_alt: torch.Tensor, strand_stride: int,
                              strand_mode: int = _lib.STRAND_BOTH, stream=None):
        """SNV sweeps on shared segments: ref windows from `codes` (uint8 [n_seg, >=seg_len]),
        alt windows = the same offsets with alt_code[s] (uint8 device tensor) at var_pos[s]
        (host ints, one per segment); the alt trunk recomputes only the rows the SNV changes
        and alt windows not holding the SNV copy their ref row.
        Row (strand s, window w) is s*strand_stride + win_row[w] of y_ref / y_alt (device
        views starting at row 0; they may alias one larger tensor).  Bit-identical to full
        forwards of both alleles."""
        import numpy as np

        if codes.dtype != torch.uint8 or codes.dim() != 2 or codes.shape[1] < seg_len or codes.stride(1) != 1:
            raise RuntimeError("codes must be uint8 [n_seg, >=seg_len] with contiguous rows")
        n_seg = codes.shape[0]
        if isinstance(var_pos, torch.Tensor):
            var_pos = var_pos.cpu().numpy()
        pos = np.ascontiguousarray(var_pos, np.int32).reshape(-1)
        if not alt_code.is_cuda or pos.size != n_seg or alt_code.numel() != n_seg:
            raise RuntimeError("var_pos (host) / alt_code (device): one entry per segment")
        alt = alt_code.to(torch.uint8).contiguous()
        ws = np.ascontiguousarray(win_seg, np.int32)
        wo = np.ascontiguousarray(win_off, np.int32)
        wr = None if win_row is None else np.ascontiguousarray(win_row, np.int32)
        _lib.check(self.lib.expecto_beluga_forward_segment_pairs(
            self.handle, _lib.dptr(codes), pos.ctypes.data, _lib.dptr(alt), n_seg, int(seg_len), codes.stride(0),
            int(strand_mode), ws.ctypes.data, wo.ctypes.data, None if wr is None else wr.ctypes.data, int(ws.size),
            _lib.dptr(y_ref), _lib.dptr(y_alt), int(strand_stride), _lib.stream_ptr(stream)), "forward_segment_pairs")

    def forward_pairs(self, ref_codes: torch.Tensor, alt_codes: torch.Tensor, var_pos, y_ref: torch.Tensor,
                      y_alt: torch.Tensor, strand_stride: int, strand_mode: int = _lib.STRAND_BOTH, stream=None):
        """SNV ref/alt window pairs with alt-cone reuse (bit-identical to two full forwards).

        ref_codes/alt_codes: uint8 [n, >=2000] device, differing at most at var_pos[v] (int32
        device tensor, or host ints which are copied to the device here).  Row (strand s, variant v) of the outputs is s*strand_stride + v; y_ref/y_alt are
        device views whose first element is row 0 (they may alias one larger tensor)."""
        import numpy as np

        for c in (ref_codes, alt_codes):
            if c.dtype != torch.uint8 or c.dim() != 2 or c.shape[1] < INPUT_LEN or c.stride(1) != 1:
                raise RuntimeError("codes must be uint8 [n, >=2000] with contiguous rows")
        if ref_codes.shape != alt_codes.shape or ref_codes.stride(0) != alt_codes.stride(0):
            raise RuntimeError("ref and alt codes must have the same shape and stride")
        n = ref_codes.shape[0]
        if isinstance(var_pos, torch.Tensor) and var_pos.is_cuda:
            pos = var_pos.to(torch.int32).contiguous()
        else:
            pos = torch.from_numpy(np.ascontiguousarray(var_pos, np.int32)).to(ref_codes.device)
        if pos.numel() != n:
            raise RuntimeError("one variant position per window pair")
        _lib.check(self.lib.expecto_beluga_forward_pairs(
            self.handle, _lib.dptr(ref_codes), _lib.dptr(alt_codes), n, ref_codes.stride(0), _lib.dptr(pos),
            int(strand_mode), _lib.dptr(y_ref), _lib.dptr(y_alt), int(strand_stride), _lib.stream_ptr(stream)),
            "forward_pairs")

    def set_profiling(self, on: bool):
        _lib.check(self.lib.expecto_beluga_set_profiling(self.handle, int(on)), "set_profiling")

    def layer_times(self):
        """{layer: (device ms, launches, executed multiply-adds)} accumulated while profiling."""
        ms = (ctypes.c_double * _lib.N_LAYERS)()
        calls = (ctypes.c_longlong * _lib.N_LAYERS)()
        macs = (ctypes.c_double * _lib.N_LAYERS)()
        n = self.lib.expecto_beluga_layer_times(self.handle, ms, calls, macs, _lib.N_LAYERS)
        if n < 0:
            _lib.check(n, "layer_times")
        return {_lib.LAYER_NAMES[i]: (ms[i], calls[i], macs[i]) for i in range(_lib.N_LAYERS)}

    def main_launches(self, layer: str):
        """(rows, device ms, launches, executed multiply-adds) of the layer's full-size conv GEMM
        launches alone (include/expecto_hip.h expecto_beluga_main_launches), accumulated while
        profiling; rows 0 if none ran."""
        rows, ms, calls, macs = ctypes.c_longlong(), ctypes.c_double(), ctypes.c_longlong(), ctypes.c_double()
        _lib.check(self.lib.expecto_beluga_main_launches(self.handle, _lib.LAYER_NAMES.index(layer), ctypes.byref(rows),
                                                         ctypes.byref(ms), ctypes.byref(calls), ctypes.byref(macs)),
                   "main_launches")
        return rows.value, ms.value, calls.value, macs.value

    def device_bytes(self) -> int:
        """Device bytes of the handle; shared k-mer tables count only for their first holder."""
        return int(self.lib.expecto_beluga_device_bytes(self.handle))

    CONV2_TABLE_REASONS = {0: "held", 1: "off (EXPECTO_CONV2_TABLE=0)", 2: "no room"}

    def conv2_table_state(self):
        """(active, reason): whether forwards from codes / exact one-hot floats gather conv1 + conv2
        + pool1 from the k-mer tables, and why not (include/expecto_hip.h)."""
        why = ctypes.c_int(0)
        r = self.lib.expecto_beluga_conv2_table_active(self.handle, ctypes.byref(why))
        if r < 0:
            _lib.check(int(r), "conv2_table_active")
        return bool(r), self.CONV2_TABLE_REASONS.get(why.value, str(why.value))

    @property
    def conv2_table_active(self) -> bool:
        return self.conv2_table_state()[0]


class Beluga(nn.Module):
    """Reference-compatible Beluga (Beluga.py:18-48) whose forward runs on gfx950 HIP kernels."""

    def __init__(self, max_batch: int = 1024):
        super().__init__()
        self.model = nn.Sequential(
            nn.Sequential(
                nn.Conv2d(4, 320, (1, 8)), nn.ReLU(),
                nn.Conv2d(320, 320, (1, 8)), nn.ReLU(), nn.Dropout(0.2), nn.MaxPool2d((1, 4), (1, 4)),
                nn.Conv2d(320, 480, (1, 8)), nn.ReLU(),
                nn.Conv2d(480, 480, (1, 8)), nn.ReLU(), nn.Dropout(0.2), nn.MaxPool2d((1, 4), (1, 4)),
                nn.Conv2d(480, 640, (1, 8)), nn.ReLU(),
                nn.Conv2d(640, 640, (1, 8)), nn.ReLU(),
            ),
            nn.Sequential(
                nn.Dropout(0.5), _Flatten(),
                nn.Sequential(nn.Identity(), nn.Linear(67840, 2003)), nn.ReLU(),
                nn.Sequential(nn.Identity(), nn.Linear(2003, 2002)),
            ),
            nn.Sigmoid(),
        )
        self.max_batch = max_batch
        self._engine = None
        self._engine_key = None

    # -- engine management: rebuilt whenever the parameters change (load_state_dict, .cuda())
    def _params(self):
        # (owner module, name) of each parameter, resolved once: a named_parameters() walk per
        # forward cost ~50 us of host time, 7 % of a batch-32 Beluga.forward.  A parameter
        # reassigned on its module is still seen (the owner's _parameters is read each call), and
        # the cached module links are checked by identity each call, so a replaced submodule
        # (model.model[0] = nn.Conv2d(...)) or a copy whose module dicts are its own (DataParallel
        # replicas copy __dict__) resolves again instead of reading stale parameters.
        cache = self.__dict__.get("_param_slots")
        if cache is not None:
            root, checks, slots = cache
            if root is not self._modules or any(parent.get(part) is not child for parent, part, child in checks):
                cache = None
        if cache is None:
            slots, seen, checks = [], set(), []
            for k in PARAM_KEYS:
                *path, name = k.split(".")
                mod = self
                for part in path:
                    child = mod._modules[part]
                    if id(child) not in seen:          # each module link once (13 identity checks)
                        seen.add(id(child))
                        checks.append((mod._modules, part, child))
                    mod = child
                slots.append((mod._parameters, name))
            cache = (self._modules, checks, slots)
            self.__dict__["_param_slots"] = cache
        return [d[name] for d, name in cache[2]]

    def _key(self, params):
        return tuple((p.data_ptr(), p._version) for p in params)

    def engine(self) -> BelugaEngine:
        params = self._params()
        key = self._key(params)
        if self._engine is None or self._engine_key != key:
            dev = params[0].device
            if dev.type != "cuda":
                raise RuntimeError("Beluga parameters are on the CPU: call .cuda() first "
                                   "(the MI355X engine has no CPU path)")
            self._engine = None
            self._engine = BelugaEngine([p.detach().contiguous() for p in params], dev.index or 0, self.max_batch)
            self._engine_key = key
        return self._engine

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not x.is_cuda:
            raise RuntimeError("Beluga.forward needs a device tensor (input.cuda()); there is no CPU path")
        return self.engine().forward_onehot(x)

    def forward_codes(self, codes: torch.Tensor, strand_mode: int = _lib.STRAND_BOTH) -> torch.Tensor:
        return self.engine().forward_codes(codes, strand_mode)


def seeded(seed: int = 0, gain: float | None = None, max_batch: int = 1024) -> Beluga:
    """``torch.manual_seed(seed); Beluga()`` -- same RNG stream as the reference -- with every
    weight optionally scaled by ``gain`` (the golden vectors use sqrt(6))."""
    torch.manual_seed(seed)
    m = Beluga(max_batch=max_batch)
    if gain is not None:
        with torch.no_grad():
            for k, p in m.named_parameters():
                if k.endswith(".weight"):
                    p.mul_(gain)
    return m.eval()
