"""ctypes binding of the C-ABI in include/expecto_hip.h (libexpecto_hip.so, gfx950).

The library is built in-tree (``python -m expecto_amd.build`` or
``__graft_entry__.build()``).  There is NO CPU fallback: if the library is missing or
fails to load, every product entry point raises ``RuntimeError``.

torch is imported before the library so that the HIP runtime torch already loaded
(soname ``libamdhip64.so.7``) is the one the library binds to: device pointers and
streams are then shared with torch tensors.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libexpecto_hip.so")

c_f32p = ctypes.POINTER(ctypes.c_float)
c_f64p = ctypes.POINTER(ctypes.c_double)
c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_i64p = ctypes.POINTER(ctypes.c_longlong)
c_i32p = ctypes.POINTER(ctypes.c_int)
c_vp = ctypes.c_void_p

# name -> (restype, argtypes); must match include/expecto_hip.h exactly.
SIGNATURES = {
    "expecto_beluga_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(c_vp), ctypes.c_int, c_vp,
                                             ctypes.POINTER(c_vp)]),
    "expecto_beluga_destroy": (None, [c_vp]),
    "expecto_beluga_device_bytes": (ctypes.c_size_t, [c_vp]),
    "expecto_beluga_conv2_table_active": (ctypes.c_int, [c_vp, c_i32p]),
    "expecto_beluga_set_fc1_role": (ctypes.c_int, [c_vp, ctypes.c_int]),
    "expecto_beluga_forward_onehot": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int, c_vp, c_vp]),
    "expecto_beluga_forward_codes": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int, ctypes.c_longlong, ctypes.c_int,
                                                    c_vp, c_vp]),
    "expecto_beluga_forward_segments": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int, ctypes.c_int, ctypes.c_longlong,
                                                       ctypes.c_int, c_vp, c_vp, c_vp, ctypes.c_int, c_vp, c_vp]),
    "expecto_gather_segments": (ctypes.c_int, [c_vp, ctypes.c_longlong, c_vp, ctypes.c_int, ctypes.c_int, c_vp,
                                               c_vp, c_vp, c_vp]),
    "expecto_beluga_forward_pairs": (ctypes.c_int, [c_vp, c_vp, c_vp, ctypes.c_int, ctypes.c_longlong, c_vp,
                                                    ctypes.c_int, c_vp, c_vp, ctypes.c_longlong, c_vp]),
    "expecto_beluga_forward_segment_pairs": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, ctypes.c_int, ctypes.c_int,
                                                            ctypes.c_longlong, ctypes.c_int, c_vp, c_vp, c_vp,
                                                            ctypes.c_int, c_vp, c_vp, ctypes.c_longlong, c_vp]),
    "expecto_beluga_set_precision": (ctypes.c_int, [c_vp, ctypes.c_int]),
    "expecto_beluga_get_precision": (ctypes.c_int, [c_vp]),
    "expecto_beluga_set_f16_target": (ctypes.c_int, [c_vp, ctypes.c_int]),
    "expecto_beluga_f16_fallbacks": (ctypes.c_longlong, [c_vp, c_i32p]),
    "expecto_beluga_set_overflow_check": (ctypes.c_int, [c_vp, ctypes.c_int]),
    "expecto_beluga_overflow_pending": (ctypes.c_int, [c_vp, c_vp]),
    "expecto_beluga_overflow_take": (ctypes.c_int, [c_vp, c_vp, c_vp]),
    "expecto_beluga_count_fallback": (ctypes.c_int, [c_vp]),
    "expecto_beluga_set_profiling": (ctypes.c_int, [c_vp, ctypes.c_int]),
    "expecto_beluga_layer_times": (ctypes.c_int, [c_vp, c_f64p, c_i64p, c_f64p, ctypes.c_int]),
    "expecto_beluga_main_launches": (ctypes.c_int, [c_vp, ctypes.c_int, c_i64p, c_f64p, c_i64p, c_f64p]),
    "expecto_variant_windows": (ctypes.c_int, [c_vp, ctypes.c_longlong, c_vp, c_vp, c_vp, ctypes.c_int, c_vp,
                                               ctypes.c_int, c_vp, c_vp]),
    "expecto_indel_windows": (ctypes.c_int, [c_vp, ctypes.c_longlong, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                             ctypes.c_int, c_vp, c_vp]),
    "expecto_tss_windows": (ctypes.c_int, [c_vp, ctypes.c_longlong, c_vp, c_vp, ctypes.c_int, c_vp, ctypes.c_int,
                                           c_vp, c_vp]),
    "expecto_diff": (ctypes.c_int, [c_vp, c_vp, ctypes.c_longlong, c_vp, c_vp]),
    "expecto_fwd_rc_average": (ctypes.c_int, [c_vp, ctypes.c_int, ctypes.c_int, c_vp, c_vp]),
    "expecto_tss_reduce": (ctypes.c_int, [c_vp, c_vp, c_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_vp, c_vp]),
    "expecto_variant_reduce": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                              c_vp, c_vp]),
    "expecto_variant_reduce_lut": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                  c_vp, ctypes.c_int, c_vp, c_vp]),
    "expecto_gblinear_predict": (ctypes.c_int, [c_vp, ctypes.c_longlong, ctypes.c_longlong, c_vp, ctypes.c_int,
                                                c_vp, ctypes.c_float, c_vp, c_vp]),
    "expecto_shift_reduce": (ctypes.c_int, [c_vp, c_vp, c_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                            c_vp, c_vp]),
    "expecto_last_error": (ctypes.c_char_p, []),
    "expecto_version": (ctypes.c_char_p, []),
}

STRAND_FWD, STRAND_RC, STRAND_BOTH = 0, 1, 2
PRECISION_FP32, PRECISION_BF16X6, PRECISION_F16X3 = 0, 1, 2
PRECISIONS = {"fp32": PRECISION_FP32, "bf16x6": PRECISION_BF16X6, "f16x3": PRECISION_F16X3}
_BASE_LAYERS = ("conv1", "conv2", "conv3", "conv4", "conv5", "conv6", "fc1", "fc1_reduce", "fc2")
# expecto_beluga_layer_times slots: the layers of every forward, then their alt-delta launches
LAYER_NAMES = _BASE_LAYERS + tuple(f"{n}_delta" for n in _BASE_LAYERS)
N_LAYERS = len(LAYER_NAMES)

_lib = None


def load(path: str = LIB_PATH):
    """Load (once) and return the ctypes library; raise RuntimeError if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    import torch  # noqa: F401  -- bind to torch's HIP runtime (see module docstring)

    if not os.path.exists(path):
        raise RuntimeError(f"HIP library {path} not built: run `python -m expecto_amd.build` "
                           "(there is no CPU fallback)")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(status: int, what: str) -> None:
    if status != 0:
        msg = _lib.expecto_last_error().decode() if _lib is not None else ""
        raise RuntimeError(f"{what} failed (status {status}): {msg}")


def stream_ptr(stream=None) -> int:
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def dptr(t) -> int:
    """Device pointer of a CUDA (HIP) tensor; fails loudly on CPU tensors."""
    if not t.is_cuda:
        raise RuntimeError("expecto_amd kernels need device (HIP) tensors; there is no CPU path")
    return int(t.data_ptr())
