"""CPU: the C-ABI library loads and exports exactly what include/expecto_hip.h declares."""
import ctypes
import os
import re

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "expecto_hip.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(expecto_\w+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    from expecto_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        from expecto_amd import build
        build.build()
    return _lib.load()


def test_header_declares_the_boundary():
    fns = declared_functions()
    for f in ("expecto_beluga_create", "expecto_beluga_forward_onehot", "expecto_beluga_forward_codes",
              "expecto_variant_windows", "expecto_tss_windows", "expecto_tss_reduce", "expecto_variant_reduce",
              "expecto_diff", "expecto_fwd_rc_average", "expecto_beluga_destroy", "expecto_last_error"):
        assert f in fns


def test_library_exports_every_declared_symbol(lib):
    from expecto_amd import _lib
    fns = declared_functions()
    for f in fns:
        assert hasattr(lib, f), f
    assert sorted(_lib.SIGNATURES) == fns          # the ctypes binding covers the whole header


def test_symbols_are_c_linkage():
    out = os.popen(f"nm -D --defined-only {os.path.join(REPO, 'expecto_amd', 'libexpecto_hip.so')}").read()
    exported = set(re.findall(r" T (expecto_\w+)", out))
    assert set(declared_functions()) <= exported


def test_host_only_calls(lib):
    """Calls that never touch the GPU: version, argument validation, empty work."""
    assert lib.expecto_version().decode().startswith("expecto_hip")
    h = ctypes.c_void_p()
    assert lib.expecto_beluga_create(0, None, 16, None, ctypes.byref(h)) == -1
    assert b"null" in lib.expecto_last_error()
    assert lib.expecto_diff(None, None, 0, None, None) == 0
    assert lib.expecto_variant_reduce(None, None, None, None, 9, 0, 2002, None, None) == 0
    assert lib.expecto_tss_reduce(None, None, None, 0, 200, 2002, None, None) == 0
    assert lib.expecto_beluga_forward_onehot(None, None, 1, None, None) == -1
    assert lib.expecto_variant_windows(None, 0, None, None, None, 1, None, 0, None, None) == -1


def test_no_cpu_fallback_without_library(tmp_path, monkeypatch):
    from expecto_amd import _lib
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(RuntimeError, match="not built"):
        _lib.load(str(tmp_path / "missing.so"))


def _function_body(src: str, name: str) -> str:
    """Text of the C++ function `name` (first definition) by brace matching."""
    m = re.search(r"\n[\w:<>,\s\*&]*\b" + name + r"\s*\([^;{]*\)\s*\{", src)
    assert m, name
    i, depth = m.end(), 1
    while depth:
        depth += {"{": 1, "}": -1}.get(src[i], 0)
        i += 1
    return src[m.start():i]


def test_production_forward_has_no_host_sync():
    """The forward paths only enqueue work: no stream/device sync and no blocking copy in the
    functions a forward call runs (forward_chunk, forward_segments, forward_pairs, run_fc,
    run_conv, run_conv1, stage_copies); the f16x3 overflow check syncs only in its per-call
    mode (run_checked) and the deferred release point (expecto_beluga_overflow_pending)."""
    src = open(os.path.join(REPO, "expecto_amd", "csrc", "beluga.hip")).read()
    for fn in ("forward_chunk", "forward_segments", "forward_pairs", "run_fc", "run_conv", "run_conv1",
               "stage_copies", "count_slab_macs"):
        body = _function_body(src, fn)
        for bad in ("hipStreamSynchronize", "hipDeviceSynchronize", "hipMemcpy(", "hipMemcpyDeviceToHost"):
            assert bad not in body, (fn, bad)
    rc = _function_body(src, "run_checked")
    assert rc.index("h->ovf_deferred") < rc.index("hipStreamSynchronize")


def test_product_gemm_header_holds_only_launched_kernels():
    """Every __global__ kernel of the library's GEMM header is launched by the library; the
    probe-only shapes live in tools/gemm_probes.h."""
    import re
    csrc = os.path.join(REPO, "expecto_amd", "csrc")
    hdr = open(os.path.join(csrc, "gemm_kernel.h")).read()
    lib = open(os.path.join(csrc, "beluga.hip")).read() + open(os.path.join(csrc, "reduce.hip")).read()
    kernels = re.findall(r"__global__\s+(?:__launch_bounds__\([^)]*\)\s+)?void\s+(\w+)", hdr)
    assert kernels
    for k in kernels:
        assert re.search(rf"\b{k}\s*(<[^;]*?>)?\s*<<<", lib), f"{k} is declared in gemm_kernel.h but never launched"
