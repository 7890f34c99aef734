"""Build libexpecto_hip.so in-tree for gfx950 (``python -m expecto_amd.build``)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SOURCES = [os.path.join(HERE, "csrc", f) for f in ("beluga.hip", "reduce.hip")]
OUT = os.path.join(HERE, "libexpecto_hip.so")
ARCH = os.environ.get("EXPECTO_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for c in ("/opt/rocm/bin/hipcc", "hipcc"):
        if os.path.exists(c) or c == "hipcc":
            return c
    raise RuntimeError("hipcc not found")


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = SOURCES + [os.path.join(HERE, "csrc", h) for h in ("common.h", "gemm_kernel.h")] + [
                      os.path.join(os.path.dirname(HERE), "include", "expecto_hip.h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        return OUT
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wno-unused-result", *SOURCES, "-o", OUT + ".tmp"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
