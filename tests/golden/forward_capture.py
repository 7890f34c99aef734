"""Golden-generation helper (never used at test time): run a reference script as __main__ with
its ``Beluga.forward`` outputs recorded, in call order, into ``captured_forward.npz`` in the
working directory.

    PYTHONPATH=stubs:/root/reference python forward_capture.py <script.py> [script args...]

The reference model class is used unchanged; the wrapper only copies each forward's output.
"""
import atexit
import runpy
import sys

import numpy as np

import Beluga as _reference_beluga   # the reference module (PYTHONPATH puts /root/reference after the stubs)

_OUTPUTS = []
_forward = _reference_beluga.Beluga.forward


def _recording_forward(self, x):
    y = _forward(self, x)
    _OUTPUTS.append(y.detach().cpu().numpy().copy())
    return y


def _dump():
    np.savez("captured_forward.npz", *_OUTPUTS)


_reference_beluga.Beluga.forward = _recording_forward
atexit.register(_dump)

if __name__ == "__main__":
    script = sys.argv[1]
    sys.argv = sys.argv[1:]
    runpy.run_path(script, run_name="__main__")
