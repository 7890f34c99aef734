"""Stand-in for xgboost used ONLY when running the reference scripts for golden vectors.

* ``DMatrix`` captures the feature matrices predict.py builds (captured_dmatrix_<i>.npy).
* ``Booster`` restates xgboost 0.7's gblinear (the reference pins xgboost==0.7.post4):
  ``load_model`` reads the legacy binary model layout (optional ``binf``; LearnerModelParam
  136 B; objective and booster names as u64-length strings; GBLinearModelParam 136 B; u64
  count + f32 weights, w[f*groups+g], biases after the features) and ``predict`` is
  GBLinear::Pred: psum = f32(bias + base_score), then psum = f32(psum + f32(f32(x_f) * w_f))
  over the features in column order.  A model path of "none" predicts zeros (feature capture
  only).  This is test infrastructure, independent of expecto_amd.xgblinear.
"""
import struct

import numpy as np

CAPTURED = []


class DMatrix:
    def __init__(self, data):
        self.data = np.asarray(data)
        CAPTURED.append(self.data)
        np.save(f"captured_dmatrix_{len(CAPTURED) - 1}.npy", self.data)


class Booster:
    def __init__(self, params=None):
        self.w = None

    def load_model(self, path):
        if path == "none":
            return
        raw = open(path, "rb").read()
        o = 4 if raw[:4] == b"binf" else 0
        base = struct.unpack_from("<f", raw, o)[0]
        o += 136
        for _ in range(2):                      # objective, booster names
            (n,) = struct.unpack_from("<Q", raw, o)
            o += 8 + n
        nf, groups = struct.unpack_from("<Ii", raw, o)
        o += 136
        (count,) = struct.unpack_from("<Q", raw, o)
        o += 8
        w = np.frombuffer(raw, "<f4", count, o).reshape(nf + 1, groups)
        self.w, self.bias, self.base = w[:nf, 0].copy(), np.float32(w[nf, 0]), np.float32(base)

    def predict(self, d):
        x = d.data
        if self.w is None:
            return np.zeros(x.shape[0], dtype=np.float32)
        x = x.astype(np.float32)
        psum = np.full(x.shape[0], np.float32(self.bias + self.base), dtype=np.float32)
        for f in range(self.w.shape[0]):
            psum = (psum + (x[:, f] * self.w[f]).astype(np.float32)).astype(np.float32)
        return psum
