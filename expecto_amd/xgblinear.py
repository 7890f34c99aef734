"""ExPecto expression models: xgboost ``gblinear`` boosters, read without xgboost.

The reference scores variant features with ``xgb.Booster.load_model(...).predict(DMatrix)``
(``predict.py:150-166``) on the models ``train.py:140-157`` writes (``booster='gblinear'``,
``objective='reg:linear'``, ``base_score`` 2, saved as ``*.save``; the pinned library is
``xgboost==0.7.post4``, ``requirements.txt``).  xgboost is not installed here, so this module
restates the published model formats and the gblinear prediction rule:

* legacy binary (``Booster.save_model`` of xgboost 0.7-0.90, the reference's ``.save``):
  optional ``binf`` magic; ``LearnerModelParam`` (136 B: f32 base_score, u32 num_feature,
  i32 num_class, i32 contain_extra_attrs, i32 contain_eval_metrics, 29 reserved i32);
  objective name and booster name as (u64 length, bytes); ``GBLinearModelParam`` (136 B:
  u32 num_feature, i32 num_output_group, 32 reserved i32); the weights as (u64 count,
  f32[count]) with ``w[f * groups + g]`` and the biases ``w[num_feature * groups + g]``;
  then, when contain_extra_attrs, the attribute pairs (ignored);
* JSON (``save_model('*.json')``, xgboost >= 1.0): ``learner.gradient_booster.model.weights``
  in the same order, ``learner.learner_model_param.base_score``;
* text dump (``dump_model``, ``train.py:158``): ``bias:`` / ``weight:`` sections; the dump
  holds no base_score, so it must be given (the reference's file names carry it:
  ``...basescore2...``).

Prediction (xgboost 0.7 ``GBLinear::Pred``): per row and output group, in float32,
``psum = bias + base_score``, then for every feature in column order
``psum += float32(x_f) * w_f`` (separate multiply and add, no FMA), dense rows (the
DMatrix of a dense numpy array keeps zeros).  ``predict`` runs that loop on the GPU
(``expecto_gblinear_predict``, one thread per row, features staged through LDS), reading
float64 feature rows directly (the DMatrix conversion is the kernel's first rounding).
Parity of the arithmetic against xgboost itself is unpinned (xgboost absent); the CLI
plumbing around it is pinned by running the reference ``predict.py`` (tests/golden).
"""
from __future__ import annotations

import json
import struct
from dataclasses import dataclass, field

import numpy as np

_LEARNER_FMT = "<fIiii29i"          # LearnerModelParam, 136 bytes
_GBLINEAR_FMT = "<Ii32i"            # GBLinearModelParam, 136 bytes
assert struct.calcsize(_LEARNER_FMT) == 136 and struct.calcsize(_GBLINEAR_FMT) == 136


@dataclass
class GBLinear:
    """weights [num_feature, groups] f32, bias [groups] f32, base_score f32."""
    weights: np.ndarray
    bias: np.ndarray
    base_score: float
    objective: str = "reg:linear"
    attrs: dict = field(default_factory=dict)

    @property
    def num_feature(self) -> int:
        return int(self.weights.shape[0])

    @property
    def groups(self) -> int:
        return int(self.weights.shape[1])

    # -- formats ------------------------------------------------------------------------
    @classmethod
    def load(cls, path: str, base_score: float | None = None) -> "GBLinear":
        with open(path, "rb") as f:
            raw = f.read()
        head = raw.lstrip()[:1]
        if head == b"{":
            return cls._from_json(json.loads(raw.decode()))
        if raw.startswith(b"bias:") or raw.startswith(b"booster[0]:\nbias:"):
            return cls._from_dump(raw.decode(), base_score)
        return cls._from_legacy(raw)

    @classmethod
    def _from_legacy(cls, raw: bytes) -> "GBLinear":
        off = 4 if raw[:4] == b"binf" else 0
        if raw[:4] == b"bs64":
            raise ValueError("base64 xgboost models are not supported (nor by xgboost 0.7)")
        try:
            lp = struct.unpack_from(_LEARNER_FMT, raw, off)
        except struct.error as e:
            raise ValueError(f"not an xgboost model: {e}") from None
        base_score, num_feature, _num_class, extra_attrs = lp[0], lp[1], lp[2], lp[3]
        off += 136

        def read_str(o):
            (n,) = struct.unpack_from("<Q", raw, o)
            o += 8
            if n >= 0xFFFFFFFF:            # pre-0.6 layout: length in the high word + a gap
                o += 4
                n >>= 32
            return raw[o:o + n].decode(), o + n

        obj, off = read_str(off)
        gbm, off = read_str(off)
        if gbm != "gblinear":
            raise ValueError(f"booster {gbm!r} is not gblinear (ExPecto models are linear)")
        gp = struct.unpack_from(_GBLINEAR_FMT, raw, off)
        nf, groups = gp[0], gp[1]
        off += 136
        (count,) = struct.unpack_from("<Q", raw, off)
        off += 8
        if count != (nf + 1) * groups:
            raise ValueError(f"gblinear weight count {count} != (num_feature+1)*groups = {(nf + 1) * groups}")
        w = np.frombuffer(raw, dtype="<f4", count=count, offset=off).astype(np.float32)
        off += 4 * count
        attrs = {}
        if extra_attrs:
            (na,) = struct.unpack_from("<Q", raw, off)
            off += 8
            for _ in range(na):
                k, off = read_str(off)
                v, off = read_str(off)
                attrs[k] = v
        if num_feature and num_feature != nf:
            raise ValueError(f"learner num_feature {num_feature} != gblinear num_feature {nf}")
        w = w.reshape(nf + 1, groups)
        return cls(w[:nf].copy(), w[nf].copy(), float(np.float32(base_score)), obj, attrs)

    @classmethod
    def _from_json(cls, js: dict) -> "GBLinear":
        lrn = js["learner"]
        gb = lrn["gradient_booster"]
        if gb.get("name") != "gblinear":
            raise ValueError(f"booster {gb.get('name')!r} is not gblinear")
        mp = lrn["learner_model_param"]
        nf = int(mp["num_feature"])
        groups = max(1, int(mp.get("num_target", mp.get("num_class", 1)) or 1))
        w = np.asarray(gb["model"]["weights"], dtype=np.float32)
        if w.size != (nf + 1) * groups:
            raise ValueError("gblinear weight count does not match num_feature")
        w = w.reshape(nf + 1, groups)
        base = float(np.float32(float(str(mp["base_score"]).strip("[]"))))
        obj = lrn.get("objective", {}).get("name", "reg:linear")
        return cls(w[:nf].copy(), w[nf].copy(), base, obj)

    @classmethod
    def _from_dump(cls, text: str, base_score: float | None) -> "GBLinear":
        if base_score is None:
            raise ValueError("a gblinear text dump has no base_score: pass base_score=")
        lines = [l.strip() for l in text.splitlines() if l.strip() and not l.startswith("booster[")]
        bi, wi = lines.index("bias:"), lines.index("weight:")
        bias = np.array([float(x) for x in lines[bi + 1:wi]], dtype=np.float32)
        groups = bias.size
        w = np.array([float(x) for x in lines[wi + 1:]], dtype=np.float32).reshape(-1, groups)
        return cls(w, bias, float(np.float32(base_score)))

    def save_legacy(self, path: str) -> None:
        """Write the xgboost 0.7 binary layout described in the module docstring."""
        nf, g = self.weights.shape

        def wstr(s: str) -> bytes:
            b = s.encode()
            return struct.pack("<Q", len(b)) + b

        w = np.concatenate([self.weights.reshape(-1), self.bias.reshape(-1)]).astype("<f4")
        out = [b"binf", struct.pack(_LEARNER_FMT, np.float32(self.base_score), nf, 0, 0, 0, *([0] * 29)),
               wstr(self.objective), wstr("gblinear"), struct.pack(_GBLINEAR_FMT, nf, g, *([0] * 32)),
               struct.pack("<Q", w.size), w.tobytes()]
        with open(path, "wb") as f:
            f.write(b"".join(out))

    # -- scoring ------------------------------------------------------------------------
    def predict(self, X, cols=None, group: int = 0, out=None):
        """GPU gblinear margin of rows of X (float64 [n, ld] device tensor): feature j of a row
        is X[:, cols[j]] (cols: int32 device tensor or None = 0..num_feature-1)."""
        import torch

        from . import _lib

        lib = _lib.load()
        if X.dtype != torch.float64 or X.dim() != 2 or X.stride(1) != 1:
            raise RuntimeError("gblinear predict: X must be a float64 [n, ld] tensor with contiguous rows")
        n = X.shape[0]
        if cols is None:
            if X.shape[1] < self.num_feature:
                raise RuntimeError("gblinear predict: fewer columns than model features")
            cols = torch.arange(self.num_feature, dtype=torch.int32, device=X.device)
        if cols.numel() != self.num_feature:
            raise RuntimeError(f"model has {self.num_feature} features, {cols.numel()} columns given")
        w = torch.from_numpy(np.ascontiguousarray(self.weights[:, group])).to(X.device)
        init = float(np.float32(self.bias[group]) + np.float32(self.base_score))   # bias + base, in f32
        if out is None:
            out = torch.empty(n, dtype=torch.float32, device=X.device)
        _lib.check(lib.expecto_gblinear_predict(_lib.dptr(X), n, X.stride(0), _lib.dptr(cols.contiguous()),
                                                self.num_feature, _lib.dptr(w), float(init), _lib.dptr(out),
                                                _lib.stream_ptr()), "gblinear_predict")
        return out
