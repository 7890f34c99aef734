"""CPU restatement of the ExPecto expression scoring -- TEST INFRASTRUCTURE (oracle) ONLY.

``predict.py:150-166`` scores feature rows with an xgboost gblinear booster
(``xgboost==0.7.post4``, ``requirements.txt``; not installed here).  Its published
prediction rule (GBLinear::Pred) per row, in float32: ``psum = bias + base_score``, then
``psum += float32(x_f) * w_f`` for the features in column order, each product and each sum
rounded separately.  Pinned against the reference predict.py run with the restated booster
(tests/golden/make_golden_predict.py); parity with xgboost itself is unpinned.
"""
from __future__ import annotations

import numpy as np


def predict(x: np.ndarray, w: np.ndarray, bias: float, base_score: float) -> np.ndarray:
    """x [n, F] (any float dtype; converted to float32 like a DMatrix), w [F] f32 -> f32 [n]."""
    x = np.asarray(x).astype(np.float32)
    w = np.asarray(w, dtype=np.float32)
    psum = np.full(x.shape[0], np.float32(np.float32(bias) + np.float32(base_score)), dtype=np.float32)
    for f in range(w.shape[0]):
        psum = np.add(psum, np.multiply(x[:, f], w[f], dtype=np.float32), dtype=np.float32)
    return psum


def keep_columns(keep_mask: np.ndarray, nfeat: int = 2002) -> np.ndarray:
    """Column of model feature j in the [n, 10*nfeat] matrix (predict.py:137-145)."""
    keep = np.nonzero(keep_mask)[0]
    return (np.arange(10)[:, None] * nfeat + keep[None, :]).reshape(-1)
