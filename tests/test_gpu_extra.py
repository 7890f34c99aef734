"""GPU: peak-masked TSS features (expecto_intersect_chip_atac.py drop-in, expecto_amd.tss
intersect) against the reference's output on seeded inputs (tests/golden/make_golden_extra.py)."""
import os
import sys

import numpy as np
import pytest

from conftest import GOLDEN, assert_close

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("tf_only", [False, True])
def test_atac_x_chip_features_match_reference(tmp_path, tf_only):
    sys.path.insert(0, GOLDEN)
    import make_golden_extra as mg
    from expecto_amd import tss
    p = mg.write_inputs(str(tmp_path))
    out = tmp_path / "ix"
    feats = tss.intersect_main([p["tss_anno"], p["peaks"], "-o", str(out), "--genome",
                                str(tmp_path / "resources" / "hg19.fa"), "--synthetic-weights", "0",
                                "--features_tsv", os.path.join(GOLDEN, "predict_sed", "deepsea_beluga_2002_features.tsv"),
                                "--gene-batch", "3"] + (["--tf_only"] if tf_only else []))
    want = np.load(os.path.join(GOLDEN, "extra", "atac_x_chip_tf.npy" if tf_only else "atac_x_chip.npy"))
    saved = np.load(out / "Xreducedall.2002.atac_x_chip.npy")
    assert saved.dtype == np.float64 and saved.shape == want.shape == (4, 20020)
    assert_close(saved, want, what="atac x chip features")
    assert np.array_equal(saved, feats)
