"""Golden outputs of the reference ``predict.py`` CLI (sed.tsv and its two sorted copies).

Run from the repo root (needs /root/reference; never read at test time):
    python tests/golden/make_golden_predict.py

Inputs are the fixtures already committed by make_golden.py: the reference chromatin.py
outputs for shifts 0/-200/200 (chromatin.npz) and the coordinate / gene-association rows
(predict_features.npz).  Two seeded synthetic gblinear models are written in xgboost 0.7's
binary layout (struct-packed here, independently of expecto_amd.xgblinear), and the reference
predict.py runs with tests/golden/stubs on PYTHONPATH (h5py reads the .npz captures; xgboost's
gblinear prediction is restated in stubs/xgboost.py since xgboost is not installed).

Runs:  all   -- every feature kept, --batchSize 3 (3 batches over 7 rows);
       notf  -- --no_tf_features --no_pol2 (keep-mask column selection), default batch size.
Writes tests/golden/predict_sed/<run>/{model.save, stdout.txt, sed.tsv,
sed_sorted_by_magnitude.tsv, sed_sorted_by_proportion.tsv}.
"""
from __future__ import annotations

import os
import shutil
import struct
import subprocess
import sys
import tempfile

import numpy as np
import pandas as pd

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = "/root/reference"
GOLD = os.path.join(REPO, "tests", "golden")
STUBS = os.path.join(GOLD, "stubs")
FEATURES_TSV = os.path.join(REF, "resources", "deepsea_beluga_2002_features.tsv")


def write_model(path, n_feature, seed):
    rng = np.random.default_rng(seed)
    w = np.concatenate([rng.normal(0, 0.02, n_feature), [0.37]]).astype("<f4")   # weights, then bias

    def s(x):
        b = x.encode()
        return struct.pack("<Q", len(b)) + b

    with open(path, "wb") as f:
        f.write(b"binf" + struct.pack("<fIiii29i", 2.0, n_feature, 0, 0, 0, *([0] * 29)) + s("reg:linear") +
                s("gblinear") + struct.pack("<Ii32i", n_feature, 1, *([0] * 32)) + struct.pack("<Q", w.size) +
                w.tobytes())


def keep_count(no_tf, no_pol2):
    df = pd.read_csv(FEATURES_TSV, sep="\t", index_col=0)
    m = np.ones(len(df), bool)
    if no_tf:
        m &= (df["Assay type"] != "TF").to_numpy()
    if no_pol2:
        m &= ~df["Assay"].str.startswith("Pol").to_numpy()
    return int(m.sum())


def main():
    chrom = np.load(os.path.join(GOLD, "chromatin.npz"))
    feats = np.load(os.path.join(GOLD, "predict_features.npz"))
    work = tempfile.mkdtemp(prefix="expecto_golden_predict_")
    os.makedirs(os.path.join(work, "out"))
    for s in (0, -200, 200):
        np.savez(os.path.join(work, "out", f"snps.shift_{s}.diff.h5.npz"),
                 **{k: chrom[f"{k}_{s}"] for k in ("diff", "ref", "alt")})
    with open(os.path.join(work, "coor.vcf"), "w") as f:
        f.write("##fileformat=VCFv4.3\n")
        for r in feats["coor_rows"]:
            f.write(str(r) + "\n")
    with open(os.path.join(work, "genes.tsv"), "w") as f:
        for r in feats["gene_rows"]:
            f.write(str(r) + "\n")
    env = dict(os.environ, PYTHONPATH=STUBS + ":" + REF, OMP_NUM_THREADS="8")
    runs = {"all": (["--batchSize", "3"], False, False, 11), "notf": (["--no_tf_features", "--no_pol2"], True, True, 12)}
    for name, (extra, no_tf, no_pol2, seed) in runs.items():
        dst = os.path.join(GOLD, "predict_sed", name)
        os.makedirs(dst, exist_ok=True)
        model = os.path.join(dst, "model.save")
        write_model(model, 10 * keep_count(no_tf, no_pol2), seed)
        pwork = os.path.join(work, name)
        os.makedirs(pwork)
        out = subprocess.run([sys.executable, os.path.join(REF, "predict.py"), "--model_save_file", model,
                              "--belugaFeatures", FEATURES_TSV, "--coorFile_chromatin", os.path.join(work, "coor.vcf"),
                              "--geneFile", os.path.join(work, "genes.tsv"),
                              "--snpEffectFilePattern", os.path.join(work, "out", "snps.shift_SHIFT.diff.h5"),
                              "--maxshift", "200", "-o", "pout", *extra], cwd=pwork, env=env, capture_output=True,
                             text=True, check=True)
        with open(os.path.join(dst, "stdout.txt"), "w") as f:
            f.write(out.stdout)
        for t in ("sed.tsv", "sed_sorted_by_magnitude.tsv", "sed_sorted_by_proportion.tsv"):
            shutil.copy(os.path.join(pwork, "pout", t), os.path.join(dst, t))
    shutil.copy(FEATURES_TSV, os.path.join(GOLD, "predict_sed", "deepsea_beluga_2002_features.tsv"))
    shutil.rmtree(work)
    print("predict.py golden outputs written to", os.path.join(GOLD, "predict_sed"))


if __name__ == "__main__":
    main()
