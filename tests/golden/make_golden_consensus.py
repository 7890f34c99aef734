"""Golden outputs of the reference eQTL / personal-genome scripts.

Run from the repo root (needs /root/reference; never read at test time):
    python tests/golden/make_golden_consensus.py

Runs ``geuvadis_sed_for_top_eqtls.py`` (2 eQTLs, + and - strand, one SNV inside the
200-window span and one 24 kb away from the TSS) and ``geuvadis_predict_consensus.py``
(2 genes x 2 samples, one sample truncated at a chromosome start -> N-padded) on seeded
synthetic 393,216-bp consensus FASTAs, with the seeded Beluga weights (make_golden.py) and a
seeded gblinear model of 20030 features (xgboost 0.7 binary layout), stubs on PYTHONPATH
(h5py -> .npz, Bio.SeqIO, natsort, seaborn, xgboost with a restated gblinear).
The sed run goes through ``forward_capture.py``, which records the reference Beluga forwards
(the per-window 200-shift chromatin predictions); the stub DMatrix records its features.
Writes tests/golden/consensus.npz (+ consensus_model.save, consensus_stdout.txt).
The inputs are regenerated at test time by ``write_inputs`` (same seed).
"""
from __future__ import annotations

import math
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = "/root/reference"
GOLD = os.path.join(REPO, "tests", "golden")
STUBS = os.path.join(GOLD, "stubs")
N = 393216
GENES = [("genea", "ENSG0000000A", 3, 1_000_000, "+"), ("geneb", "ENSG0000000B", 7, 2_500_000, "-")]


def _seq(rng, n):
    s = rng.choice(np.frombuffer(b"ACGTacgtN", np.uint8), n, p=[.24, .24, .24, .24, .01, .01, .005, .005, .01])
    return s.tobytes().decode()


def _fasta(path, rid, seq):
    with open(path, "w") as f:
        f.write(f">{rid} consensus\n")
        for i in range(0, len(seq), 60):
            f.write(seq[i:i + 60] + "\n")


def write_inputs(d: str) -> dict:
    """Consensus dir, gene/eQTL tables and the gblinear model under d; returns the paths."""
    import struct
    rng = np.random.default_rng(2024)
    cdir = os.path.join(d, "consensus")
    eqtl_rows = []
    for gi, (gene, ens, chrom, tss, strand) in enumerate(GENES):
        start = tss - N // 2
        os.makedirs(os.path.join(cdir, gene, "samples"))
        ref = _seq(rng, N)
        _fasta(os.path.join(cdir, gene, "ref.fa"), f"chr{chrom}:{start}-{start + N - 1}", ref)
        tss_i = N // 2
        snp_off = 730 if gi == 0 else -24_000            # inside the window span / outside it
        snp_i = tss_i + snp_off
        refb = ref[snp_i].upper()
        if refb not in "ACGT":
            ref = ref[:snp_i] + "A" + ref[snp_i + 1:]
            refb = "A"
            _fasta(os.path.join(cdir, gene, "ref.fa"), f"chr{chrom}:{start}-{start + N - 1}", ref)
        alt = "ACGT".replace(refb, "")[gi]
        eqtl_rows.append((gene, chrom, tss + snp_off, tss, refb, alt))
        for si in range(2):
            s = _seq(rng, N)
            if gi == 1 and si == 1:                      # truncated at the chromosome start
                _fasta(os.path.join(cdir, gene, "samples", f"HG{si:05d}.fa"), f"chr{chrom}:-{1000}-{N - 1001}",
                       s[1000:])
            else:
                _fasta(os.path.join(cdir, gene, "samples", f"HG{si:05d}.fa"), f"chr{chrom}:{start}-{start + N - 1}", s)
    genes_csv = os.path.join(d, "genes.csv")
    with open(genes_csv, "w") as f:
        for gene, ens, chrom, tss, strand in GENES:
            f.write(f"{ens},{chrom},{tss},{gene.upper()},{strand}\n")
    eqtls_csv = os.path.join(d, "eqtls.csv")
    with open(eqtls_csv, "w") as f:
        f.write("name,CHR_SNP,SNPpos,TSSpos_x,REF,ALT\n")
        for r in eqtl_rows:
            f.write(",".join(map(str, r)) + "\n")
    model = os.path.join(d, "model.save")
    w = np.concatenate([np.random.default_rng(13).normal(0, 0.02, 20030), [0.25]]).astype("<f4")
    st = lambda x: struct.pack("<Q", len(x)) + x.encode()
    with open(model, "wb") as f:
        f.write(b"binf" + struct.pack("<fIiii29i", 2.0, 20030, 0, 0, 0, *([0] * 29)) + st("reg:linear") +
                st("gblinear") + struct.pack("<Ii32i", 20030, 1, *([0] * 32)) + struct.pack("<Q", w.size) + w.tobytes())
    return {"consensus": cdir, "genes_csv": genes_csv, "eqtls_csv": eqtls_csv, "model": model}


def main():
    import torch
    sys.path.insert(0, REPO)
    from oracle import weights as oweights
    work = tempfile.mkdtemp(prefix="expecto_golden_consensus_")
    paths = write_inputs(work)
    sd = oweights.seeded_state_dict(0)
    torch.save(sd, os.path.join(work, "beluga.pth"))
    env = dict(os.environ, PYTHONPATH=STUBS + ":" + REF, OMP_NUM_THREADS="8")
    out1 = subprocess.run([sys.executable, os.path.join(GOLD, "forward_capture.py"),
                           os.path.join(REF, "geuvadis_sed_for_top_eqtls.py"), paths["model"],
                           paths["consensus"], paths["genes_csv"], paths["eqtls_csv"], "--beluga_model",
                           os.path.join(work, "beluga.pth"), "-o", "sed_out"], cwd=work, env=env,
                          capture_output=True, text=True, check=True)
    # the sed run's per-window forwards (one [400, 2002] call per eQTL and allele: 200 shifts fwd
    # then rc) and its two feature matrices (stub DMatrix: ref then alt, [n_eqtl, 20030] f64)
    with np.load(os.path.join(work, "captured_forward.npz")) as z:
        fw = [z[f"arr_{i}"] for i in range(len(z.files))]
    assert len(fw) == 2 * len(GENES) and all(a.shape == (400, 2002) for a in fw), [a.shape for a in fw]
    sed_feats = [np.load(os.path.join(work, f"captured_dmatrix_{i}.npy")) for i in range(2)]
    out2 = subprocess.run([sys.executable, os.path.join(REF, "geuvadis_predict_consensus.py"), paths["model"],
                           paths["consensus"], paths["genes_csv"], "--beluga_model", os.path.join(work, "beluga.pth"),
                           "-o", "cons_out"], cwd=work, env=env, capture_output=True, text=True, check=True)
    res = {}
    for gi, (gene, *_) in enumerate(GENES):
        # chromatin predictions of the 200-shift sed path: every window whose alt differs from its
        # ref (the SNV's cone) and every 8th window, every 5th feature; full-row f64 sums of all
        ref_w, alt_w = fw[2 * gi], fw[2 * gi + 1]
        rows = np.union1d(np.nonzero((ref_w != alt_w).any(1))[0], np.arange(0, 400, 8))
        res[f"sed_win_rows_{gene}"] = rows
        res[f"sed_win_ref_{gene}"] = ref_w[rows, ::5]
        res[f"sed_win_alt_{gene}"] = alt_w[rows, ::5]
        res[f"sed_win_refsum_{gene}"] = ref_w.astype(np.float64).sum(1)
        res[f"sed_win_altsum_{gene}"] = alt_w.astype(np.float64).sum(1)
        res[f"sed_feat_ref_{gene}"] = sed_feats[0][gi, ::4]
        res[f"sed_feat_alt_{gene}"] = sed_feats[1][gi, ::4]
    for gene, *_ in GENES:
        g = gene
        with np.load(os.path.join(work, "sed_out", g, f"{g}.h5.npz")) as z:
            res[f"sed_ref_{gene}"] = z["ref_preds"]
            res[f"sed_alt_{gene}"] = z["alt_preds"]
        with np.load(os.path.join(work, "cons_out", gene, f"{gene}.h5.npz")) as z:
            res[f"cons_preds_{gene}"] = z["expecto_preds"]
            res[f"cons_ids_{gene}"] = z["record_ids"]
        with np.load(os.path.join(work, "cons_out", gene, f"{gene}_chromatin.h5.npz")) as z:
            cp = z["chromatin_preds"]
            res[f"cons_chrom_rows_{gene}"] = cp[:, ::25, ::7]
            res[f"cons_chrom_shape_{gene}"] = np.array(cp.shape)
            res[f"cons_chrom_sum_{gene}"] = cp.sum(axis=(1, 2))
    np.savez_compressed(os.path.join(GOLD, "consensus.npz"), **res)
    with open(os.path.join(GOLD, "consensus_stdout.txt"), "w") as f:
        f.write(out2.stdout)
    shutil.copy(paths["model"], os.path.join(GOLD, "consensus_model.save"))
    shutil.rmtree(work)
    print("consensus golden written; stdout:", out1.stdout[-200:], out2.stdout[-200:])


if __name__ == "__main__":
    main()
