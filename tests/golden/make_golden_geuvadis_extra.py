"""Golden outputs of the remaining reference geuvadis scripts (VERDICT r02 "missing" 1-3):

* ``geuvadis_predict_ref_all_genes.py`` -- reference-genome consensus (``{gene}/ref.fa``,
  393,216 bp, TSS at len // 2) per gene of a genes table: 200 shifts x fwd/rc, float64 mean,
  legacy 20030 features, gblinear score -> ``ref_preds.csv``.  3 genes: + strand, - strand
  with the record truncated at the chromosome start (N-padded), and one whose gene symbol is
  empty (the Ensembl id names it).
* ``geuvadis_predict_consensus_for_top_eqtls.py`` -- per gene of its fixed list (HLA-B, HLA-C,
  RPL28, CPAMD8, TMEM121B, SCN11A) one gzipped Basenji-length (131,072 bp) consensus record
  whose id carries the strand (TSS at (len - 1) // 2 on +, len // 2 on -) -> ``{gene}.h5`` with
  ``preds``, ``record_ids`` and the 41,800-bp ``seqs``.  One record per file: the script's
  feature concatenation (np.zeros((1, 10, 1)) against n records) only runs for n = 1.
* ``merge_geuvadis_predict_consensus.py`` -- run on the for_top_eqtls outputs.

Run from the repo root (needs /root/reference; never read at test time):
    python tests/golden/make_golden_geuvadis_extra.py
Stubs on PYTHONPATH as make_golden_consensus.py (h5py -> .npz, Bio.SeqIO, natsort, seaborn,
matplotlib, xgboost with the restated gblinear); the reference Beluga forwards are recorded by
forward_capture.py.  Writes tests/golden/geuvadis_extra.npz and geuvadis_ref_preds.csv.  The
inputs are regenerated at test time by ``write_inputs`` (same seed).
"""
from __future__ import annotations

import glob
import gzip
import hashlib
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
N_ENF = 393216
N_BASENJI = 131072
REF_GENES = [("ENSG00000000011", 5, 1_500_000, "GENEA", "+"), ("ENSG00000000022", 9, 150_000, "GENEB", "-"),
             ("ENSG00000000033", 11, 3_000_000, "", "+")]
TOP_GENES = ['HLA-B', 'HLA-C', 'RPL28', 'CPAMD8', 'TMEM121B', 'SCN11A']   # the script's list (:73)


def _seq(rng, n):
    s = rng.choice(np.frombuffer(b"ACGTacgtN", np.uint8), n, p=[.24, .24, .24, .24, .01, .01, .005, .005, .01])
    return s.tobytes().decode()


def _fasta_text(rid, seq):
    return f">{rid} consensus\n" + "".join(seq[i:i + 60] + "\n" for i in range(0, len(seq), 60))


def write_inputs(d: str) -> dict:
    rng = np.random.default_rng(77)
    ref_dir = os.path.join(d, "ref_consensus")
    for ens, chrom, tss, sym, strand in REF_GENES:
        gene = (sym or ens).lower()
        os.makedirs(os.path.join(ref_dir, gene))
        start = tss - N_ENF // 2
        s = _seq(rng, N_ENF)
        if start < 0:        # truncated at the chromosome start: the record lacks the first -start bases
            rid, s = f"chr{chrom}:-{-start}-{start + N_ENF - 1}", s[-start:]
        else:
            rid = f"chr{chrom}:{start}-{start + N_ENF - 1}"
        with open(os.path.join(ref_dir, gene, "ref.fa"), "w") as f:
            f.write(_fasta_text(rid, s))
    genes_csv = os.path.join(d, "ref_genes.csv")
    with open(genes_csv, "w") as f:
        for ens, chrom, tss, sym, strand in REF_GENES:
            f.write(f"{ens},{chrom},{tss},{sym},{strand}\n")
    top_dir = os.path.join(d, "top_consensus")
    eq = []
    for gi, g in enumerate(TOP_GENES):
        gene = g.lower()
        os.makedirs(os.path.join(top_dir, gene))
        strand = "+-"[gi % 2]
        start = 30_000_000 + 1_000_000 * gi
        # one sample (the same id in every gene's file, as the merge script requires)
        rid = f"chr6:{start}-{start + N_BASENJI - 1}|NA20828|{strand}|1pIu"
        with gzip.open(os.path.join(top_dir, gene, f"{gene}.fa.gz"), "wt") as f:
            f.write(_fasta_text(rid, _seq(rng, N_BASENJI)))
        eq.append((g, f"ENSG9{gi:010d}", 6, start + 60_000 + 17 * gi))
    eqtls_csv = os.path.join(d, "top_eqtls.csv")
    with open(eqtls_csv, "w") as f:
        f.write("name,geneID,CHR_SNP,SNPpos\n")
        for name, gid, c, p in eq:
            f.write(f"{name if name != 'RPL28' else ''},{gid},{c},{p}\n")
    vcf = os.path.join(d, "top_snps.vcf")
    with open(vcf, "w") as f:
        f.write("##fileformat=VCFv4.2\n")
        for name, gid, c, p in eq + eq[:2]:              # duplicated rows are dropped by the script
            f.write(f"chr{c}\t{p}\t.\tA\tG\n")
    return {"ref_dir": ref_dir, "genes_csv": genes_csv, "top_dir": top_dir, "eqtls_csv": eqtls_csv, "vcf": vcf,
            "model": os.path.join(GOLD, "consensus_model.save")}


def main():
    import torch
    sys.path.insert(0, REPO)
    from oracle import weights as oweights
    work = tempfile.mkdtemp(prefix="expecto_golden_geuvadis_")
    paths = write_inputs(work)
    torch.save(oweights.seeded_state_dict(0), os.path.join(work, "beluga.pth"))
    env = dict(os.environ, PYTHONPATH=STUBS + ":" + REF, OMP_NUM_THREADS="8")
    res = {}
    # --- geuvadis_predict_ref_all_genes.py
    r1 = os.path.join(work, "r1")
    os.makedirs(r1)
    subprocess.run([sys.executable, os.path.join(GOLD, "forward_capture.py"),
                    os.path.join(REF, "geuvadis_predict_ref_all_genes.py"), paths["model"], paths["ref_dir"],
                    paths["genes_csv"], "--beluga_model", os.path.join(work, "beluga.pth"), "-o", "out"],
                   cwd=r1, env=env, capture_output=True, text=True, check=True)
    with np.load(os.path.join(r1, "captured_forward.npz")) as z:
        fw = [z[f"arr_{i}"] for i in range(len(z.files))]
    assert len(fw) == len(REF_GENES) and all(a.shape == (400, 2002) for a in fw)
    for gi, a in enumerate(fw):
        res[f"ref_win_{gi}"] = a[::8, ::5]
        res[f"ref_winsum_{gi}"] = a.astype(np.float64).sum(1)
        res[f"ref_feat_{gi}"] = np.load(os.path.join(r1, f"captured_dmatrix_{gi}.npy"))[0, ::4]
    shutil.copy(os.path.join(r1, "out", "ref_preds.csv"), os.path.join(GOLD, "geuvadis_ref_preds.csv"))
    # --- geuvadis_predict_consensus_for_top_eqtls.py
    r2 = os.path.join(work, "r2")
    os.makedirs(r2)
    out2 = subprocess.run([sys.executable, os.path.join(GOLD, "forward_capture.py"),
                           os.path.join(REF, "geuvadis_predict_consensus_for_top_eqtls.py"), paths["model"],
                           paths["top_dir"], paths["eqtls_csv"], paths["vcf"], "--beluga_model",
                           os.path.join(work, "beluga.pth"), "-o", "out"],
                          cwd=r2, env=env, capture_output=True, text=True, check=True)
    with np.load(os.path.join(r2, "captured_forward.npz")) as z:
        fw = [z[f"arr_{i}"] for i in range(len(z.files))]
    assert len(fw) == len(TOP_GENES) and all(a.shape == (400, 2002) for a in fw)
    for gi, g in enumerate(TOP_GENES):
        gene = g.lower()
        res[f"top_win_{gi}"] = fw[gi][::8, ::5]
        res[f"top_winsum_{gi}"] = fw[gi].astype(np.float64).sum(1)
        res[f"top_feat_{gi}"] = np.load(os.path.join(r2, f"captured_dmatrix_{gi}.npy"))[0, ::4]
        with np.load(os.path.join(r2, "out", gene, f"{gene}.h5.npz")) as z:
            res[f"top_preds_{gi}"] = z["preds"]
            res[f"top_ids_{gi}"] = z["record_ids"]
            res[f"top_seq_sha1_{gi}"] = np.array([hashlib.sha1(bytes(s)).hexdigest() for s in z["seqs"]], "S")
            res[f"top_seq_len_{gi}"] = np.array([len(bytes(s)) for s in z["seqs"]])
    res["top_stdout"] = np.array(out2.stdout.encode())
    # --- merge_geuvadis_predict_consensus.py over the for_top_eqtls outputs (stub h5: the .h5
    # paths the script globs must exist beside their .npz)
    for f in glob.glob(os.path.join(r2, "out", "*", "*.h5.npz")):
        open(f[:-4], "w").close()
    subprocess.run([sys.executable, os.path.join(REF, "merge_geuvadis_predict_consensus.py"), "--batch_dir",
                    os.path.join(r2, "out"), "--n_genes", str(len(TOP_GENES)), "-o", "merged"],
                   cwd=r2, env=env, capture_output=True, text=True, check=True)
    with np.load(os.path.join(r2, "merged", "expecto_preds.h5.npz")) as z:
        for k in ("record_ids", "genes", "preds"):
            res[f"merge_{k}"] = z[k]
    np.savez_compressed(os.path.join(GOLD, "geuvadis_extra.npz"), **res)
    shutil.rmtree(work)
    print("geuvadis extra golden written")


if __name__ == "__main__":
    main()
