"""Generate the golden vectors by running the REFERENCE in this (build) container.

Run from the repo root:  python tests/golden/make_golden.py
Needs /root/reference (read-only) -- it is never read at test time; only the
fixtures written here (tests/golden/*.npz, *.json, *.txt) are.

What runs (SURVEY.md 8c recipe):
  1. weights: reference ``Beluga()`` after ``torch.manual_seed(0)``, every weight x sqrt(6);
     checked equal to ``oracle.weights.seeded_state_dict`` and pinned by checksum.
  2. ``Beluga.forward`` (Beluga.py:50) on encoded synthetic windows (+ rc, + all-N).
  3. ``expecto_utils.encodeSeqs`` (expecto_utils.py:5-39) on encoder edge cases.
  4. ``chromatin.py`` end-to-end (SNVs, an unprefixed contig, a ref mismatch, a
     non-canonical contig, an insertion and a deletion; --maxshift 200) with
     pyfasta/h5py/liftover replaced by the stand-ins in tests/golden/stubs.
  5. ``predict.py``'s feature matrices (predict.py:87-147) for those outputs, captured
     from the xgboost stand-in.
  6. ``compute_expecto_features.py`` (2 genes) and ``replicate_expecto_features.py``
     (1 gene) on the synthetic genome.
"""
from __future__ import annotations

import json
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
sys.path.insert(0, REPO)

from expecto_amd import synthetic  # noqa: E402
from oracle import weights as oweights  # noqa: E402

GENOME_ARGS = dict(n_contigs=3, contig_len=60000, seed=7)


def ref_state_dict():
    import torch
    sys.path.insert(0, REF)
    import Beluga as RB
    torch.manual_seed(0)
    m = RB.Beluga()
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    for k in sd:
        if k.endswith(".weight"):
            sd[k].mul_(math.sqrt(6.0))
    m.load_state_dict(sd)
    m.eval()
    return m, sd


def main():
    import torch
    torch.set_num_threads(8)
    model, sd = ref_state_dict()
    mine = oweights.seeded_state_dict(0)
    for k in sd:
        assert torch.equal(sd[k], mine[k]), k
    with open(os.path.join(GOLD, "weights_checksum.json"), "w") as f:
        json.dump({"seed": 0, "gain": "sqrt(6)", "checksum": oweights.checksum(sd)}, f, indent=1)

    genome = synthetic.genome_bytes(**GENOME_ARGS)
    sys.path.insert(0, REF)
    from expecto_utils import encodeSeqs

    # ---- 2. forward golden ------------------------------------------------------------
    g1 = genome["chr1"].decode()
    seqs = [g1[10000:12000], g1[30500:32500], "N" * 2000]
    x = encodeSeqs(seqs, inputsize=2000).astype(np.float32)           # [6,4,2000]
    with torch.no_grad():
        y = model.forward(torch.from_numpy(x).unsqueeze(2)).numpy()
    np.savez_compressed(os.path.join(GOLD, "forward.npz"),
                        seqs=np.array([s.encode() for s in seqs]), y=y)

    # ---- 3. encoder golden --------------------------------------------------------------
    rng = np.random.default_rng(3)
    alpha = np.array(list("ACGTacgtNnH-"))
    enc_seqs = ["".join(rng.choice(alpha, n)) for n in (2000, 2001, 2100, 2101, 2003)]
    enc = encodeSeqs(enc_seqs, inputsize=2000)
    np.savez_compressed(os.path.join(GOLD, "encode.npz"),
                        seqs=np.array([s.encode() for s in enc_seqs]), onehot=np.packbits(enc, axis=-1))

    # ---- 4. chromatin.py end-to-end -----------------------------------------------------
    work = tempfile.mkdtemp(prefix="expecto_golden_")
    os.makedirs(os.path.join(work, "resources"))
    synthetic.write_fasta(os.path.join(work, "resources", "hg19.fa"), genome)
    torch.save(sd, os.path.join(work, "resources", "deepsea.beluga.pth"))
    c1, c2, c3 = genome["chr1"], genome["chr2"], genome["chr3"]
    up = lambda b: chr(b).upper()
    b = lambda c, p: up(c[p - 1])               # 1-based base
    snv_alt = lambda r: "ACGT".replace(r, "")[0] if r in "ACGT" else "A"
    vcf_rows = [
        ("chr1", 20001, "-", b(c1, 20001), snv_alt(b(c1, 20001))),
        ("2", 30001, "-", b(c2, 30001), snv_alt(b(c2, 30001))),       # no chr prefix
        ("chr2", 25000, "-", snv_alt(b(c2, 25000)), b(c2, 25000)),    # ref mismatch
        ("chrUn_gl000220", 100, "-", "A", "G"),                       # filtered by CHRS
        ("chr3", 40000, "-", b(c3, 40000), b(c3, 40000) + "T"),       # insertion
        ("chr3", 45000, "-", b(c3, 45000) + b(c3, 45001) + b(c3, 45002), b(c3, 45000)),  # deletion
        ("chr1", 41234, "-", b(c1, 41234), snv_alt(b(c1, 41234))),
    ]
    with open(os.path.join(work, "in.vcf"), "w") as f:
        f.write("##fileformat=VCFv4.1\n")
        for r in vcf_rows:
            f.write("\t".join(map(str, r)) + "\n")
    env = dict(os.environ, PYTHONPATH=STUBS + ":" + REF, OMP_NUM_THREADS="8")
    out = subprocess.run([sys.executable, os.path.join(REF, "chromatin.py"), "in.vcf", "--maxshift", "200",
                          "--batchsize", "4", "--output_dir", "out"], cwd=work, env=env,
                         capture_output=True, text=True, check=True)
    stdout_lines = [l for l in out.stdout.splitlines() if l.startswith("Number of")]
    shifts = [0, -200, 200]
    chrom = {}
    for s in shifts:
        with np.load(os.path.join(work, "out", f"snps.shift_{s}.diff.h5.npz")) as z:
            for k in ("diff", "ref", "alt"):
                chrom[f"{k}_{s}"] = z[k]
    with open(os.path.join(work, "out", "snps_hg19.vcf")) as f:
        vcf_out = f.read()
    np.savez_compressed(os.path.join(GOLD, "chromatin.npz"), **chrom)
    with open(os.path.join(GOLD, "chromatin_vcf.txt"), "w") as f:
        for r in vcf_rows:
            f.write("\t".join(map(str, r)) + "\n")
    with open(os.path.join(GOLD, "chromatin_snps_hg19.vcf"), "w") as f:
        f.write(vcf_out)
    with open(os.path.join(GOLD, "chromatin_stdout.txt"), "w") as f:
        f.write("\n".join(stdout_lines) + "\n")

    # ---- 5. predict.py feature matrices ---------------------------------------------------
    canon = [r for r in vcf_rows if not r[0].startswith("chrUn")]
    with open(os.path.join(work, "coor.vcf"), "w") as f:
        f.write("##fileformat=VCFv4.3\n")
        for r in canon:
            f.write("\t".join(map(str, r)) + "\n")
    grng = np.random.default_rng(5)
    gene_rows = []
    for i, r in enumerate(canon):
        for j in range(2 if i == 0 else 1):
            tss = r[1] + int(grng.integers(-1500, 1500))
            strand = "+" if grng.random() < 0.5 else "-"
            gene_rows.append((r[0].replace("chr", ""), r[1] - 1, r[1], r[3], r[4], r[0].replace("chr", ""),
                              tss - 1, tss, strand, f"ENSG{i:05d}{j}", tss - r[1]))
    with open(os.path.join(work, "genes.tsv"), "w") as f:
        for r in gene_rows:
            f.write("\t".join(map(str, r)) + "\n")
    pwork = os.path.join(work, "pred")
    os.makedirs(pwork)
    subprocess.run([sys.executable, os.path.join(REF, "predict.py"), "--model_save_file", "none",
                    "--belugaFeatures", os.path.join(REF, "resources", "deepsea_beluga_2002_features.tsv"),
                    "--coorFile_chromatin", os.path.join(work, "coor.vcf"),
                    "--geneFile", os.path.join(work, "genes.tsv"),
                    "--snpEffectFilePattern", os.path.join(work, "out", "snps.shift_SHIFT.diff.h5"),
                    "--maxshift", "200", "-o", "pout"], cwd=pwork, env=env, capture_output=True,
                   text=True, check=True)
    cap = [np.load(os.path.join(pwork, f"captured_dmatrix_{i}.npy")) for i in range(4)]
    np.savez_compressed(os.path.join(GOLD, "predict_features.npz"), diff=cap[1], ref=cap[2], alt=cap[3],
                        gene_rows=np.array(["\t".join(map(str, r)) for r in gene_rows]),
                        coor_rows=np.array(["\t".join(map(str, r)) for r in canon]))

    # ---- 6. TSS scripts ---------------------------------------------------------------------
    with open(os.path.join(work, "anno.csv"), "w") as f:
        f.write("id,symbol,seqnames,strand,TSS,CAGE_representative_TSS,type\n")
        f.write("ENSGT0001,G1,chr1,+,30000,30000,protein_coding\n")
        f.write("ENSGT0002,G2,chr2,-,29000,29123,protein_coding\n")
    with open(os.path.join(work, "tss.tsv"), "w") as f:
        f.write("idx\tens_id\tchrom\ttss\tstrand\tcount\tis_default\n")
        f.write("0\tENSGT0002\tchr2\t29123\t-\t5\tTrue\n")
    subprocess.run([sys.executable, "-c",
                    "import sys; sys.argv=['c','anno.csv','tss.tsv','-o','tss_out'];"
                    "sys.path.insert(0,'/root/reference'); import compute_expecto_features as m; m.main()"],
                   cwd=work, env=env, capture_output=True, text=True, check=True)
    feats = np.load(os.path.join(work, "tss_out", "Xreducedall.2002.representative_tss_top.npy"))
    with open(os.path.join(work, "anno1.csv"), "w") as f:
        f.write("id,symbol,seqnames,strand,TSS,CAGE_representative_TSS,type\n")
        f.write("ENSGT0002,G2,chr2,-,29000,29123,protein_coding\n")
    subprocess.run([sys.executable, "-c",
                    "import sys; sys.argv=['r','anno1.csv','-o','rep_out'];"
                    "sys.path.insert(0,'/root/reference'); import replicate_expecto_features as m; m.main()"],
                   cwd=work, env=env, capture_output=True, text=True, check=True)
    rep = np.load(os.path.join(work, "rep_out", "ENSGT0002.npy"))
    np.savez_compressed(os.path.join(GOLD, "tss.npz"), features=feats, rep_rows=rep[::8], rep_shape=np.array(rep.shape),
                        rep_sum=np.array([rep.astype(np.float64).sum(), (rep.astype(np.float64) ** 2).sum()]))
    shutil.rmtree(work)
    print("golden vectors written to", GOLD)


if __name__ == "__main__":
    main()
