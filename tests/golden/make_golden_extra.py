"""Golden outputs of the reference make_closest_genes_file.py and expecto_intersect_chip_atac.py
(SURVEY.md §8f row 4), run in this container with stubs (pyfasta, liftover, h5py, pybedtools).

    python tests/golden/make_golden_extra.py      (needs /root/reference; never read by tests)

Inputs are regenerated at test time by ``write_inputs`` (seeded).  Writes
tests/golden/extra/{closest_genes.tsv, closest_genes_rf.tsv, snps_hg19.vcf, snps_hg19_rf.vcf,
atac_x_chip.npy, atac_x_chip_tf.npy}.
"""
from __future__ import annotations

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
GENOME_ARGS = dict(n_contigs=3, contig_len=60000, seed=7)       # = make_golden.GENOME_ARGS


def write_inputs(d: str) -> dict:
    sys.path.insert(0, REPO)
    from expecto_amd import synthetic
    os.makedirs(os.path.join(d, "resources"), exist_ok=True)
    synthetic.write_fasta(os.path.join(d, "resources", "hg19.fa"), synthetic.genome_bytes(**GENOME_ARGS))
    rng = np.random.default_rng(31)
    anno = os.path.join(d, "geneanno.csv")
    genes = []
    with open(anno, "w") as f:
        f.write("id,symbol,seqnames,strand,TSS,CAGE_representative_TSS,type\n")
        for i, (chrom, tss) in enumerate([("chr1", 25000), ("chr1", 33000), ("chr2", 27000), ("chr3", 31000),
                                          ("chr1", 52000), ("chr2", 24000)]):
            strand = "+" if i % 2 == 0 else "-"
            f.write(f"ENSG{i:011d},G{i},{chrom},{strand},{tss + 17},{tss},protein_coding\n")
            genes.append((chrom, tss))
    vcf = os.path.join(d, "snps.vcf")
    with open(vcf, "w") as f:
        f.write("##fileformat=VCFv4.3\n")
        for chrom, pos in [("chr1", 24000), ("chr1", 29000), ("chr2", 45000), ("chr3", 12000), ("chr1", 53111),
                           ("chr2", 25500)]:
            f.write(f"{chrom}\t{pos}\t-\tA\tG\n")
    peaks = os.path.join(d, "peaks.bed")
    with open(peaks, "w") as f:
        for chrom, tss in genes[:4]:
            for _ in range(12):
                s = int(tss + rng.integers(-21000, 21000))
                f.write(f"{chrom}\t{s}\t{s + int(rng.integers(50, 900))}\tpeak\n")
    tss_anno = os.path.join(d, "tss_anno.csv")                   # the genes the TSS tiling fits in
    with open(anno) as src, open(tss_anno, "w") as dst:
        lines = src.read().splitlines()
        dst.write("\n".join(lines[:5]) + "\n")
    return {"anno": anno, "vcf": vcf, "peaks": peaks, "tss_anno": tss_anno, "dir": d}


def main():
    import torch
    sys.path.insert(0, REPO)
    from oracle import weights as oweights
    work = tempfile.mkdtemp(prefix="expecto_golden_extra_")
    p = write_inputs(work)
    env = dict(os.environ, PYTHONPATH=STUBS + ":" + REF, OMP_NUM_THREADS="8")
    dst = os.path.join(GOLD, "extra")
    os.makedirs(dst, exist_ok=True)
    for tag, extra in (("", []), ("_rf", ["--all_in_receptive_field"])):
        subprocess.run([sys.executable, os.path.join(REF, "make_closest_genes_file.py"), p["vcf"], "--geneanno_file",
                        p["anno"], "-o", f"cg{tag}", *extra], cwd=work, env=env, capture_output=True, text=True,
                       check=True)
        shutil.copy(os.path.join(work, f"cg{tag}", "closest_genes.tsv"), os.path.join(dst, f"closest_genes{tag}.tsv"))
        shutil.copy(os.path.join(work, f"cg{tag}", "snps_hg19.vcf"), os.path.join(dst, f"snps_hg19{tag}.vcf"))
    torch.save(oweights.seeded_state_dict(0), os.path.join(work, "resources", "deepsea.beluga.pth"))
    shutil.copy(os.path.join(REF, "resources", "deepsea_beluga_2002_features.tsv"), os.path.join(work, "resources"))
    np.save(os.path.join(work, "resources", "Xreducedall.2002.npy"), np.zeros((1, 1)))   # loaded, unused
    for tag, extra in (("", []), ("_tf", ["--tf_only"])):
        subprocess.run([sys.executable, os.path.join(REF, "expecto_intersect_chip_atac.py"), p["tss_anno"],
                        p["peaks"], "-o", f"ix{tag}", *extra], cwd=work, env=env, capture_output=True, text=True,
                       check=True)
        shutil.copy(os.path.join(work, f"ix{tag}", "Xreducedall.2002.atac_x_chip.npy"),
                    os.path.join(dst, f"atac_x_chip{tag}.npy"))
    shutil.rmtree(work)
    print("extra goldens written to", dst)


if __name__ == "__main__":
    main()
