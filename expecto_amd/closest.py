"""Drop-in for the reference ``make_closest_genes_file.py``: the gene
association file predict.py consumes.

    python -m expecto_amd.closest snps_hg19.vcf [--all_in_receptive_field] [--add_chr_prefix]
        [--geneanno_file ./resources/geneanno.csv] [-o out_dir]

For every SNV: the gene whose representative (CAGE) TSS on the same chromosome is closest
(``find_closest_gene``: first minimum of |TSS - pos| in annotation order), or with
``--all_in_receptive_field`` every gene whose 200-shift TSS tiling covers the SNV
(``get_genes_in_receptive_field`` / ``is_in_receptive_field``; the closest gene when none).
Writes ``closest_genes.tsv`` (snp chrom without 'chr', pos-1, pos, ref, alt, tss chrom, tss-1,
tss, strand, ens id, tss - pos) and ``snps_hg19.vcf`` (VCF rows repeated per association), the
reference's outputs (``make_closest_genes_file.py:31-64``).  Host-side table work: per
chromosome the TSS arrays are built once (the reference filters the annotation per SNV).
"""
from __future__ import annotations

import argparse
import os

import numpy as np
import pandas as pd

SHIFTS = np.arange(-20000, 20000, 200)
WINDOW_HALF = 1000                        # make_closest_genes_file.py:88 (windowsize = 1000)


def receptive_bounds(strand_plus: np.ndarray):
    """(start, stop) of is_in_receptive_field per gene strand (make_closest_genes_file.py:101-106)."""
    s = np.where(strand_plus, 1, -1)[:, None]
    start = (SHIFTS[None, :] * s - int(WINDOW_HALF / 2 - 1)).min(1)
    stop = (SHIFTS[None, :] * s + int(WINDOW_HALF / 2)).max(1)
    return start, stop


def associate(vcf: pd.DataFrame, geneanno: pd.DataFrame, all_in_rf: bool):
    """[(vcf row index, gene iloc)] in output order."""
    by_chrom = {}
    for chrom, sub in geneanno.groupby('seqnames', sort=False):
        idx = np.nonzero((geneanno['seqnames'] == chrom).to_numpy())[0]   # annotation order
        tss = geneanno['CAGE_representative_TSS'].to_numpy()[idx].astype(np.int64)
        start, stop = receptive_bounds((geneanno['strand'].to_numpy()[idx] == '+'))
        by_chrom[chrom] = (idx, tss, start, stop)
    out = []
    for i in range(vcf.shape[0]):
        chrom, pos = vcf.iat[i, 0], int(vcf.iat[i, 1])
        if chrom not in by_chrom:
            raise ValueError(f"attempt to get argmin of an empty sequence (no gene on {chrom})")
        idx, tss, start, stop = by_chrom[chrom]
        dists = tss - pos
        if all_in_rf:
            inside = np.nonzero((start <= -dists) & (-dists <= stop))[0]
            if inside.size:
                out.extend((i, int(idx[j])) for j in inside)
                continue
        out.append((i, int(idx[int(np.argmin(np.abs(dists)))])))
    return out


def main(argv=None):
    p = argparse.ArgumentParser(description='Make closest gene file required by predict.py')
    p.add_argument('hg19_snps_file')
    p.add_argument('--all_in_receptive_field', action='store_true')
    p.add_argument('--add_chr_prefix', action='store_true')
    p.add_argument('--geneanno_file', dest='geneanno_file', type=str, default='./resources/geneanno.csv')
    p.add_argument('-o', dest="out_dir", type=str, default='temp_closest_gene_file', help='Output directory')
    args = p.parse_args(argv)
    os.makedirs(args.out_dir, exist_ok=True)
    vcf = pd.read_csv(args.hg19_snps_file, sep='\t', header=None, comment='#')
    if args.add_chr_prefix:
        vcf[0] = 'chr' + vcf[0].astype(str)
    geneanno = pd.read_csv(args.geneanno_file, index_col=0)
    pairs = associate(vcf, geneanno, args.all_in_receptive_field)
    vcf_out_path = f'{args.out_dir}/snps_hg19.vcf'
    with open(vcf_out_path, 'w') as f:
        print('##fileformat=VCFv4.3', file=f)
        print('#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO', file=f)
    rows, vrows = [], []
    ens = geneanno.index.to_numpy()
    for i, j in pairs:
        snp_chrom, snp_pos, ref, alt = vcf.iat[i, 0], int(vcf.iat[i, 1]), vcf.iat[i, 3], vcf.iat[i, 4]
        g = geneanno.iloc[j]
        tss_pos = int(g['CAGE_representative_TSS'])
        rows.append([snp_chrom[3:], snp_pos - 1, snp_pos, ref, alt, g['seqnames'][3:], tss_pos - 1, tss_pos,
                     g['strand'], ens[j], tss_pos - snp_pos])
        vrows.append(list(vcf.iloc[i]))
    cols = ('snp_chrom', 'snp_pos_start', 'snp_pos', 'ref', 'alt', 'tss_chrom', 'tss_pos_start', 'tss_pos',
            'tss_strand', 'ens_id', 'dist_to_tss')
    pd.DataFrame(rows, columns=cols, dtype=object).to_csv(f'{args.out_dir}/closest_genes.tsv', sep='\t', index=False,
                                                          header=False)
    pd.DataFrame(vrows, columns=np.arange(vcf.shape[1]), dtype=object).to_csv(vcf_out_path, sep='\t', header=False,
                                                                               index=False, mode='a')
    return rows


if __name__ == "__main__":
    main()
