"""Drop-in for the reference ``predict.py`` CLI: ``.diff.h5`` chromatin effects -> expression
effects (SED) with an ExPecto gblinear model.

    python -m expecto_amd.predict --model_save_file M.save --belugaFeatures features.tsv \\
        --coorFile_chromatin snps_hg19.vcf --geneFile closestgene.tsv \\
        --snpEffectFilePattern out/snps.shift_SHIFT.diff.h5 [--maxshift 800] -o out_dir

Same arguments (``predict.py:15-56``), stdout lines, and outputs ``sed.tsv``,
``sed_sorted_by_magnitude.tsv`` and ``sed_sorted_by_proportion.tsv`` (``predict.py:253-280``).
The reference's numpy pipeline is replaced by device work on the whole variant set at once:

* fwd/rc averaging of every shift's ``diff``/``ref``/``alt`` (``predict.py:186-194``):
  ``expecto_fwd_rc_average``;
* duplicate masking and the gene-association repeats (``predict.py:197-235``): host tables,
  then one device gather;
* the spatial feature reduction (``predict.py:87-136``): ``expecto_variant_reduce`` into
  float64 ``[n, 10*2002]``;
* the keep-mask column selection and the gblinear scoring (``predict.py:137-160``):
  ``expecto_gblinear_predict`` reads the float64 rows through a column map (no copy).

The model file is read by :mod:`expecto_amd.xgblinear` (xgboost is not needed).
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import pandas as pd
import torch

from . import h5
from .features import fwd_rc_average, variant_features
from .pipeline import shift_order
from .xgblinear import GBLinear

LAMBERT_HGNC_PATH = './resources/Lambert-hgnc-symbol-check.csv'     # cluster_utils.py:5-6
HGNC_MAPPING_PATH = './resources/beluga_hgnc_mapping.csv'
NFEAT = 2002


def build_parser():
    p = argparse.ArgumentParser(description='Process some integers.')
    p.add_argument('--model_save_file', action="store", dest="model_save_file",
                   help="Save file containing model to use for predictions")
    p.add_argument('--belugaFeatures', action="store", dest="belugaFeatures", help="tsv file denoting Beluga features")
    p.add_argument('--coorFile_chromatin', action="store", dest="coorFile_chromatin")
    p.add_argument('--geneFile', action="store", dest="geneFile")
    p.add_argument('--snpEffectFilePattern', action="store", dest="snpEffectFilePattern",
                   help="SNP effect hdf5 filename pattern. Use SHIFT as placeholder for shifts.")
    p.add_argument('--rsat_clusters_tab', action="store", dest="rsat_clusters_tab", help="clusters_motif_names.tab")
    p.add_argument('--nfeatures', action="store", dest="nfeatures", type=int, default=2002)
    p.add_argument('--fixeddist', action="store", dest="fixeddist", default=0, type=int)
    p.add_argument('--maxshift', action="store", dest="maxshift", type=int, default=800)
    p.add_argument('--batchSize', action="store", dest="batchSize", type=int, default=500)
    p.add_argument('--splitIndex', action="store", dest="splitIndex", type=int, default=0)
    p.add_argument('--splitFold', action="store", dest="splitFold", type=int, default=10)
    p.add_argument('--threads', action="store", dest="threads", type=int, default=16, help="Number of threads.")
    p.add_argument('--no_tf_features', action='store_true', dest='no_tf_features', default=False)
    p.add_argument('--no_dnase_features', action='store_true', dest='no_dnase_features', default=False)
    p.add_argument('--no_histone_features', action='store_true', dest='no_histone_features', default=False)
    p.add_argument('--intersect_with_lambert', action='store_true', dest='intersect_with_lambert', default=False)
    p.add_argument('--no_pol2', action='store_true', dest='no_pol2', default=False)
    p.add_argument('-o', action="store", dest="out_dir")
    # not in the reference: a text-dump model has no base_score (train.py writes it in the name)
    p.add_argument('--base_score', type=float, default=None, help=argparse.SUPPRESS)
    return p


def get_keep_mask(beluga_features_df, no_tf_features, no_dnase_features, no_histone_features,
                  intersect_with_lambert, no_pol2):
    """cluster_utils.py:8-50 (same filters, same messages)."""
    keep_mask = np.ones(beluga_features_df.shape[0], dtype=bool)
    if no_tf_features:
        print("not including TF features")
        keep_mask = keep_mask & (beluga_features_df['Assay type'] != 'TF')
    if no_dnase_features:
        print("not including DNase features")
        keep_mask = keep_mask & (beluga_features_df['Assay type'] != 'DNase')
    if no_histone_features:
        print("not including histone features")
        keep_mask = keep_mask & (beluga_features_df['Assay type'] != 'Histone')
    if intersect_with_lambert:
        print("intersecting with Lambert data")
        lambert_df = pd.read_csv(LAMBERT_HGNC_PATH, index_col=0)
        mapping = pd.read_csv(HGNC_MAPPING_PATH, index_col=0).dropna(subset=["Approved symbol"])
        assays = list(beluga_features_df['Assay'].values)
        for i, assay in enumerate(assays):
            if assay in mapping.index:
                match = mapping.loc[assay][["Match type", "Approved symbol"]]
                if len(match.shape) != 1:
                    match = match[match["Match type"] == "Approved symbol"].iloc[0]
                assays[i] = match["Approved symbol"].upper()
        hgnc = pd.Series(assays, index=beluga_features_df.index)
        keep_mask = keep_mask & hgnc.isin(lambert_df['Approved symbol'].values).values
        keep_mask = keep_mask & ~hgnc.isnull().values
    if no_pol2:
        print("taking out Pol2*")
        keep_mask = keep_mask & ~(beluga_features_df['Assay'].str.startswith('Pol'))
    keep_mask = np.asarray(keep_mask, dtype=bool)
    print(f"Number of features included in model: {np.sum(keep_mask)}")
    return keep_mask


def get_num_repeats(genes_df: pd.DataFrame) -> list:
    """predict.py:204-216: lengths of the runs of consecutive gene rows with the same
    ``chrom:start:end:ref:alt`` key (one run per chromatin row)."""
    keys = genes_df.iloc[:, 0:5].astype(str).agg(':'.join, axis=1).to_numpy()
    if len(keys) == 0:
        return [0]
    starts = np.r_[0, np.nonzero(keys[1:] != keys[:-1])[0] + 1]
    return list(np.diff(np.r_[starts, len(keys)]))


def load_effects(pattern: str, shifts, dev) -> dict:
    """Per shift, the fwd/rc-averaged diff/ref/alt [N, F] fp32 on the device (predict.py:173-194)."""
    out = {"diff": [], "ref": [], "alt": []}
    for s in shifts:
        d = h5.read(pattern.replace('SHIFT', str(s)))
        for k in out:
            x = torch.from_numpy(np.ascontiguousarray(d[k], dtype=np.float32)).to(dev)
            out[k].append(fwd_rc_average(x))
    return {k: torch.stack(v, 0) for k, v in out.items()}      # [S, N, F]


def run(args) -> pd.DataFrame:
    os.makedirs(args.out_dir, exist_ok=True)
    dev = torch.device("cuda", torch.cuda.current_device())
    beluga_features_df = pd.read_csv(args.belugaFeatures, sep='\t', index_col=0)
    beluga_features_df['Assay type + assay + cell type'] = (beluga_features_df['Assay type'] + '/' +
                                                           beluga_features_df['Assay'] + '/' +
                                                           beluga_features_df['Cell type'])
    mask_args = (args.no_tf_features, args.no_dnase_features, args.no_histone_features,
                 args.intersect_with_lambert, args.no_pol2)
    keep_mask = get_keep_mask(beluga_features_df, *mask_args)          # predict.py:61-62
    model = GBLinear.load(args.model_save_file.strip(), base_score=args.base_score)
    maxshift = int(args.maxshift)
    shifts = shift_order(maxshift)
    eff = load_effects(args.snpEffectFilePattern, shifts, dev)

    coor = pd.read_csv(args.coorFile_chromatin, sep='\t', header=None, comment='#')
    gene = pd.read_csv(args.geneFile, sep='\t', header=None, comment='#')
    gene = gene.drop_duplicates(keep="first")
    coor_mask = ~coor.duplicated(keep="first")
    coor = coor[coor_mask]
    repeats = get_num_repeats(gene)
    if len(repeats) != coor.shape[0] and not (coor.shape[0] == 0 and repeats == [0]):
        raise ValueError(f"repeat counts ({len(repeats)}) do not match the chromatin rows ({coor.shape[0]})")
    coor_new = pd.DataFrame(np.repeat(coor.values, repeats, axis=0))
    coor_new.columns = coor.columns
    coor = coor_new
    # chromatin rows kept by coor_mask, each repeated per associated gene (one device gather)
    rows = np.repeat(np.nonzero(coor_mask.to_numpy())[0], repeats)
    ridx = torch.from_numpy(rows.astype(np.int64)).to(dev)
    n = len(rows)
    geneinds = np.arange(coor.shape[0])
    if args.fixeddist == 0:
        dist = -np.asarray(gene.iloc[geneinds, -1])
    else:
        dist = np.full(n, args.fixeddist, dtype=np.int64) if n else np.zeros(0, np.int64)
    genename = np.asarray(gene.iloc[geneinds, -2])
    strand = np.asarray(gene.iloc[geneinds, -3])

    keep_idx = np.nonzero(keep_mask)[0].astype(np.int32)
    n_keep = len(keep_idx)
    if model.num_feature != 10 * n_keep:
        raise ValueError(f"model has {model.num_feature} features, the keep mask gives 10 x {n_keep}")
    cols = torch.from_numpy((np.arange(10, dtype=np.int32)[:, None] * args.nfeatures + keep_idx[None, :])
                            .reshape(-1).astype(np.int32)).to(dev)
    strand_plus = strand == '+'
    ref = np.zeros(n)
    alt = np.zeros(n)
    bs = int(args.batchSize)
    get_keep_mask(beluga_features_df, *mask_args)                      # predict.py:118 (messages)
    for i in range(int((n - 1) / bs) + 1):                             # predict.py:122-160
        print("Processing " + str(i) + "th batch of " + str(bs))
        get_keep_mask(beluga_features_df, *mask_args)                  # predict.py:138 (messages)
        lo, hi = i * bs, min(n, (i + 1) * bs)
        if hi <= lo:
            continue
        sel = ridx[lo:hi]
        preds = {}
        for k in ("ref", "alt"):
            x = variant_features(eff[k][:, sel], dist[lo:hi], strand_plus[lo:hi], shifts)
            preds[k] = model.predict(x, cols).cpu().numpy()
        ref[lo:hi] = preds["ref"]
        alt[lo:hi] = preds["alt"]

    df = coor
    df['dist'] = dist
    df['gene'] = genename
    df['strand'] = strand
    df = pd.concat([df.reset_index(), pd.DataFrame(ref, columns=['REF']), pd.DataFrame(alt, columns=['ALT']),
                    pd.DataFrame(alt - ref, columns=['SED'])], axis=1, ignore_index=False)
    df.to_csv(f'{args.out_dir}/sed.tsv', header=True, sep='\t', index=False)
    by_mag = df.copy()
    by_mag['SED_MAGNITUDES'] = np.abs(by_mag['SED'])
    by_mag = by_mag.sort_values(by='SED_MAGNITUDES', axis=0, ascending=False)
    by_mag.to_csv(f'{args.out_dir}/sed_sorted_by_magnitude.tsv', header=True, sep='\t', index=False)
    by_prop = df.copy()
    by_prop['SED_PROPORTION'] = np.abs(by_prop['SED'] / ((by_prop['REF'] + by_prop['ALT']) / 2))
    by_prop = by_prop.sort_values(by='SED_PROPORTION', axis=0, ascending=False)
    by_prop.to_csv(f'{args.out_dir}/sed_sorted_by_proportion.tsv', header=True, sep='\t', index=False)
    return df


def main(argv=None):
    args = build_parser().parse_args(argv)
    if not torch.cuda.is_available():
        raise RuntimeError("expecto_amd.predict needs a GPU (HIP); there is no CPU path")
    return run(args)


if __name__ == "__main__":
    main(sys.argv[1:])
