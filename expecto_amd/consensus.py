"""Personal-genome / eQTL 200-shift scoring on the GPU: drop-ins for the reference
``geuvadis_sed_for_top_eqtls.py``, ``geuvadis_predict_consensus.py``,
``geuvadis_predict_ref_all_genes.py``, ``geuvadis_predict_consensus_for_top_eqtls.py`` and
``merge_geuvadis_predict_consensus.py`` CLIs:

    python -m expecto_amd.consensus {sed|consensus|ref_all_genes|top_eqtls|merge} ...

They score consensus sequences -- 393,216-bp Enformer records whose TSS sits at index
``len(seq) // 2``, or (top_eqtls) Basenji records with the TSS at ``(len - 1) // 2`` on + and
``len // 2`` on - -- with 200 Beluga windows at ``tss + shift*strand`` for
``shift in range(-20000, 20000, 200)`` (``get_seq_shifts_for_sample_seq``), each on the window
and its reverse complement (``encodeSeqs``), fwd/rc averaged in float64, reduced with the
10 exp-decay position weights, written in the legacy 20030-feature layout (a zero column
ahead of every decay block) and scored with the ExPecto gblinear model.

Device path per batch of sequences: the 41,800-bp span of the 200 windows is one segment per
sequence (``forward_segments``: conv1..conv4 once per segment); for an eQTL SNV the alt
sequence goes through ``forward_segment_pairs`` (only the rows the SNV changes are
recomputed, windows not holding it copy their ref rows; bit-identical to full forwards);
``expecto_shift_reduce`` (float64 average, legacy layout) and ``expecto_gblinear_predict``
finish on the device.  Outputs and stdout follow the reference scripts.
"""
from __future__ import annotations

import argparse
import glob
import math
import os
import re
from pathlib import Path

import numpy as np
import pandas as pd
import torch

from . import _lib, h5
from .beluga import Beluga, seeded
from .encode import seq_codes
from .features import tss_pos_weights
from .xgblinear import GBLinear

ENFORMER_SEQ_LENGTH = 393216
SHIFTS = np.arange(-20000, 20000, 200)
WINDOW = 2000
REDUCE_F64AVG, REDUCE_LEGACY20030 = 1, 2


# ---- FASTA (Bio.SeqIO 'fasta' subset) -------------------------------------------------------
def parse_fasta(path: str):
    """(id, sequence) per record: id = first word of the header, sequence lines joined
    (``.gz`` paths are read through gzip, as the reference's ``gzip.open(..., 'rt')``)."""
    import gzip
    rid, parts = None, []
    with (gzip.open(path, "rt") if str(path).endswith(".gz") else open(path)) as f:
        for line in f:
            if line.startswith(">"):
                if rid is not None:
                    yield rid, "".join(parts)
                rid, parts = (line[1:].split() or [""])[0], []
            elif rid is not None:
                parts.append(line.strip())
    if rid is not None:
        yield rid, "".join(parts)


def normalize_consensus(rid: str, seq: str) -> str:
    """Upper-case and N-pad a record truncated at a chromosome end (geuvadis_*.py
    get_1_id_and_seq_from_fasta / gen_sample_seqs_and_id_for_gene)."""
    seq = seq.upper()
    interval = rid.split(":")[1]
    if interval.startswith("-"):
        bp_start = -int(interval.split("-")[-2])
        bp_end = int(interval.split("-")[-1])
        assert bp_end - bp_start + 1 == ENFORMER_SEQ_LENGTH
        seq = "N" * (ENFORMER_SEQ_LENGTH - len(seq)) + seq
    else:
        bp_start, bp_end = map(int, interval.split("-"))
        assert bp_end - bp_start + 1 == ENFORMER_SEQ_LENGTH
        if len(seq) < ENFORMER_SEQ_LENGTH:
            seq = seq + "N" * (ENFORMER_SEQ_LENGTH - len(seq))
    assert len(seq) == ENFORMER_SEQ_LENGTH, f"Sequence length is {len(seq)} for {rid}"
    return seq


def read_one_consensus(path: str):
    records = list(parse_fasta(path))
    assert len(records) == 1, f"Expected 1 record in fasta file {path}, but got {len(records)} records"
    rid, seq = records[0]
    return f"{rid}|{Path(path).stem}", normalize_consensus(rid, seq)


def natsorted(items):
    """natsort.natsorted's default key for plain names: digit runs compare as integers."""
    key = lambda s: [(0, int(t), "") if t.isdigit() else (1, 0, t) for t in re.split(r"(\d+)", s) if t != ""]
    return sorted(items, key=key)


# ---- device scoring -----------------------------------------------------------------------
class ConsensusScorer:
    """200-shift chromatin predictions, features and expression scores of consensus sequences."""

    def __init__(self, engine, shifts=SHIFTS):
        self.engine = engine
        self.dev = torch.device("cuda", engine.device)
        self.shifts = np.asarray(shifts, np.int64)
        self.lib = _lib.load()
        self.w_d = torch.from_numpy(tss_pos_weights(self.shifts)).to(self.dev)

    def _geometry(self, seq_len: int, strand: int, tss_i: int | None = None):
        """Segment start (index into the sequence) and per-window offsets inside it (TSS at
        tss_i, default len // 2)."""
        if tss_i is None:
            tss_i = seq_len // 2
        starts = tss_i + self.shifts * strand - (WINDOW // 2 - 1)      # get_seq_shifts_for_sample_seq
        lo = int(starts.min())
        L = int(starts.max()) - lo + WINDOW
        L += (-L) % 4
        if lo < 0 or lo + L > seq_len:
            raise AssertionError(f"Expected seq of length f{WINDOW} but got a window outside the sequence")
        return lo, L, (starts - lo).astype(np.int32)

    def _segments(self, seqs, strands, tss=None):
        geo = [self._geometry(len(s), st, None if tss is None else tss[i]) for i, (s, st) in enumerate(zip(seqs, strands))]
        L = max(g[1] for g in geo)
        codes = np.full((len(seqs), L), 4, np.uint8)
        for i, (s, (lo, Li, _)) in enumerate(zip(seqs, geo)):
            codes[i, :Li] = seq_codes(s[lo:lo + Li], Li)
        return geo, L, torch.from_numpy(codes).to(self.dev)

    def predict(self, seqs, strands, tss=None) -> torch.Tensor:
        """[2 (fwd, rc), n, S, 2002] fp32 window predictions (TSS indices `tss`, default len // 2)."""
        n, S = len(seqs), len(self.shifts)
        y = torch.empty((2, n, S, 2002), dtype=torch.float32, device=self.dev)
        if n == 0:
            return y
        geo, L, codes = self._segments(seqs, strands, tss)
        win_seg = np.repeat(np.arange(n, dtype=np.int32), S)
        win_off = np.concatenate([g[2] for g in geo])
        self.engine.forward_segments(codes, L, win_seg, win_off, None, _lib.STRAND_BOTH, out=y.view(2 * n * S, 2002))
        return y

    def predict_snv_pairs(self, seqs, strands, snp_i, alt_bases):
        """Ref and alt ([2, n, S, 2002] each) for SNVs: alt = seq with alt_bases[i] at snp_i[i]."""
        n, S = len(seqs), len(self.shifts)
        y_ref = torch.empty((2, n, S, 2002), dtype=torch.float32, device=self.dev)
        y_alt = torch.empty_like(y_ref)
        if n == 0:
            return y_ref, y_alt
        geo, L, codes = self._segments(seqs, strands)
        pos = np.array([p - g[0] for p, g in zip(snp_i, geo)], np.int64)
        inside = (pos >= 0) & (pos < L)
        alt_code = torch.from_numpy(np.array([seq_codes(b, 1)[0] for b in alt_bases], np.uint8))
        win_off = np.concatenate([g[2] for g in geo])
        win_seg = np.repeat(np.arange(n, dtype=np.int32), S)
        yr, ya = y_ref.view(2 * n * S, 2002), y_alt.view(2 * n * S, 2002)
        if inside.all():
            self.engine.forward_segment_pairs(codes, L, pos.astype(np.int32), alt_code.to(self.dev), win_seg, win_off,
                                              None, yr, ya, n * S, _lib.STRAND_BOTH)
            return y_ref, y_alt
        # an SNV outside every window leaves all alt windows equal to the ref ones
        self.engine.forward_segments(codes, L, win_seg, win_off, None, _lib.STRAND_BOTH, out=yr)
        ya.copy_(yr)
        idx = np.nonzero(inside)[0]
        if idx.size:
            sub = codes[torch.from_numpy(idx).to(self.dev)].contiguous()
            m = idx.size
            tr = torch.empty((2, m, S, 2002), dtype=torch.float32, device=self.dev)
            ta = torch.empty_like(tr)
            self.engine.forward_segment_pairs(sub, L, pos[idx].astype(np.int32), alt_code[idx].to(self.dev),
                                              np.repeat(np.arange(m, dtype=np.int32), S),
                                              np.concatenate([geo[i][2] for i in idx]), None,
                                              tr.view(2 * m * S, 2002), ta.view(2 * m * S, 2002), m * S,
                                              _lib.STRAND_BOTH)
            y_alt[:, torch.from_numpy(idx).to(self.dev)] = ta
        return y_ref, y_alt

    def features(self, y: torch.Tensor, legacy: bool = True) -> torch.Tensor:
        """[n, 20030] (legacy) or [n, 20020] float64 from [2, n, S, 2002] predictions."""
        _, n, S, F = y.shape
        out = torch.empty((n, 10 * (F + (1 if legacy else 0))), dtype=torch.float64, device=self.dev)
        if n:
            y = y.contiguous()
            _lib.check(self.lib.expecto_shift_reduce(_lib.dptr(y[0]), _lib.dptr(y[1]), _lib.dptr(self.w_d), n, S, F,
                                                     REDUCE_F64AVG | (REDUCE_LEGACY20030 if legacy else 0),
                                                     _lib.dptr(out), _lib.stream_ptr()), "shift_reduce")
        return out

    @staticmethod
    def fwd_rc_mean64(y: torch.Tensor) -> torch.Tensor:
        """[n, S, 2002] float64 (a + b) / 2 of the fp32 fwd / rc predictions (numpy float64)."""
        return (y[0].double() + y[1].double()) / 2


def _strand_sign(strand) -> int:
    if strand == '+':
        return 1
    if strand == '-':
        return -1
    raise AssertionError(f'strand {strand} not recognized')


def _load_beluga(args) -> Beluga:
    if args.synthetic_weights is not None:
        m = seeded(args.synthetic_weights, gain=math.sqrt(6.0), max_batch=args.max_batch)
    else:
        m = Beluga(max_batch=args.max_batch)
        m.load_state_dict(torch.load(args.beluga_model, map_location="cpu", weights_only=True))
    return m.eval().cuda()


def _extra_args(p):
    p.add_argument('--synthetic-weights', type=int, default=None, help=argparse.SUPPRESS)
    p.add_argument('--max-batch', type=int, default=4096, help="windows per device chunk")
    p.add_argument('--seq-batch', type=int, default=16, help="sequences per device batch")


# ---- geuvadis_sed_for_top_eqtls.py --------------------------------------------------------
def sed_main(argv=None, capture: dict | None = None):
    """geuvadis_sed_for_top_eqtls.py main() (:21-135).  ``capture`` (a dict, for tests) receives
    the per-batch window predictions ("y_ref"/"y_alt": [2 strands, n, 200, 2002] f32) and the
    features ("x_ref"/"x_alt": [n, 20030] f64) the scores were computed from."""
    p = argparse.ArgumentParser(description='Predict expression for consensus sequences using ExPecto')
    p.add_argument('expecto_model')
    p.add_argument('consensus_dir')
    p.add_argument('eur_top_eqtl_genes_csv')
    p.add_argument('eqtls_csv')
    p.add_argument('--beluga_model', type=str, default='./resources/deepsea.beluga.pth')
    p.add_argument('--batch_size', action="store", dest="batch_size", type=int, default=1024,
                   help="Batch size for neural network predictions.")
    p.add_argument('-o', dest="out_dir", type=str, default='temp_sed_for_top_eqtls', help='Output directory')
    _extra_args(p)
    args = p.parse_args(argv)
    os.makedirs(args.out_dir, exist_ok=True)
    model = _load_beluga(args)
    bst = GBLinear.load(args.expecto_model.strip())
    eqtls_df = pd.read_csv(args.eqtls_csv)
    all_eqtls_df = pd.read_csv(args.eur_top_eqtl_genes_csv, names=["ens_id", "chr", "pos", "gene", "strand"])
    all_eqtls_df["gene"] = all_eqtls_df["gene"].str.lower()
    all_eqtls_df["gene"] = all_eqtls_df["gene"].fillna(all_eqtls_df["ens_id"].str.lower())
    eqtls_df["strand"] = pd.merge(eqtls_df, all_eqtls_df, left_on="name", right_on="gene", how="left")["strand"]

    scorer = ConsensusScorer(model.engine())
    genes, ref_pred, alt_pred = [], [], []
    batch = []

    def flush():
        if not batch:
            return
        seqs = [b[0] for b in batch]
        strands = [b[1] for b in batch]
        snv = [len(b[3]) == 1 for b in batch]
        if all(snv):
            y_ref, y_alt = scorer.predict_snv_pairs(seqs, strands, [b[2] for b in batch], [b[3] for b in batch])
        else:   # insertions: the alt sequence (and its centre) differ -> own windows
            y_ref = scorer.predict(seqs, strands)
            alts = [s[:i] + a + s[i + 1:] for s, _, i, a in batch]
            y_alt = scorer.predict(alts, strands)
        for y, dst, tag in ((y_ref, ref_pred, "ref"), (y_alt, alt_pred, "alt")):
            x = scorer.features(y)
            dst.append(bst.predict(x).cpu().numpy())
            if capture is not None:
                capture.setdefault(f"y_{tag}", []).append(y.cpu().numpy())
                capture.setdefault(f"x_{tag}", []).append(x.cpu().numpy())
        batch.clear()

    for i in range(eqtls_df.shape[0]):
        eqtl = eqtls_df.iloc[i]
        genes.append(eqtl['name'])
        gene = eqtl['name'].lower()
        ref_id, ref_seq = read_one_consensus(f'{args.consensus_dir}/{gene}/ref.fa')
        ref_id = ref_id.split("|")[0]
        ref_chr = int(ref_id.split(':')[0].replace("chr", ""))
        ref_start, ref_end = map(int, ref_id.split(':')[1].split('-'))
        assert (ref_end - ref_start + 1) == len(ref_seq), "record ID does not match fasta seq length"
        assert eqtl["CHR_SNP"] == ref_chr, "Chromosomes do not match between eQTL df and ref fasta id"
        assert eqtl['TSSpos_x'] == (ref_start + (len(ref_seq) // 2)), \
            "TSSpos in eQTL file not consistent with fasta record"
        tss_i = len(ref_seq) // 2
        snp_i = int(tss_i - (eqtl['TSSpos_x'] - eqtl['SNPpos']))
        assert ref_seq[snp_i] == eqtl['REF'], "Ref sequence does not match ref allele"
        batch.append((ref_seq, _strand_sign(eqtl['strand']), snp_i, eqtl['ALT']))
        if len(batch) >= args.seq_batch:
            flush()
    flush()
    ref_all = np.concatenate(ref_pred) if ref_pred else np.zeros(0, np.float32)
    alt_all = np.concatenate(alt_pred) if alt_pred else np.zeros(0, np.float32)
    for i, gene in enumerate(genes):
        preds_dir = f'{args.out_dir}/{gene}'
        os.makedirs(preds_dir, exist_ok=True)
        h5.write(f'{preds_dir}/{gene}.h5', {'ref_preds': np.float32(ref_all[i]), 'alt_preds': np.float32(alt_all[i])})
    return genes, ref_all, alt_all


# ---- geuvadis_predict_consensus.py --------------------------------------------------------
def consensus_main(argv=None):
    p = argparse.ArgumentParser(description='Predict expression for consensus sequences using ExPecto')
    p.add_argument('expecto_model')
    p.add_argument('consensus_dir')
    p.add_argument('genes_file')
    p.add_argument('--beluga_model', type=str, default='./resources/deepsea.beluga.pth')
    p.add_argument('--batch_size', action="store", dest="batch_size", type=int, default=1024,
                   help="Batch size for neural network predictions.")
    p.add_argument('--overwrite', action="store_true", dest="overwrite", default=False)
    p.add_argument('--exp_only', action="store_true", dest="exp_only", default=False)
    p.add_argument("--num_chunks", action="store", dest="num_chunks", type=int, default=None)
    p.add_argument("--chunk_i", action="store", dest="chunk_i", type=int, default=None)
    p.add_argument('-o', dest="out_dir", type=str, default='temp_predict_consensus', help='Output directory')
    _extra_args(p)
    args = p.parse_args(argv)
    os.makedirs(args.out_dir, exist_ok=True)
    model = None if args.exp_only else _load_beluga(args)
    bst = GBLinear.load(args.expecto_model.strip())
    genes = natsorted([os.path.basename(f) for f in glob.glob(f'{args.consensus_dir}/*')])
    genes_df = pd.read_csv(args.genes_file, names=['ens_id', 'chrom', 'bp', 'gene_symbol', 'strand'], index_col=False)
    genes_df['gene_symbol'] = genes_df['gene_symbol'].fillna(genes_df['ens_id']).str.lower()
    genes_df = genes_df.set_index('gene_symbol')
    if args.num_chunks is not None:
        genes = np.array_split(genes, args.num_chunks)[args.chunk_i]
        assert len(genes) > 0, "Gene split resulted in empty list"
    scorer = ConsensusScorer(model.engine()) if model is not None else None
    dev = torch.device("cuda", torch.cuda.current_device())
    w_d = torch.from_numpy(tss_pos_weights(SHIFTS)).to(dev)
    print("Predicting chromatin for all samples for all genes...")
    for gene in genes:
        fasta_files = glob.glob(f'{args.consensus_dir}/{gene}/samples/*.fa')
        strand = genes_df.loc[gene, 'strand']
        preds_dir = f'{args.out_dir}/{gene}'
        os.makedirs(preds_dir, exist_ok=True)
        if not args.overwrite and os.path.exists(f'{preds_dir}/{gene}.h5'):
            print(f"Skipping gene {gene} since h5 is already present.")
            continue
        if args.exp_only:
            d = h5.read(f"{preds_dir}/{gene}_chromatin.h5")
            preds = torch.from_numpy(np.asarray(d['chromatin_preds'], np.float64)).to(dev)
            record_ids = [x.decode('utf-8') for x in d['record_ids']]
            feats = _legacy_features_f64(preds, w_d)
        else:
            record_ids, seqs = [], []
            for f in fasta_files:
                for rid, seq in parse_fasta(f):
                    seqs.append(normalize_consensus(rid, seq))
                    record_ids.append(f"{rid}|{Path(f).stem}")
            sign = _strand_sign(strand)
            ys = []
            for b0 in range(0, len(seqs), args.seq_batch):
                ys.append(scorer.predict(seqs[b0:b0 + args.seq_batch], [sign] * len(seqs[b0:b0 + args.seq_batch])))
            y = torch.cat(ys, 1) if ys else torch.empty((2, 0, len(SHIFTS), 2002), device=dev)
            preds = ConsensusScorer.fwd_rc_mean64(y)
            feats = scorer.features(y)
        expecto_preds = bst.predict(feats).cpu().numpy()
        ids = np.array(record_ids, 'S')
        h5.write(f'{preds_dir}/{gene}_chromatin.h5', {'chromatin_preds': preds.cpu().numpy(), 'record_ids': ids})
        h5.write(f'{preds_dir}/{gene}.h5', {'expecto_preds': expecto_preds, 'record_ids': ids})


# ---- geuvadis_predict_ref_all_genes.py ----------------------------------------------------
def ref_all_genes_main(argv=None, capture: dict | None = None):
    """geuvadis_predict_ref_all_genes.py main() (:23-101): the reference-genome consensus
    ``{consensus_dir}/{gene}/ref.fa`` of every gene in the genes table (gene symbol, else the
    Ensembl id), 200 shifts x fwd/rc on the segment path, float64 fwd/rc mean, legacy 20030
    features, gblinear score; writes ``ref_preds.csv`` (columns genes, ref_preds).  ``capture``
    (tests) receives the window predictions and features per batch."""
    p = argparse.ArgumentParser(description='Predict expression for consensus sequences using ExPecto')
    p.add_argument('expecto_model')
    p.add_argument('consensus_dir')
    p.add_argument('genes_file')
    p.add_argument('--beluga_model', type=str, default='./resources/deepsea.beluga.pth')
    p.add_argument('--batch_size', action="store", dest="batch_size", type=int, default=1024,
                   help="Batch size for neural network predictions.")
    p.add_argument('-o', dest="out_dir", type=str, default='temp_sed_for_top_eqtls', help='Output directory')
    _extra_args(p)
    args = p.parse_args(argv)
    os.makedirs(args.out_dir, exist_ok=True)
    model = _load_beluga(args)
    bst = GBLinear.load(args.expecto_model.strip())
    genes_df = pd.read_csv(args.genes_file, names=['ens_id', 'chrom', 'bp', 'gene_symbol', 'strand'], index_col=False)
    genes_df['gene_symbol'] = genes_df['gene_symbol'].fillna(genes_df['ens_id'])
    genes_df = genes_df.set_index('gene_symbol')
    scorer = ConsensusScorer(model.engine())
    preds, batch = [], []

    def flush():
        if not batch:
            return
        y = scorer.predict([b[0] for b in batch], [b[1] for b in batch])
        x = scorer.features(y)
        preds.extend(bst.predict(x).cpu().numpy()[:, None])     # one (1,) array per gene, as the reference
        if capture is not None:
            capture.setdefault("y", []).append(y.cpu().numpy())
            capture.setdefault("x", []).append(x.cpu().numpy())
        batch.clear()

    for gene in genes_df.index:
        strand = genes_df.loc[gene, 'strand']
        _, seq = read_one_consensus(f'{args.consensus_dir}/{gene.lower()}/ref.fa')
        batch.append((seq, _strand_sign(strand)))
        if len(batch) >= args.seq_batch:
            flush()
    flush()
    expecto_ref_preds = np.array(preds).squeeze()
    df = pd.DataFrame({"genes": np.array(genes_df.index.values), "ref_preds": expecto_ref_preds})
    df.to_csv(f'{args.out_dir}/ref_preds.csv', header=True, index=False)
    return df


# ---- geuvadis_predict_consensus_for_top_eqtls.py -------------------------------------------
TOP_EQTL_GENES = ['HLA-B', 'HLA-C', 'RPL28', 'CPAMD8', 'TMEM121B', 'SCN11A']   # the script's list (:72-73)


def top_eqtl_tss(seq_len: int, strand: str) -> int:
    """TSS index of a Basenji consensus record (get_seq_shifts_for_sample_seq, :160-168)."""
    return (seq_len - 1) // 2 if strand == '+' else seq_len // 2


def sample_seq_for_expecto(seq: str, strand: str, shifts=SHIFTS, windowsize: int = WINDOW) -> str:
    """get_sample_seq_for_expecto (:143-152): the 41,800-bp span the 200 windows cover."""
    sign = _strand_sign(strand)
    tss_i = top_eqtl_tss(len(seq), strand)
    c = tss_i + np.asarray(shifts) * sign
    out = seq[min(c - int(windowsize / 2 - 1)):max(c + int(windowsize / 2) + 1)]
    assert len(out) == 41800, "length of sequence should be 41800 to match ExPecto receptive field"
    return out


def top_eqtls_main(argv=None, capture: dict | None = None):
    """geuvadis_predict_consensus_for_top_eqtls.py main() (:23-128): for each gene of the
    script's list, every record of ``{consensus_dir}/{gene}/{gene}.fa.gz`` (upper-cased; the
    strand is the id's second-to-last '|' field) through 200 shifts x fwd/rc, float64 mean,
    legacy 20030 features, gblinear score -> ``{out}/{gene}/{gene}.h5`` with ``preds``,
    ``record_ids`` and the 41,800-bp ``seqs``.  The eQTL table and VCF are read and joined as
    the script does (the join is validated m:1, its result otherwise unused).
    Deviation: the script builds the legacy feature layout with np.zeros((1, 10, 1)), which
    only concatenates for files of ONE record (numpy raises for more); here every record gets
    its zero column (geuvadis_predict_consensus.py's corrected form, same values for one record).
    ``--genes`` (extra) replaces the fixed list."""
    p = argparse.ArgumentParser(description='Predict expression for consensus sequences using ExPecto')
    p.add_argument('expecto_model')
    p.add_argument('consensus_dir')
    p.add_argument('eqtls_df_file')
    p.add_argument('snps_vcf')
    p.add_argument('--beluga_model', type=str, default='./resources/deepsea.beluga.pth')
    p.add_argument('--batch_size', action="store", dest="batch_size", type=int, default=1024,
                   help="Batch size for neural network predictions.")
    p.add_argument('-o', dest="out_dir", type=str, default='temp_predict_consensus', help='Output directory')
    p.add_argument('--genes', type=str, default=None, help="comma-separated genes (default: the script's six)")
    _extra_args(p)
    args = p.parse_args(argv)
    os.makedirs(args.out_dir, exist_ok=True)
    model = _load_beluga(args)
    bst = GBLinear.load(args.expecto_model.strip())
    eur = pd.read_csv(args.eqtls_df_file)
    eur['gene_symbol'] = eur['name'].fillna(eur['geneID'])
    eur['SNPpos'] = eur['SNPpos'].astype(int).astype(str)
    eur = eur.set_index('chr' + eur['CHR_SNP'].astype(str) + '_' + eur['SNPpos'])
    vcf_df = pd.read_csv(args.snps_vcf, sep='\t', comment='#', header=None).iloc[:, 0:5]
    vcf_df.columns = ['SNP_CHROM', 'SNP_POS', 'ID', 'REF', 'ALT']
    vcf_df.index = vcf_df.iloc[:, 0] + '_' + vcf_df.iloc[:, 1].astype(str)
    vcf_df = vcf_df.drop_duplicates()
    eur.merge(vcf_df, left_index=True, right_index=True, validate='m:1', how='inner')
    genes = args.genes.split(",") if args.genes else TOP_EQTL_GENES
    scorer = ConsensusScorer(model.engine())
    print("Predicting chromatin for all samples for all genes...")
    for gene in genes:
        gene = gene.lower()
        preds_dir = f'{args.out_dir}/{gene}'
        os.makedirs(preds_dir, exist_ok=True)
        ids, seqs, strands = [], [], []
        for rid, seq in parse_fasta(f'{args.consensus_dir}/{gene}/{gene}.fa.gz'):
            ids.append(rid)
            seqs.append(seq.upper())
            strands.append(rid.split('|')[-2])
        sample_seqs = [sample_seq_for_expecto(s, st) for s, st in zip(seqs, strands)]
        feats = []
        for b0 in range(0, len(seqs), args.seq_batch):
            sl = slice(b0, b0 + args.seq_batch)
            y = scorer.predict(seqs[sl], [_strand_sign(st) for st in strands[sl]],
                               [top_eqtl_tss(len(s), st) for s, st in zip(seqs[sl], strands[sl])])
            feats.append(scorer.features(y))
            if capture is not None:
                capture.setdefault("y", []).append(y.cpu().numpy())
        x = torch.cat(feats) if feats else torch.empty((0, 20030), dtype=torch.float64, device=scorer.dev)
        if capture is not None:
            capture.setdefault("x", []).append(x.cpu().numpy())
        expecto_preds = bst.predict(x).cpu().numpy()
        h5.write(f'{preds_dir}/{gene}.h5', {'preds': expecto_preds, 'record_ids': np.array(ids, 'S'),
                                             'seqs': np.array(sample_seqs, 'S')})


# ---- merge_geuvadis_predict_consensus.py ---------------------------------------------------
def parse_record_id(x: bytes) -> str:
    """b'chr19:58832097-58897632|NA20828|-|1pIu' -> 'NA20828|1pIu' (:48-55)."""
    x = x.decode("utf-8").split("|")
    return f"{x[1]}|{x[3]}"


def merge_main(argv=None):
    """merge_geuvadis_predict_consensus.py main() (:12-45): stack the per-gene ``preds`` of
    ``{batch_dir}/*/*.h5`` (natsorted; every file must carry the same samples) into
    ``{out}/expecto_preds.h5`` with ``record_ids``, ``genes`` (file stems) and ``preds``.
    Host only: no device work."""
    p = argparse.ArgumentParser(description='Merge output batches of geuvadis_predict_consensus.py')
    p.add_argument("--batch_dir", dest="batch_dir", type=str)
    p.add_argument("--n_genes", dest="n_genes", type=int, default=3259, help="Expected number of genes")
    p.add_argument('-o', dest="out_dir", type=str, default='merge_geuvadis_predict_consensus', help='Output directory')
    args = p.parse_args(argv)
    os.makedirs(args.out_dir, exist_ok=True)
    h5_files = natsorted(glob.glob(f"{args.batch_dir}/*/*.h5"))
    assert len(h5_files) == args.n_genes, f"Expected {args.n_genes} genes but got {len(h5_files)} h5 files"
    record_ids, preds = None, []
    for f in h5_files:
        d = h5.read(f)
        cur = np.array([parse_record_id(x) for x in d["record_ids"]])
        if record_ids is None:
            record_ids = cur
        else:
            assert (record_ids == cur).all()
        preds.append(np.array(d["preds"]))
    preds = np.stack(preds)
    genes = [Path(x).stem for x in h5_files]
    h5.write(f"{args.out_dir}/expecto_preds.h5", {"record_ids": np.array(record_ids, 'S'),
                                                  "genes": np.array(genes, 'S'), "preds": preds})


def _legacy_features_f64(preds: torch.Tensor, w_d: torch.Tensor) -> torch.Tensor:
    """--exp_only: features from stored float64 averaged predictions [n, S, F] (shifts summed in order)."""
    n, S, F = preds.shape
    out = torch.zeros((n, 10, F + 1), dtype=torch.float64, device=preds.device)
    acc = torch.zeros((n, 10, F), dtype=torch.float64, device=preds.device)
    for s in range(S):
        acc += w_d[None, :, s, None] * preds[:, None, s, :]
    out[:, :, 1:] = acc
    return out.reshape(n, -1)


COMMANDS = {"sed": sed_main, "consensus": consensus_main, "ref_all_genes": ref_all_genes_main,
            "top_eqtls": top_eqtls_main, "merge": merge_main}

if __name__ == "__main__":
    import sys
    if len(sys.argv) > 1 and sys.argv[1] in COMMANDS:
        COMMANDS[sys.argv[1]](sys.argv[2:])
    else:
        raise SystemExit(f"usage: python -m expecto_amd.consensus {{{'|'.join(COMMANDS)}}} ...")
