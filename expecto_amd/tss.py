"""TSS-tiling feature precompute on the device: drop-ins for the reference
``compute_expecto_features.py`` and ``replicate_expecto_features.py`` CLIs.

Per gene: 200 windows at ``tss + s*strand`` for ``s in range(-20000, 20000, 200)``
(``compute_expecto_features.py:88,107-111``), the Beluga forward on each window and on
its reverse complement (``:115-122``), ``pred = 0.5*(fwd+rc)`` (``:123``), and either the
10x200 exp-decay reduction to 20020 float64 features (``:124-128``) or the raw
``(200,2002)`` float32 ``pred`` per gene (``replicate_expecto_features.py:86``).

All of it runs on the GPU for batches of genes: ``expecto_tss_windows`` cuts the windows
from the HBM-resident genome, one ``forward_codes(BOTH)`` covers fwd and rc, and
``expecto_tss_reduce`` / ``expecto_fwd_rc_average`` finish it.
"""
from __future__ import annotations

import argparse
import math
import os
import sys

import numpy as np
import pandas as pd
import torch

from . import _lib
from . import dist as edist
from .beluga import Beluga, seeded
from .features import TSS_SHIFTS, fwd_rc_average, tss_pos_weights, tss_reduce
from .genome import DeviceGenome, Fasta
from .pipeline import gather_segments


class TSSPipeline:
    def __init__(self, engine, dgenome, shifts=TSS_SHIFTS):
        self.engine = engine
        self.dg = dgenome
        self.dev = dgenome.codes.device
        self.shifts = list(shifts)
        self.lib = _lib.load()
        self.sh_d = torch.tensor(self.shifts, dtype=torch.int32, device=self.dev)
        self.w_d = torch.from_numpy(tss_pos_weights(self.shifts)).to(self.dev)

    def _check(self, chroms, off, strands):
        rel = np.asarray(self.shifts, np.int64)[None, :] * np.asarray(strands, np.int64).reshape(-1, 1)
        self.dg.check_spans(list(chroms), off + rel.min(1) - 999, off + rel.max(1) + 1000)

    def window_codes(self, chroms, tss, strands) -> torch.Tensor:
        G, S = len(chroms), len(self.shifts)
        off = np.array([self.dg.offset(c, int(t)) for c, t in zip(chroms, tss)], np.int64)
        self._check(chroms, off, strands)
        codes = torch.empty((G, S, 2000), dtype=torch.uint8, device=self.dev)
        if G:
            # keep the argument tensors referenced until the launch is queued (a temporary's
            # block would go back to the caching allocator and be reused by the next one)
            off_d = torch.from_numpy(off).to(self.dev)
            strand_d = torch.tensor(np.asarray(strands, np.int8), device=self.dev)
            _lib.check(self.lib.expecto_tss_windows(
                _lib.dptr(self.dg.codes), self.dg.codes.numel(), _lib.dptr(off_d), _lib.dptr(strand_d), G,
                _lib.dptr(self.sh_d), S, _lib.dptr(codes), _lib.stream_ptr()), "tss_windows")
        return codes

    def predict(self, chroms, tss, strands, use_segments: bool = True) -> torch.Tensor:
        """[2 (fwd, rc), G, S, 2002] fp32.

        Segment path: one sequence per gene covering all 200 windows (41.8 kb), trunk computed
        once (bit-identical to the per-window path, which is kept for use_segments=False)."""
        G, S = len(chroms), len(self.shifts)
        y = torch.empty((2, G, S, 2002), dtype=torch.float32, device=self.dev)
        if G == 0:
            return y
        sh = np.asarray(self.shifts)
        if use_segments and all((x - sh.min()) % 4 == 0 for x in sh):
            strands = np.asarray(strands, np.int64)
            off = np.array([self.dg.offset(c, int(t)) for c, t in zip(chroms, tss)], np.int64)
            self._check(chroms, off, strands)
            rel = sh[None, :] * strands[:, None]                  # window start - (tss_off - 999)
            lo = rel.min(1)
            L = 2000 + int((rel.max(1) - lo).max())
            L += (-L) % 4
            start = torch.from_numpy(off + lo - 999).to(self.dev)
            codes = gather_segments(self.lib, self.dg, start, L)
            win_seg = np.repeat(np.arange(G), S).astype(np.int32)
            win_off = (rel - lo[:, None]).ravel().astype(np.int32)
            self.engine.forward_segments(codes, L, win_seg, win_off, None, _lib.STRAND_BOTH,
                                         out=y.view(2 * G * S, 2002))
            return y
        codes = self.window_codes(chroms, tss, strands)
        self.engine.forward_codes(codes.view(G * S, 2000), _lib.STRAND_BOTH, out=y.view(2 * G * S, 2002))
        return y

    def features(self, chroms, tss, strands) -> torch.Tensor:
        """[G, 20020] float64 (compute_expecto_features.py:123-124)."""
        y = self.predict(chroms, tss, strands)
        return tss_reduce(y[0], y[1], self.w_d)

    def pred_fwd_rc(self, chroms, tss, strands) -> torch.Tensor:
        """[G, S, 2002] float32 0.5*(fwd+rc) (replicate_expecto_features.py:83)."""
        y = self.predict(chroms, tss, strands)
        G, S = y.shape[1], y.shape[2]
        return fwd_rc_average(y.view(2 * G * S, 2002)).view(G, S, 2002)


def _load_model(args) -> Beluga:
    if getattr(args, "synthetic_weights", None) is not None:
        m = seeded(args.synthetic_weights, gain=math.sqrt(6.0), max_batch=args.max_batch)
    else:
        m = Beluga(max_batch=args.max_batch)
        m.load_state_dict(torch.load(args.weights, map_location="cpu", weights_only=True))
        m.eval()
    return m.cuda()


def _common_args(p, gene_batch: int = 16, max_batch: int = 2048):
    p.add_argument('--windowsize', action="store", dest="windowsize", type=int, default=2000)
    p.add_argument('--cuda', action='store_true')
    p.add_argument('--genome', default='./resources/hg19.fa')
    p.add_argument('--weights', default='./resources/deepsea.beluga.pth')
    p.add_argument('--synthetic-weights', type=int, default=None, dest='synthetic_weights')
    p.add_argument('--max-batch', type=int, default=max_batch, dest='max_batch',
                   help="windows per device chunk / FC slice (handle workspace: ~5 MB per window)")
    p.add_argument('--gene-batch', type=int, default=gene_batch, dest='gene_batch')


def _anno_genes(path):
    """(gene_id, chrom, CAGE_TSS, strand) per annotation row (replicate_expecto_features.py:40-43)."""
    out = []
    for i, line in enumerate(open(path)):
        if i == 0:
            continue
        gene_id, _, chrom, strand, _, tss, _ = line.rstrip().split(",")
        out.append((gene_id, chrom, int(tss), 1 if strand == "+" else -1))
    return out


def _batches(items, size):
    for i in range(0, len(items), size):
        yield items[i:i + size]


def compute_main(argv=None):
    """compute_expecto_features.py main() (:17-128).  Under torch.distributed.run the genes are
    sharded by contiguous rank ranges and rank 0 gathers the features and writes the .npy."""
    p = argparse.ArgumentParser(description='Compute ExPecto chromatin features for TSS list')
    p.add_argument('annoFile')
    p.add_argument('tss_file')
    p.add_argument('-o', dest="out_dir", type=str, default='temp_compute_expecto_features')
    p.add_argument('--no-liftover', action='store_true', dest='no_liftover',
                   help='treat every hg38 TSS as unmapped (the reference needs the liftover package)')
    p.add_argument('--chain-file', default=None, dest='chain_file',
                   help='UCSC hg38ToHg19 chain file for the TSS liftover (default: $EXPECTO_CHAIN_FILE, '
                        'else the liftover package)')
    _common_args(p)
    args = p.parse_args(argv)
    if args.windowsize != 2000:
        raise ValueError("--windowsize must be 2000 (Beluga.py:43)")
    rank, world, local = edist.init()
    if world > 1:
        torch.cuda.set_device(edist.local_device(local))
    os.makedirs(args.out_dir, exist_ok=True)
    fasta = Fasta(args.genome)
    model = _load_model(args)
    tss_df = pd.read_csv(args.tss_file, sep='\t', index_col=0).set_index('ens_id')
    if args.no_liftover:
        converter = None
    else:
        from .liftover import get_lifter
        try:
            converter = get_lifter('hg38', 'hg19', args.chain_file)
        except RuntimeError as e:
            raise RuntimeError(f"{e}; or pass --no-liftover to keep the annotated TSSs") from e
    genes = []
    found = no_map = 0
    for i, line in enumerate(open(args.annoFile)):
        if i == 0:
            continue
        gene_id, _, chrom, strand, _, tss, _ = line.rstrip().split(",")
        if gene_id in tss_df.index:
            found += 1
            chrom38, tss38, strand, _, is_default = tss_df.loc[gene_id]
            coords = converter.convert_coordinate(chrom38, tss38) if converter is not None else []
            if len(coords) == 0:
                no_map += 1
            elif not is_default:
                assert len(coords) == 1, f"hg38 to hg19 conversion returned multiple entries for {chrom38}," \
                                         f"position {tss38}"
                chrom, tss, _ = coords[0]
        genes.append((gene_id, chrom, int(tss), 1 if strand == "+" else -1))
    anno = pd.read_csv(args.annoFile, index_col=0)
    changed = sum(1 for g, c, t, s in genes if anno.loc[g, 'CAGE_representative_TSS'] != t)
    if rank == 0:
        print(f"Found {found} genes in geneAnno file that match a TSS in provided TSS file...")
        print(f"Failed to convert {no_map} hg38 positions to hg19 with liftover tool...")
        print(f"Found {changed} altered TSSs out of {anno.shape[0]} total TSSs...")
    dg = DeviceGenome(fasta)
    pipe = TSSPipeline(model.engine(), dg)
    # genes shard by contiguous rank ranges; rank 0 gathers the f64 [G_r, 20020] blocks (RCCL)
    lo, hi = edist.shard_range(len(genes), rank, world)
    feats = [pipe.features([g[1] for g in b], [g[2] for g in b], [g[3] for g in b])
             for b in _batches(genes[lo:hi], args.gene_batch)]
    mine = torch.cat(feats, 0) if feats else torch.zeros((0, 20020), dtype=torch.float64, device=dg.codes.device)
    full = edist.gather_rows_to(mine, 0, len(genes), world, rank)
    if rank != 0:
        return None
    arr = full.cpu().numpy()
    np.save(f'{args.out_dir}/Xreducedall.2002.representative_tss_top', arr)
    return arr


REPLICATE_LAST = {}   # timing of the last replicate run (bench.py's replicate_rank extra reads it)


def replicate_batch_genes(args, n_shifts: int) -> int:
    """Genes per streamed replicate batch: --gene-batch, capped so that one batch's host slot
    (n_shifts x 2002 fp32 per gene, two pinned slots) stays within --batch-gb."""
    per_gene = n_shifts * 2002 * 4
    cap = max(1, int(float(args.batch_gb) * (1 << 30)) // per_gene)
    return max(1, min(int(args.gene_batch), cap))


def replicate_main(argv=None):
    """replicate_expecto_features.py main() (:16-86): one (200,2002) float32 .npy per gene."""
    p = argparse.ArgumentParser(description='Replicate ExPecto chromatin features')
    p.add_argument('annoFile')
    p.add_argument('-o', dest="out_dir", type=str, default='temp_replicate_expecto_features')
    _common_args(p, gene_batch=96, max_batch=8192)
    p.add_argument('--batch-gb', type=float, default=2.0, dest='batch_gb',
                   help="cap on one batch's pinned host slot in GiB (two slots are kept)")
    p.add_argument('--write-threads', type=int, default=4, dest='write_threads',
                   help="threads writing a batch's per-gene .npy files")
    return replicate_run(p.parse_args(argv))


def replicate_run(args):
    """Streamed replicate (replicate_expecto_features.py:65-86): this rank's genes go through
    the device in batches of --gene-batch (default 96, the bench's step); batch k+1's windows,
    forward and fwd/rc mean are enqueued, with its D2H copy into one of two pinned slots, while
    batch k's per-gene .npy files are written from the other slot.  The f16x3 overflow check is
    deferred to each batch's release point (a flagged batch is recomputed in bf16x6 before its
    files are written), so no forward call waits on the host.

    Genes shard by contiguous rank ranges with no collective (per-gene files).  A gene id that
    appears more than once is computed once, at its LAST row: the reference writes every row in
    order, so the last one's file is what remains (replicate_expecto_features.py:86)."""
    from concurrent.futures import ThreadPoolExecutor
    import time
    t_start = time.perf_counter()
    if args.windowsize != 2000:
        raise ValueError("--windowsize must be 2000 (Beluga.py:43)")
    rank, world, local = edist.init()
    if world > 1:
        torch.cuda.set_device(edist.local_device(local))
    os.makedirs(args.out_dir, exist_ok=True)
    setup = {}
    t1 = time.perf_counter()
    fasta = Fasta(args.genome)
    setup["fasta_s"] = time.perf_counter() - t1
    t1 = time.perf_counter()
    model = _load_model(args)
    torch.cuda.synchronize()
    setup["model_s"] = time.perf_counter() - t1
    rows = _anno_genes(args.annoFile)
    last = {g[0]: i for i, g in enumerate(rows)}
    genes = [g for i, g in enumerate(rows) if last[g[0]] == i]
    lo, hi = edist.shard_range(len(genes), rank, world)
    mine = genes[lo:hi]
    t1 = time.perf_counter()
    dg = DeviceGenome(fasta)
    setup["device_genome_s"] = time.perf_counter() - t1
    eng = model.engine()
    pipe = TSSPipeline(eng, dg)
    S = len(pipe.shifts)
    B = replicate_batch_genes(args, S)
    nb = -(-len(mine) // B)
    slots = [torch.empty((min(B, len(mine)), S, 2002), dtype=torch.float32, pin_memory=True)
             for _ in range(min(2, nb))]
    tm = {"launch_s": 0.0, "wait_s": 0.0, "write_s": 0.0, "recomputed_batches": 0}

    def launch(k):
        b = mine[k * B:(k + 1) * B]
        job = {"genes": b, "flag": torch.zeros(1, dtype=torch.int32).pin_memory(), "event": torch.cuda.Event()}
        job["pred"] = pipe.pred_fwd_rc([g[1] for g in b], [g[2] for g in b], [g[3] for g in b])
        eng.overflow_take(job["flag"])
        job["host"] = slots[k % 2][:len(b)]
        job["host"].copy_(job["pred"], non_blocking=True)
        job["event"].record()
        return job

    def complete(job, pool):
        t1 = time.perf_counter()
        job["event"].synchronize()
        tm["wait_s"] += time.perf_counter() - t1
        b = job["genes"]
        if int(job["flag"][0]):
            # f16x3 overflow in this batch: recompute it in bf16x6 before its files are written
            with eng.precision_override("bf16x6"):
                pred = pipe.pred_fwd_rc([g[1] for g in b], [g[2] for g in b], [g[3] for g in b])
            eng.count_fallback()
            job["host"].copy_(pred)
            tm["recomputed_batches"] += 1
        t1 = time.perf_counter()
        arr = job["host"].numpy()
        list(pool.map(lambda i: np.save(f'{args.out_dir}/{b[i][0]}', arr[i]), range(len(b))))
        tm["write_s"] += time.perf_counter() - t1

    eng.set_overflow_check(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    try:
        with ThreadPoolExecutor(max(1, args.write_threads)) as pool:
            pending = None
            for k in range(nb):
                t1 = time.perf_counter()
                job = launch(k)                 # batch k computes while batch k-1 is written
                tm["launch_s"] += time.perf_counter() - t1
                if pending is not None:
                    complete(pending, pool)
                pending = job
            if pending is not None:
                complete(pending, pool)
    finally:
        eng.set_overflow_check(False)
    loop_s = time.perf_counter() - t0
    REPLICATE_LAST.clear()
    REPLICATE_LAST.update(loop_s=loop_s, setup_s=t0 - t_start, total_s=time.perf_counter() - t_start, setup=setup,
                          genes=len(mine), batches=nb, gene_batch=B, rank=rank, world=world,
                          conv2_table=dict(zip(("active", "state"), eng.conv2_table_state())), **tm)
    return dict(REPLICATE_LAST)


def atac_peak_bins(chrom, tss, strand, peaks: dict) -> np.ndarray:
    """expecto_intersect_chip_atac.py:198-217 get_atac_peak_bins: the 200 200-bp bins of the
    TSS receptive field, 1 where more than half a bin is covered by peaks.  The intersection
    (pybedtools ``tss_rf.intersect(peaks)``: the overlapping part of each peak) and the
    reference's inclusive ``[start, end + 1)`` marking are reproduced; bins are in genomic
    order for either strand, as in the reference."""
    rf_start = tss - 20899 - strand * 100
    rf_end = tss + 20900 - strand * 100
    regions = np.zeros(200 * 200)
    st, en = peaks.get(chrom, (np.zeros(0, np.int64), np.zeros(0, np.int64)))
    hit = (st < rf_end) & (en > rf_start)
    for s0, e0 in zip(np.maximum(st[hit], rf_start), np.minimum(en[hit], rf_end)):
        regions[int(s0) - rf_start:int(e0) - rf_start + 1] = 1
    return (regions.reshape(-1, 200).sum(axis=1) > 100).astype('float')


def read_bed(path) -> dict:
    """chrom -> (starts, ends) of a BED file (first three columns)."""
    df = pd.read_csv(path, sep='\t', header=None, comment='#', usecols=[0, 1, 2], dtype={0: str})
    return {c: (g[1].to_numpy(np.int64), g[2].to_numpy(np.int64)) for c, g in df.groupby(0, sort=False)}


def intersect_main(argv=None):
    """expecto_intersect_chip_atac.py main() (:16-111): TSS features with the ChIP-seq tracks
    (TF, or TF + histone) of every window multiplied by the ATAC peak bin of its shift."""
    p = argparse.ArgumentParser(description='Replicate ExPecto chromatin features')
    p.add_argument('annoFile')
    p.add_argument('peaks_file', help='Bed file containing ATAC binary peak calls')
    p.add_argument('-o', dest="out_dir", type=str, default='temp_expecto_intersect')
    p.add_argument('--tf_only', action='store_true')
    p.add_argument('--features_tsv', default='./resources/deepsea_beluga_2002_features.tsv')
    _common_args(p)
    args = p.parse_args(argv)
    if args.windowsize != 2000:
        raise ValueError("--windowsize must be 2000 (Beluga.py:43)")
    os.makedirs(args.out_dir, exist_ok=True)
    fasta = Fasta(args.genome)
    model = _load_model(args)
    feats_df = pd.read_csv(args.features_tsv, sep='\t', header=0, index_col=0)
    if args.tf_only:
        chip = np.where(feats_df['Assay type'] == 'TF')[0]
    else:
        chip = np.where((feats_df['Assay type'] == 'Histone') | (feats_df['Assay type'] == 'TF'))[0]
    genes = _anno_genes(args.annoFile)
    peaks = read_bed(args.peaks_file)
    dg = DeviceGenome(fasta)
    pipe = TSSPipeline(model.engine(), dg)
    chip_d = torch.from_numpy(chip.astype(np.int64)).to(pipe.dev)
    out = []
    for b in _batches(genes, args.gene_batch):
        y = pipe.predict([g[1] for g in b], [g[2] for g in b], [g[3] for g in b])     # [2, G, S, 2002]
        bins = np.stack([atac_peak_bins(g[1], g[2], g[3], peaks) for g in b]).astype(np.float32)
        mask = torch.from_numpy(bins).to(pipe.dev)                                   # [G, S]
        y[..., chip_d] *= mask[None, :, :, None]                                      # x1.0 / x0.0: exact
        out.append(tss_reduce(y[0], y[1], pipe.w_d).cpu().numpy())
    arr = np.concatenate(out, 0) if out else np.zeros((0, 20020))
    np.save(f'{args.out_dir}/Xreducedall.2002.atac_x_chip', arr)
    return arr


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "replicate":
        replicate_main(sys.argv[2:])
    elif len(sys.argv) > 1 and sys.argv[1] == "intersect":
        intersect_main(sys.argv[2:])
    else:
        compute_main(sys.argv[1:] if len(sys.argv) > 1 and sys.argv[1] != "compute" else sys.argv[2:])
