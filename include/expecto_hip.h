/*
 * expecto_hip.h -- C-ABI of the MI355X-native ExPecto Beluga hot path (gfx950).
 *
 * Every entry point takes plain pointers and sizes; device pointers are HIP device
 * memory, `stream` is a hipStream_t passed as void* (NULL = the null stream).  All
 * functions return 0 on success and a negative status on failure; the message of the
 * last failure on the calling thread is returned by expecto_last_error().
 *
 * Reference interfaces each entry point replaces (paths relative to the reference repo):
 *   expecto_beluga_create          Beluga() + load_state_dict(torch.load(pth)) + .cuda()
 *                                  (Beluga.py:18-48; chromatin.py:102-106;
 *                                   compute_expecto_features.py:36-40)
 *   expecto_beluga_forward_onehot  Beluga.forward(x[B,4,1,2000]) -> [B,2002]
 *                                  (Beluga.py:50-51; called at chromatin.py:270,278,
 *                                   compute_expecto_features.py:121-122)
 *   expecto_beluga_forward_codes   encodeSeqs(...) one-hot + Beluga.forward, fused: the
 *                                  one-hot / reverse-complement of chromatin.py:153-171
 *                                  is generated from base codes inside the conv1 + conv2
 *                                  k-mer gather (or the conv1 kernel)
 *   expecto_variant_windows        fetchSeqs window splice for SNVs (chromatin.py:175-209)
 *                                  from a device-resident genome
 *   expecto_indel_windows          fetchSeqs splice + centre crop for indels / MNPs
 *                                  (chromatin.py:164,202-209) from a device-resident genome
 *   expecto_tss_windows            TSS tiling genome.sequence(...) + encodeSeqs
 *                                  (compute_expecto_features.py:107-113)
 *   expecto_diff                   diff = alt - ref (chromatin.py:281)
 *   expecto_fwd_rc_average         (x[:N] + x[N:]) / 2 (predict.py:186-190;
 *                                   0.5*(fwd+rc) of compute_expecto_features.py:123)
 *   expecto_tss_reduce             pos_weights x pred_fwd_rc (compute_expecto_features.py:91-124)
 *   expecto_variant_reduce(_lut)   exp-decay shift weights x effects (predict.py:87-136)
 *   expecto_gblinear_predict       xgboost gblinear scoring of feature rows (predict.py:150-166)
 *   expecto_shift_reduce           200-shift reduction of consensus / eQTL sequences
 *                                  (geuvadis_sed_for_top_eqtls.py:95-121, geuvadis_predict_consensus.py:110-128)
 *   expecto_beluga_destroy         (model teardown)
 */
#ifndef EXPECTO_HIP_H
#define EXPECTO_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct expecto_beluga* expecto_beluga_t;

enum {
  EXPECTO_OK = 0,
  EXPECTO_EINVAL = -1,   /* bad argument (shape, pointer, mode)            */
  EXPECTO_EHIP = -2,     /* HIP runtime error                              */
  EXPECTO_ENOMEM = -3,   /* device allocation failed                       */
};

/* Strand modes of expecto_beluga_forward_codes. */
enum {
  EXPECTO_STRAND_FWD = 0,   /* n output rows: the windows as given                       */
  EXPECTO_STRAND_RC = 1,    /* n output rows: reverse complement of each window          */
  EXPECTO_STRAND_BOTH = 2,  /* 2n output rows: [fwd rows 0..n-1 ; rc rows n..2n-1]
                               (encodeSeqs row order, chromatin.py:170-171)             */
};

/* GEMM arithmetic (expecto_beluga_set_precision).  All accumulate in fp32:
 *  FP32   exact fp32 products and accumulation (v_mfma_f32_32x32x2_f32);
 *  BF16X6 every fp32 operand split exactly into three bf16 terms, the six products of
 *         combined order <= 2 accumulated in fp32 (v_mfma_f32_16x16x32_bf16); representation
 *         error < 2^-24 relative, products exact, over fp32's whole exponent range;
 *  F16X3  operands scaled by powers of 2 (weights per output channel; activations per layer,
 *         calibrated once per handle on a seeded batch) and split into two fp16 terms
 *         (22 significant bits), three products per k (v_mfma_f32_16x16x32_f16) -- half the
 *         MFMA work of BF16X6.  An activation that does not fit fp16 after scaling raises an
 *         overflow flag and the whole call is recomputed with BF16X6 (counted by
 *         expecto_beluga_f16_fallbacks), so F16X3 never returns a saturated result. */
enum {
  EXPECTO_PRECISION_FP32 = 0,
  EXPECTO_PRECISION_BF16X6 = 1,
  EXPECTO_PRECISION_F16X3 = 2,
};

/* Number of parameter tensors and their order (the reference state-dict keys,
 * SURVEY.md 2.2): model.0.{0,2,6,8,12,14}.{weight,bias}, model.1.2.1.{weight,bias},
 * model.1.4.1.{weight,bias}. */
#define EXPECTO_BELUGA_NPARAMS 16
#define EXPECTO_BELUGA_INPUT_LEN 2000
#define EXPECTO_BELUGA_NFEAT 2002

/* Build a model handle on `device`.  `params` are 16 DEVICE pointers to fp32 tensors in
 * the reference layouts (conv weight [Cout,Cin,1,8], fc weight [out,in]); they are
 * repacked into the kernels' layouts, so the caller may free them afterwards.
 * `max_batch` bounds the windows processed per internal chunk (workspace size).
 * The handle also builds (or shares, with other handles of this device holding the same
 * conv1 / conv2 weights) the k-mer tables its forwards from base codes gather conv1 + conv2
 * + pool1 from: 20.7 GB, ~40 ms, freed with the last handle using them; if they do not fit,
 * conv2 runs on the MFMAs.  EXPECTO_CONV2_TABLE=0 skips them. */
int expecto_beluga_create(int device, const float* const* params, int max_batch, void* stream,
                          expecto_beluga_t* out);
void expecto_beluga_destroy(expecto_beluga_t h);

/* Bytes of device memory the handle owns (weights + workspace) plus the k-mer tables it
 * holds (20.7 GB) if it is their first live holder: summed over handles that share one set of
 * tables, the tables count once. */
size_t expecto_beluga_device_bytes(expecto_beluga_t h);

/* 1 if the handle's forwards from base codes (and exact one-hot floats) gather conv1 + conv2 +
 * pool1 from the k-mer tables, 0 if they run conv1 / conv2 on the MFMAs (same parity bar, other
 * bits; about -25 % throughput).  *reason (may be NULL): 0 tables held, 1 switched off
 * (EXPECTO_CONV2_TABLE=0), 2 no room (the device allocation failed, or the tables exceed
 * EXPECTO_KMER_MAX_BYTES; the library then prints one line on stderr at creation). */
int expecto_beluga_conv2_table_active(expecto_beluga_t h, int* reason);

/* F16X3 computes FC1 (Beluga.py:43-44) as a block-Karatsuba convolution over 25-row blocks of the
 * conv6 rows: 4 windows 400 bp apart in one pool2-phase block of a segment share 9 block products
 * instead of 16 (DESIGN.md "FC1 as a block-Karatsuba convolution"; EXPECTO_FC1_KARATSUBA=0: the
 * direct FC1).  A window's FC1 is a sum of products of its own rows fixed by its ROLE, its position
 * in such a group: on the segment path (conv6 offset / 25) mod 4, every per-window forward (codes,
 * one-hot, pairs) the handle's role, 0 by default.  Role 4 is the direct FC1: segment-pair calls in
 * which more than a third of the windows hold the SNV run it for every window (their alt windows
 * would recompute nearly every product).  A window computed in the same role gives the same bits
 * on every path; other roles agree to the parity bar.  Sets the per-window role (0..4). */
int expecto_beluga_set_fc1_role(expecto_beluga_t h, int role);

/* y[n,2002] = Beluga.forward(x[n,4,1,2000]) (x contiguous fp32, any values).  When the handle
 * holds the k-mer tables, runs F16X3 or BF16X6, x is 16-byte aligned and every column of x is an
 * exact one-hot column (one 1.0f, three +0.0f) or all zeros, as encodeSeqs writes them
 * (chromatin.py:138-172), the call converts x to base codes and equals
 * expecto_beluga_forward_codes(FWD) bit for bit; otherwise conv1 / conv2 run on the MFMAs.  The
 * check costs one pass over x and one stream sync. */
int expecto_beluga_forward_onehot(expecto_beluga_t h, const float* x, int n, float* y, void* stream);

/* Windows given as base codes (uint8, 0=A 1=G 2=C 3=T 4=zero column for N/n/H/-),
 * window i at codes + i*code_stride, 2000 codes each.  y has n rows (FWD, RC) or 2n rows
 * (BOTH). */
int expecto_beluga_forward_codes(expecto_beluga_t h, const uint8_t* codes, int n, long long code_stride,
                                 int strand_mode, float* y, void* stream);

/* Windows that are slices of longer sequences ("segments") with a shared trunk: segment i
 * is seg_len codes at codes + i*code_stride (seg_len % 4 == 0); window w is the 2000 codes at
 * offset win_off[w] (a multiple of 4) of segment win_seg[w] (HOST arrays, sorted by segment).
 * conv1..conv4 run once per segment, conv5/conv6 once per (segment, pool2 phase), FC once per
 * window; every output equals the per-window forward bit for bit.  y has n_win rows (FWD:
 * the windows; RC: their reverse complements) or 2*n_win rows (BOTH: fwd rows then rc rows);
 * window w lands in row win_row[w] of its strand block (HOST array, a permutation of
 * 0..n_win-1; NULL = row w).
 * Replaces the per-shift re-encoding + forward of chromatin.py:243-279 and the 200-window
 * TSS tiling of compute_expecto_features.py:105-122. */
int expecto_beluga_forward_segments(expecto_beluga_t h, const uint8_t* codes, int n_seg, int seg_len,
                                    long long code_stride, int strand_mode, const int* win_seg, const int* win_off,
                                    const int* win_row, int n_win, float* y, void* stream);

/* Genome slices for segments: codes[i*seg_len + j] = genome[start[i] + j] (zero code outside
 * [0, genome_len)), with codes[i*seg_len + splice_pos[i]] = splice_code[i] when splice_code
 * is not NULL (the fetchSeqs allele splice of chromatin.py:209 for SNVs). */
int expecto_gather_segments(const uint8_t* genome, long long genome_len, const long long* start, int n,
                            int seg_len, const int* splice_pos, const uint8_t* splice_code, uint8_t* codes,
                            void* stream);

/* SNV ref/alt window pairs with alt-cone reuse: ref_codes/alt_codes are n windows each
 * (2000 codes at + v*code_stride) that differ at most at window index var_pos[v] (DEVICE array).
 * The ref windows run the full forward; each alt window recomputes, layer by layer, only the
 * rows the SNV changes (conv1 8, pool1 5, conv3 12, pool2 6, conv5 13, conv6 20 rows) from
 * input patches assembled out of the ref activations, so the alt trunk costs ~6 % of a window
 * -- outputs are bit-identical to the full alt forward.
 * strand_mode FWD (rows: fwd) or BOTH (fwd and reverse complement).  Output row of (strand s,
 * variant v) is s*strand_stride + v in y_ref and in y_alt (chromatin.py:262-281 row order
 * when strand_stride = n). */
int expecto_beluga_forward_pairs(expecto_beluga_t h, const uint8_t* ref_codes, const uint8_t* alt_codes, int n,
                                 long long code_stride, const int* var_pos, int strand_mode, float* y_ref,
                                 float* y_alt, long long strand_stride, void* stream);

/* SNV shift sweeps on the segment path with alt reuse: segment i (as in
 * expecto_beluga_forward_segments) is the REF sequence; its alt sequence has code
 * alt_code[i] (DEVICE array) at index var_pos[i] (HOST array, 0 <= var_pos[i] < seg_len).
 * Both alleles' windows are computed (same win_* tables): the ref trunk once per segment, and
 * for the alt only the rows the SNV changes at each layer (conv1 8, pool1 5, conv3 12, conv4
 * 19, pool2 6 per phase, conv5 13, conv6 20), assembled from the ref activations; alt windows
 * that do not hold the SNV equal their ref window and get a copy of its row -- bit-identical
 * to the full alt forward.  Window w of strand s lands in row s*strand_stride + win_row[w] of y_ref and of
 * y_alt.  Replaces the ref/alt forwards of chromatin.py:243-281 for --maxshift sweeps (and
 * the 200-shift eQTL variant scoring of geuvadis_sed_for_top_eqtls.py:61-98). */
int expecto_beluga_forward_segment_pairs(expecto_beluga_t h, const uint8_t* codes, const int* var_pos,
                                         const uint8_t* alt_code, int n_seg, int seg_len, long long code_stride,
                                         int strand_mode, const int* win_seg, const int* win_off, const int* win_row,
                                         int n_win, float* y_ref, float* y_alt, long long strand_stride,
                                         void* stream);

/* Select the GEMM arithmetic for later calls (a new handle starts in F16X3).  F16X3's fp16
 * weight planes and activation scales are built at handle creation: a BF16X6 forward of 256
 * seeded random windows; each layer's scale puts its largest calibration activation at
 * 2^target_log2, default 10, leaving >= 2^5 of headroom below fp16's 65504 before the
 * fallback. */
int expecto_beluga_set_precision(expecto_beluga_t h, int precision);
int expecto_beluga_get_precision(expecto_beluga_t h);
/* F16X3 calibration target (log2 of the scaled calibration maximum, 0..20); re-derives the
 * scales.  Tests use a large target to force the overflow fallback. */
int expecto_beluga_set_f16_target(expecto_beluga_t h, int target_log2);
/* F16X3 state: activation scale exponents of the 7 layer inputs (conv2..fc2) into sx[7];
 * returns the number of calls recomputed with BF16X6 after an overflow (or < 0 on error). */
long long expecto_beluga_f16_fallbacks(expecto_beluga_t h, int* sx);

/* F16X3 overflow check mode.  deferred = 0 (default): every forward call reads the device
 * overflow flag when its kernels are done (one stream sync per call) and recomputes itself with
 * BF16X6 if an activation did not fit fp16, so outputs are final when the call returns.
 * deferred = 1: calls only enqueue work (no host sync inside a forward); the flag stays set on
 * the device until expecto_beluga_overflow_pending() is called at the caller's release point
 * (before outputs are copied out), which syncs `stream`, returns 1 if any call since the last
 * check overflowed (and clears the flag; the caller then recomputes those calls with BF16X6),
 * else 0 (< 0 on error).  One exception to "no host sync": expecto_beluga_forward_onehot on a
 * handle that holds the k-mer tables runs a one-hot check pass over x and syncs once per call to
 * pick its path (codes through the tables, or the MFMA conv1 / conv2 for other floats) before it
 * enqueues the forward; EXPECTO_ONEHOT_CODES=0 (always the MFMA path) or forward_codes avoid it. */
int expecto_beluga_set_overflow_check(expecto_beluga_t h, int deferred);
int expecto_beluga_overflow_pending(expecto_beluga_t h, void* stream);
/* Deferred mode, streamed batches: enqueue on `stream` a copy of the flag into *dst (pinned host
 * or device memory) followed by its reset, without a host sync.  Enqueued right after a batch's
 * forward calls, *dst holds exactly that batch's overflow state once an event recorded after it
 * has completed (the stream runs in order), while later batches are already queued. */
int expecto_beluga_overflow_take(expecto_beluga_t h, int* dst, void* stream);
/* Deferred mode: the caller acted on a flag obtained through expecto_beluga_overflow_take and
 * recomputed that batch with BF16X6; adds one to the count expecto_beluga_f16_fallbacks reports
 * (expecto_beluga_overflow_pending counts its own). */
int expecto_beluga_count_fallback(expecto_beluga_t h);

/* Per-layer device time accumulated over forward calls while profiling is on (ms), launches
 * (`calls`) and executed multiply-adds (`macs`: GEMM M x N x K actually run, including the
 * few padding rows; reuse paths execute fewer than the dense per-window count).
 * Layers: 0 conv1, 1 conv2, 2 conv3, 3 conv4 (+ pool2 on the segment/patch paths), 4 conv5,
 * 5 conv6, 6 fc1, 7 fc1-reduce, 8 fc2; entries 9..17 are the same layers' alt-delta launches
 * (forward_pairs / forward_segment_pairs), timed apart from the full-window launches.
 * Fills min(max_layers, 18) entries and returns 18. */
int expecto_beluga_set_profiling(expecto_beluga_t h, int on);
int expecto_beluga_layer_times(expecto_beluga_t h, double* ms, long long* calls, double* macs, int max_layers);

/* While profiling, every conv GEMM launch (conv2-6) is also timed alone -- its own HIP event pair on
 * the launch stream, without the pool2 pass that shares the conv4 slot -- and logged by (slot, rows).
 * Returns the group of slot `slot` (layer_times numbering) with the most rows: the full-size
 * launches, *rows each, *calls of them, their summed *ms and executed *macs.  bench.py's roofline
 * reads this (the rocprofv3 launch_groups.csv of the same command lists the same launches). */
int expecto_beluga_main_launches(expecto_beluga_t h, int slot, long long* rows, double* ms, long long* calls,
                                 double* macs);

/* SNV windows from a device-resident genome (uint8 codes as above).  For variant v and
 * shift s the 2000-code window is genome[off_v + shift - 999 + i], i = 0..1999, with the
 * code at index 999 - shift replaced by ref_code[v] (allele 0) or alt_code[v] (allele 1)
 * (chromatin.py:202-209 then the centre crop of :164).  off_v = 0-based genome offset of
 * the variant base.  Output codes[((a*n_shift + j)*n + v)*2000 + i] for allele a in {0,1}. */
int expecto_variant_windows(const uint8_t* genome, long long genome_len, const long long* var_off,
                            const uint8_t* ref_code, const uint8_t* alt_code, int n,
                            const int* shifts, int n_shift, uint8_t* codes, void* stream);

/* Indel / MNP windows (chromatin.py:202-209, centre crop :164).  Item t's 2100-base fetch
 * window starts at 0-based genome offset start0[t]; the allele (lalt[t] codes at
 * allele_codes[allele_off[t]..]) replaces lref[t] bases at mutpos[t]; output
 * codes[t*2000 + i] = S[crop[t] + i] of the spliced sequence S (crop = floor((len(S)-2000)/2)).
 * Callers keep items with a window past the contig, mutpos < 0, mutpos + lref > 2100 or
 * len(S) < 2000 on the host (the reference's Python-slicing corner cases). */
int expecto_indel_windows(const uint8_t* genome, long long genome_len, const long long* start0,
                          const int* mutpos, const int* lref, const int* lalt, const int* crop,
                          const int* allele_off, const uint8_t* allele_codes, int n, uint8_t* codes,
                          void* stream);

/* TSS tiling windows (compute_expecto_features.py:107-111): gene g, shift j covers the
 * 0-based genome offsets tss_off[g] + shifts[j]*strand[g] - 999 + i, i = 0..1999
 * (strand = +1/-1).  Output codes[(g*n_shift + j)*2000 + i]. */
int expecto_tss_windows(const uint8_t* genome, long long genome_len, const long long* tss_off, const int8_t* strand,
                        int n_genes, const int* shifts, int n_shift, uint8_t* codes, void* stream);

/* out[i] = a[i] - b[i], i < count (fp32). */
int expecto_diff(const float* alt, const float* ref, long long count, float* out, void* stream);

/* out[r, f] = (x[r, f] + x[r + rows, f]) / 2 for r < rows, f < cols (fp32). */
int expecto_fwd_rc_average(const float* x, int rows, int cols, float* out, void* stream);

/* TSS reduction for n_genes genes: fwd and rc are [n_genes, n_shift, nfeat] fp32;
 * weights [10, n_shift] fp64; out [n_genes, 10*nfeat] fp64 with
 * out[g, k*nfeat + f] = sum_s weights[k,s] * (0.5f*(fwd[g,s,f] + rc[g,s,f])).
 * The reductions below stage their weights in 64 KiB of LDS: n_shift <= 819 (EXPECTO_EINVAL
 * otherwise; the reference sweeps 9 to 201 shifts). */
int expecto_tss_reduce(const float* fwd, const float* rc, const double* weights, int n_genes, int n_shift,
                       int nfeat, double* out, void* stream);

/* Variant reduction: effects [n_shift, n, nfeat] fp32 (fwd/rc-averaged, shift order of
 * chromatin.py:243), dist[n] (pos - TSS, int64), strand_plus[n] (1 '+', 0 '-'),
 * shifts[n_shift]; out [n, 10*nfeat] fp64 (predict.py:87-124 feature layout). */
int expecto_variant_reduce(const float* effects, const long long* dist, const uint8_t* strand_plus,
                           const int* shifts, int n_shift, int n, int nfeat, double* out, void* stream);
/* The same with the decay factors from a table: exp_lut[k*lut_len + fl] = exp(-c_k * fl)
 * (c = 0.01, 0.02, 0.05, 0.1, 0.2; DEVICE array) computed by the caller with the reference's
 * own exp (numpy, predict.py:88-107), so the features equal the reference's bit for bit;
 * expecto_variant_reduce uses the device exp (within 1 ulp).  A distance whose fl =
 * floor(|d|/200) is >= lut_len takes the device exp too (never a read past the table). */
int expecto_variant_reduce_lut(const float* effects, const long long* dist, const uint8_t* strand_plus,
                               const int* shifts, int n_shift, int n, int nfeat, const double* exp_lut, int lut_len,
                               double* out, void* stream);

/* Shift reduction of per-sequence window predictions (fwd and rc [n, n_shift, nfeat] f32, DEVICE)
 * with exp-decay weights [10, n_shift] f64 into float64 features, shifts summed in order.
 * flags bit 0 (EXPECTO_REDUCE_F64AVG): average fwd/rc in float64 (numpy on float64 prediction
 * arrays, geuvadis_*.py) instead of 0.5f*(a+b) in float32 (compute_expecto_features.py:123);
 * bit 1 (EXPECTO_REDUCE_LEGACY20030): out[n, 10, nfeat+1] with a zero column ahead of each
 * decay block ("backwards compatibility" layout, geuvadis_sed_for_top_eqtls.py:112-120),
 * else out[n, 10, nfeat]. */
#define EXPECTO_REDUCE_F64AVG 1
#define EXPECTO_REDUCE_LEGACY20030 2
int expecto_shift_reduce(const float* fwd, const float* rc, const double* weights, int n_genes, int n_shift, int nfeat,
                         int flags, double* out, void* stream);

/* ExPecto expression scoring with an xgboost gblinear model (predict.py:150-166;
 * xgboost 0.7 GBLinear::Pred): out[m] = init + sum_j float32(X[m*ld + cols[j]]) * w[j],
 * summed in float32 in column order with every product and sum rounded separately;
 * init = float32(bias + base_score).  X: float64 feature rows (DEVICE), cols: int32[ncols]
 * (the keep-mask column map of predict.py:137-145), w: float32[ncols]. */
int expecto_gblinear_predict(const double* X, long long n, long long ld, const int* cols, int ncols, const float* w,
                             float init, float* out, void* stream);

const char* expecto_last_error(void);
const char* expecto_version(void);

#ifdef __cplusplus
}
#endif
#endif /* EXPECTO_HIP_H */
