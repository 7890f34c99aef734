// fp32-MFMA implicit-GEMM kernel template (gfx950) shared by the library and tools/gemm_bench.
//
// C[m][n] = epilogue( sum_k A[m][k] * B[n][k] ), A rows may overlap (conv Toeplitz rows).
// Tile: (32*WM) rows x 160 cols x BK k; WM waves stacked along M, each 32 x 160 =
// five 32x32 accumulators of v_mfma_f32_32x32x2_f32 (exact fp32, fmaf-chain numerics).
// K is consumed in 32-wide "blocks" (one (chunk, tap) pair of a conv); a BK=64 stage holds
// two consecutive blocks.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

namespace expecto {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int GBN = 160;
constexpr int GBK = 32;               // K block (one conv (chunk, tap) pair)
constexpr int GTN = GBN / 32;

enum { EPI_RELU = 0, EPI_RELU_POOL4 = 1, EPI_SIGMOID = 2, EPI_PARTIAL = 3, EPI_POOL_PH02 = 4 };

struct GemmArgs {
  const float* A;
  long long lda;
  long long M;
  const float* B;  // [Npad][ldb], K-contiguous
  long long ldb;
  int kper;        // K range per split, multiple of the stage depth BK
  int taps;        // conv: 8 (K order = [ci/32][tap][ci%32]); fc: 1
  int n_tiles;
  long long m_tiles;
  int m_fastest;
  const float* bias;
  float* C;
  long long ldc;
  int n_store;
  int s_in;     // rows per window in the A/M index space
  int t_valid;  // valid output positions (pooled count for EPI_RELU_POOL4)
  int s_out;    // rows per window in C
  long long split_stride;
  const long long* a_rows;  // optional: A row m starts at A + a_rows[m] (FC1 over segment windows)
  const long long* c_rows;  // optional: C row of M row m (non-pool epilogues; FC2 output order)
  const void* Bp;           // bf16x6 GEMM: B as bf16 planes [Npad][K/32][3][32] (split_planes)
  int linear_order;         // bf16x6 GEMM: blocks in dispatch order (no XCD grouping); FC1 sets it
                            // so every XCD sweeps the same K slab at once (Infinity-Cache reuse)
  const float* col_scale;   // f16x3: per-column 2^-(s_in + s_w[n]) undoing the operand scales (else null)
  float out_scale;          // f16x3: 2^s_out applied to stored activations (next layer's input scale)
  int* ovf;                 // f16x3: set to 1 when a stored activation does not fit fp16
  const unsigned* ks_mask;  // split-K planes GEMM: bit ks of ks_mask[m_tile] = compute that slab
                            // (others keep the partials already in C: alt FC1 of SNV pairs)
  int m_group;              // FC m_fastest 3: M tiles per dispatch group (see gemm_fc_h3p_body)
  int n_tile_cols;          // f16x3 split-K FC: columns per N tile the caller tiled for (FCW_BN:
                            // beluga_fc_h3w; 0 = the 160-column kernels)
  // conv2 with conv1 fused (f16x3, beluga_conv_h3p with TM & H3P_FUSE_CONV1): A is not read; the
  // producer waves compute each 32-channel chunk's slab of conv1 rows from base codes.  Conv1 row
  // m = (window w, position t) with w = m / s_in; window w is code row c1_row0 + w of c1_codes
  // (c1_mode: 0 fwd, 1 rc, 2 both = rows >= c1_n_src are the rc of row - c1_n_src, as
  // EXPECTO_STRAND_*), c1_len bases; c1_n_win windows, c1_len - 7 valid conv1 rows each.
  const unsigned char* c1_codes;
  long long c1_stride;
  long long c1_row0;
  int c1_n_src, c1_mode, c1_len, c1_n_win;
  const _Float16* c1_w;     // conv1 weight planes [320][hi 32 | lo 32] (k = tap*4 + ci)
  const float* c1_cs;       // conv1 per-channel unscale
  const float* c1_b;        // conv1 bias
  float c1_osc;             // conv2 input scale 2^sx[0]
  unsigned long long* stamps;   // diagnostic builds only (TM & H3P_STAMP, tools/ck_bench): per-wave cycle sums
  // EPI_POOL_PH02 (segment path, conv4 + pool2 phases 0 and 2 in the epilogue): C = the phase blocks
  // (segment w, phase i at rows (2 w + i) * s_out).  Unpooled rows (plain split) only where others
  // read them: c_seam gets each 256-row tile's rows 0, 1, 254, 255 (4 rows per tile, pool2_tile_seams),
  // and with unp_tab c_edge the ref rows seg_delta_pool pools (phase 0 from pooled row tab[5], phase
  // 2 from tab[6], unp_dw pooled rows each): 32 rows per segment from the first of them
  float* c_seam;
  float* c_edge;
  const int* unp_tab;
  int unp_ld, unp_dw;
};
constexpr int H3P_FUSE_CONV1 = 16384;
// Diagnostic build of beluga_conv_h3p (tools/ck_bench "stamp"; the library never sets it): s_memtime
// stamps around each stage's barrier (consumers) and each stage's vmcnt wait + barrier (producers),
// summed per wave into p.stamps[(block * 8 + wave) * 4 + {0 loop, 1 barrier, 2 vmcnt wait, 3 epilogue}].
constexpr int H3P_STAMP = 4096;
__device__ __forceinline__ unsigned long long h3p_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

// Exact 3-way bf16 split x = x0 + x1 + x2 (RNE at each level; 3 x 8 significant bits cover
// fp32's 24).  Every split site (weights, epilogues, pooling, reduce) uses this one routine,
// so a value always has the same planes wherever it was split.
__device__ __forceinline__ void split1(const float x, __bf16& x0, __bf16& x1, __bf16& x2) {
  x0 = (__bf16)x;
  const float r = x - (float)x0;
  x1 = (__bf16)r;
  x2 = (__bf16)(r - (float)x1);
}

__device__ __forceinline__ void split3(const floatx4 x, bf16x4& h, bf16x4& m, bf16x4& l) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    __bf16 a, b, c;
    split1(x[j], a, b, c);
    h[j] = a;
    m[j] = b;
    l[j] = c;
  }
}

// Activation storage formats (FMT):
//   0  fp32 rows [rows][ld];
//   1  bf16x6 path: bf16 planes [rows][ld/32][3][32] -- each 32-channel block of a row holds its
//      x0, x1, x2 planes back to back (192 B), so a consumer's 32-deep K block is one contiguous
//      192-B run per row;
//   2  f16x3 path: fp16 planes [rows][ld/32][2][32] of the SCALED value x * 2^s (x = hi + lo,
//      128 B per 32-channel block).  s is the consumer layer's input scale (calibrated per
//      handle so that activations sit well inside fp16's exponent range); a value that does not
//      fit (|x * 2^s| >= 65504) raises the handle's overflow flag and the call is recomputed
//      on the bf16x6 path.
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));
typedef _Float16 halfx4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// fp16 1.0 (0x3C00) in the half of channel c within the channel pair (0,1) or (2,3): one dword of
// a one-hot conv1 operand fragment (codes 0..3 = A,G,C,T; 4 = N, all zero)
__device__ __forceinline__ unsigned onehot_h2(unsigned c, unsigned hi_pair) {
  return (c >> 1) == hi_pair ? (0x3C00u << ((c & 1u) * 16u)) : 0u;
}

template <int PL>
__device__ __forceinline__ long long act_index(long long row, long long ld, int n) {
  return ((row * (ld >> 5) + (n >> 5)) * PL) * 32 + (n & 31);
}
__device__ __forceinline__ long long x3_index(long long row, long long ld, int n) { return act_index<3>(row, ld, n); }

// 2-way fp16 split of an (already scaled) fp32 value.  r = RNE16(x) + RNE16(x - RNE16(x)) is x
// rounded to >= 22 significant bits and is exact in fp32; the stored pair is the CANONICAL
// split of r, hi = RNE16(r), lo = r - hi (exact in fp16).  The pair then depends on r alone, so
// re-splitting a recovered value (max pooling of stored rows on the segment path) reproduces
// the pair the per-window path stores for the same value -- bit-identical paths.  (Without the
// second step a tie |lo| = ulp(hi)/2 re-splits to (hi +- ulp, -lo): same value, other products.)
__device__ __forceinline__ void split_h2(const float x, _Float16& hi, _Float16& lo) {
  const _Float16 h0 = (_Float16)x;
  const float r = (float)h0 + (float)(_Float16)(x - (float)h0);
  hi = (_Float16)r;
  lo = (_Float16)(r - (float)hi);
}

// Plain 2-way split, hi = RNE16(x), lo = RNE16(x - hi): the same recovered value hi + lo as
// split_h2 (x rounded to >= 22 bits) at 2 conversions fewer.  Used wherever the planes are
// consumed as stored; values that are recovered and re-split (the unpooled conv4 rows of the
// segment path, pooled by pool4_phases / seg_delta_pool) must meet the values the other paths
// store as the CANONICAL pair of that recovered value: conv4's pooled epilogue and the pool
// kernels keep split_h2 (tools/gemm_bench: conv3 / conv5 / conv6 +3-4 % from the plain split).
__device__ __forceinline__ void split_h2p(const float x, _Float16& hi, _Float16& lo) {
  hi = (_Float16)x;
  lo = (_Float16)(x - (float)hi);
}

template <int FMT>
__device__ __forceinline__ void store_act(float* C, long long row, long long ld, int n, float v, float osc = 1.f,
                                          int* ovf = nullptr) {
  if constexpr (FMT == 1) {
    __bf16* d = reinterpret_cast<__bf16*>(C) + act_index<3>(row, ld, n);
    split1(v, d[0], d[32], d[64]);
  } else if constexpr (FMT == 2) {
    const float x = v * osc;
    if (!(fabsf(x) < 65504.f) && ovf) *ovf = 1;
    _Float16* d = reinterpret_cast<_Float16*>(C) + act_index<2>(row, ld, n);
    split_h2(x, d[0], d[32]);
  } else {
    C[row * ld + n] = v;
  }
}

// value as stored (fmt 2: still scaled -- max pooling commutes with the power-of-2 scale)
template <int FMT>
__device__ __forceinline__ float load_act(const float* A, long long row, long long ld, int n) {
  if constexpr (FMT == 1) {
    const __bf16* s = reinterpret_cast<const __bf16*>(A) + act_index<3>(row, ld, n);
    return (float)s[0] + ((float)s[32] + (float)s[64]);   // exact: recovers the split value
  } else if constexpr (FMT == 2) {
    const _Float16* s = reinterpret_cast<const _Float16*>(A) + act_index<2>(row, ld, n);
    return (float)s[0] + (float)s[32];                      // exact (22 significant bits)
  } else {
    return A[row * ld + n];
  }
}
__device__ __forceinline__ float load_x3(const float* A, long long row, long long ld, int n) {
  return load_act<1>(A, row, ld, n);
}

// runtime-format helpers for the small kernels (conv1, pooling, FC1 reduce)
__device__ __forceinline__ void store_act_rt(int fmt, float* C, long long row, long long ld, int n, float v,
                                             float osc = 1.f, int* ovf = nullptr) {
  if (fmt == 1)
    store_act<1>(C, row, ld, n, v);
  else if (fmt == 2)
    store_act<2>(C, row, ld, n, v, osc, ovf);
  else
    store_act<0>(C, row, ld, n, v);
}
__device__ __forceinline__ float load_act_rt(int fmt, const float* A, long long row, long long ld, int n) {
  return fmt == 1 ? load_act<1>(A, row, ld, n) : fmt == 2 ? load_act<2>(A, row, ld, n) : load_act<0>(A, row, ld, n);
}

// Epilogue shared by both GEMM kernels. C/D layout of 32x32 MFMA (every dtype on gfx950):
// col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5), so rows 4g..4g+3 of a pool window sit
// in registers 4q..4q+3 of ONE lane.
template <int EPI, bool X3 = false>
__device__ __forceinline__ void gemm_epilogue(const GemmArgs& p, const floatx16 (&acc)[GTN], long long mw, int n0,
                                              int ks, int li, int lh) {
#pragma unroll
  for (int t = 0; t < GTN; ++t) {
    const int n = n0 + t * 32 + li;
    if (n >= p.n_store) continue;
    if (EPI == EPI_PARTIAL) {
      float* cp = p.C + (long long)ks * p.split_stride + n;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long long m = mw + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m < p.M) cp[m * p.ldc] = acc[t][r];
      }
    } else if (EPI == EPI_RELU_POOL4) {
      const float bn = p.bias[n];
#pragma unroll
      for (int qd = 0; qd < 4; ++qd) {
        const long long m = mw + 8 * qd + 4 * lh;  // first of 4 pooled rows (multiple of 4)
        if (m >= p.M) continue;
        const long long w = m / p.s_in;
        const int tp = (int)(m - w * p.s_in) >> 2;
        if (tp >= p.t_valid) continue;
        float mx = fmaxf(fmaxf(acc[t][4 * qd], acc[t][4 * qd + 1]), fmaxf(acc[t][4 * qd + 2], acc[t][4 * qd + 3]));
        // maxpool(relu(x+b)) == relu(max(x)+b): x -> fl(x+b) and relu are monotone.
        store_act<X3>(p.C, w * p.s_out + tp, p.ldc, n, fmaxf(mx + bn, 0.f));
      }
    } else {
      const float bn = p.bias[n];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long long m = mw + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m >= p.M) continue;
        const long long w = m / p.s_in;
        const int tpos = (int)(m - w * p.s_in);
        if (tpos >= p.t_valid) continue;
        const float v = acc[t][r] + bn;
        const long long orow = p.c_rows ? p.c_rows[m] : (w * p.s_out + tpos);
        if (EPI == EPI_SIGMOID)
          p.C[orow * p.ldc + n] = 1.0f / (1.0f + expf(-v));
        else
          store_act<X3>(p.C, orow, p.ldc, n, fmaxf(v, 0.f));
      }
    }
  }
}

// LAYER only makes the symbol distinct per layer (rocprof attributes time per layer).
template <int LAYER, int EPI, int WM = 4, int MINB = 2, int BK = 32, int PIPE = 0>
__global__ __launch_bounds__(64 * WM, MINB * WM / 4) void beluga_gemm(GemmArgs p) {
  constexpr int BM = 32 * WM;
  constexpr int NT = 64 * WM;
  constexpr int LDS_STRIDE = BK + 4;             // rows of 36/68 floats: b128 reads conflict-free
  constexpr int F4 = BK / 4;                     // float4 per tile row
  constexpr int RSTEP = NT / F4;                 // rows covered by one load pass
  constexpr int ALD = BM / RSTEP;                // float4 A loads per thread
  constexpr int BLD = (GBN + RSTEP - 1) / RSTEP; // float4 B loads per thread
  constexpr int KB = BK / GBK;                   // K blocks per stage
  static_assert(BM % RSTEP == 0, "tile rows must be a multiple of the load pass");
  __shared__ __attribute__((aligned(16))) float smem[(BM + GBN) * LDS_STRIDE];
  float* As = smem;
  float* Bs = smem + BM * LDS_STRIDE;

  // XCD-aware remap: blocks b, b+8, b+16.. share an XCD; give them consecutive tiles.
  const unsigned nblk = gridDim.x, bid = blockIdx.x;
  const unsigned xcd = bid & 7u, q = nblk >> 3, rr = nblk & 7u;
  const unsigned lin = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  long long mt;
  int nt, ks;
  if (p.m_fastest) {
    mt = lin % p.m_tiles;
    const long long rest = lin / p.m_tiles;
    nt = (int)(rest % p.n_tiles);
    ks = (int)(rest / p.n_tiles);
  } else {
    nt = (int)(lin % (unsigned)p.n_tiles);
    const long long rest = lin / (unsigned)p.n_tiles;
    mt = rest % p.m_tiles;
    ks = (int)(rest / p.m_tiles);
  }

  const int tid = threadIdx.x;
  const int lr = tid / F4, lc = (tid % F4) * 4;
  const int lkb = lc / GBK, lcc = lc % GBK;        // K block of this thread's A column
  const long long m0 = mt * BM;
  const int n0 = nt * GBN;
  // K stages: global stage gs -> (chunk = gs / taps, tap = gs % taps).  A stage = rows
  // m+tap of channels chunk*32..+31 (taps innermost keeps the 32-channel slice L1/L2-hot
  // across the 8 taps); B is repacked in the same [chunk][tap][32] order, so its stage
  // offset is simply gs*32.
  const int gs0 = ks * (p.kper / GBK);             // first K block of this split

  const float* ag[ALD];
#pragma unroll
  for (int i = 0; i < ALD; ++i) {
    long long m = m0 + lr + RSTEP * i;
    if (m > p.M - 1) m = p.M - 1;  // clamp: tail rows read valid memory, never stored
    ag[i] = p.A + (p.a_rows ? p.a_rows[m] : m * p.lda) + lcc;
  }
  const float* bg[BLD];
#pragma unroll
  for (int i = 0; i < BLD; ++i) {
    const int r = min(lr + RSTEP * i, GBN - 1);
    bg[i] = p.B + (long long)(n0 + r) * p.ldb + (long long)gs0 * GBK + lc;
  }
  auto a_off = [&](int gs) -> long long {
    const int chunk = gs / p.taps, tap = gs - chunk * p.taps;
    return (long long)tap * p.lda + chunk * GBK;
  };
  auto b_ok = [&](int i) { return (GBN % RSTEP == 0) || (lr + RSTEP * i < GBN); };

  floatx4 ra[ALD], rb[BLD];
  const int wave = tid >> 6, lane = tid & 63, li = lane & 31, lh = lane >> 5;
  floatx16 acc[GTN];
#pragma unroll
  for (int t = 0; t < GTN; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  // k order inside a 32-deep stage: MFMA step s = 4g+qq, lane half h takes k = 8g+4h+qq,
  // so each lane feeds 4 consecutive MFMAs from one ds_read_b128 (same order for A and B).
  const float* aw = As + (wave * 32 + li) * LDS_STRIDE + 4 * lh;
  const float* bw = Bs + li * LDS_STRIDE + 4 * lh;
  const int nk = p.kper / BK;

  auto gload = [&](int s) {
    const long long ao = a_off(gs0 + s * KB + lkb);
#pragma unroll
    for (int i = 0; i < ALD; ++i) ra[i] = *(const floatx4*)(ag[i] + ao);
#pragma unroll
    for (int i = 0; i < BLD; ++i) rb[i] = *(const floatx4*)(bg[i] + s * BK);
  };
  auto sstore = [&]() {
#pragma unroll
    for (int i = 0; i < ALD; ++i) *(floatx4*)(As + (lr + RSTEP * i) * LDS_STRIDE + lc) = ra[i];
#pragma unroll
    for (int i = 0; i < BLD; ++i)
      if (b_ok(i)) *(floatx4*)(Bs + (lr + RSTEP * i) * LDS_STRIDE + lc) = rb[i];
  };

  gload(0);
  sstore();
  __syncthreads();

  for (int s = 0; s < nk; ++s) {
    const bool more = (s + 1) < nk;
    if (more) gload(s + 1);
    // Fragment reads are software-pipelined one 8-k group ahead (two register sets), so
    // the ds_read latency of group g+1 hides under the 20 MFMAs of group g.
    floatx4 fa[2], fb[2][GTN];
    fa[0] = *(const floatx4*)(aw);
#pragma unroll
    for (int t = 0; t < GTN; ++t) fb[0][t] = *(const floatx4*)(bw + t * 32 * LDS_STRIDE);
#pragma unroll
    for (int g = 0; g < BK / 8; ++g) {
      const int cur = g & 1, nxt = cur ^ 1;
      if (g + 1 < BK / 8) {
        fa[nxt] = *(const floatx4*)(aw + 8 * (g + 1));
#pragma unroll
        for (int t = 0; t < GTN; ++t) fb[nxt][t] = *(const floatx4*)(bw + t * 32 * LDS_STRIDE + 8 * (g + 1));
      }
#pragma unroll
      for (int qq = 0; qq < 4; ++qq)
#pragma unroll
        for (int t = 0; t < GTN; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[cur][qq], fb[cur][t][qq], acc[t], 0, 0, 0);
      if (PIPE && g + 1 < BK / 8) {
        // pin the order: the 1 + GTN reads of group g+1 interleave with group g's first MFMAs
#pragma unroll
        for (int i = 0; i < 1 + GTN; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 4 * GTN - 1 - GTN, 0);
      }
    }
    __syncthreads();
    if (more) {
      sstore();
      __syncthreads();
    }
  }

  gemm_epilogue<EPI>(p, acc, m0 + wave * 32, n0, ks, li, lh);
}

// ---- bf16x6 on pre-split planes with LDS-DMA staging (the library's bf16x6 GEMM) ----------
// Every fp32 operand x is split exactly into three bf16 terms x = x0 + x1 + x2 (split1 /
// split3); each 32-deep k-step issues the six products of combined order <= 2 (x0y0, x0y1,
// x1y0, x0y2, x1y1, x2y0) into one fp32 accumulator.  Products of bf16 terms are exact in fp32,
// so the result is fp32-accurate (tools/split_precision_study.py: 0.06 of the parity bound on
// alt-ref diffs, vs 0.08 for oneDNN fp32).  Data movement:
//  * B (weights) is split once at handle creation into planes [n][k/32][3][32] (split_planes);
//  * A (activations) is split once by the PRODUCING layer's epilogue into the same planes
//    layout (store_act<true>), not once per Toeplitz tap;
//  * both tiles arrive by LDS-DMA (buffer_load_dwordx4 ... lds: constant lane offsets in
//    voffset, the stage offset in soffset) into a double-buffered LDS ring, one raw barrier
//    per 32-deep K block; each wave stages its own 64 A rows, so it waits for them with its
//    own counted vmcnt, not a barrier;
//  * each wave owns 64 x 160 as 4 x 10 blocks of v_mfma_f32_16x16x32_bf16 (160 AGPRs), four
//    waves = 256 x 160, one workgroup per CU; B fragments are prefetched one unit ahead and the
//    LDS-DMA pieces are issued between units (sched_group_barrier-pinned).
// Stage = A planes 48 KB + B planes 30 KB + 2 KB pad = 80 KB; two stages fill the CU's LDS.
// Per wave and stage: 12 A pieces (its rows x 3 planes) + 8 B pieces (30 real + 2 dummies).
// tools/gemm_bench, conv2 shape, 1000 windows (fp32-equivalent TF/s): 284 here, vs 234 for
// the same data path on 32x32x16 MFMAs (the 16x16x32 form holds a higher clock under load,
// MI355X_MICROARCH.md DVFS item 7), 197 for a register-staged kernel that re-split A per tap
// (tools/gemm_probes.h) and 140 for the fp32 kernel.
constexpr int X6P_BM = 256;
constexpr int X6P_B_PLANE = GBN * 64;                     // 10 KB
constexpr int X6P_A_PLANE = X6P_BM * 64;                  // 16 KB

// Stage bytes for PL operand planes: A planes + B planes (+ room for the B pieces' dummy tail).
template <int PL>
struct PlaneGeo {
  static constexpr int A_BYTES = PL * X6P_A_PLANE;
  static constexpr int B_GROUPS = PL * 10;                  // 1 KiB B pieces (16 rows x 64 B)
  static constexpr int B_PER_WAVE = (B_GROUPS + 3) / 4;     // 8 (PL 3: 30 real + 2 dummies) / 5
  static constexpr int STAGE = A_BYTES + 4 * B_PER_WAVE * 1024;   // 81,920 / 53,248 B
  static constexpr int A_PIECES = 4 * PL;                   // per wave and stage
  static constexpr int ROW_KB = 64 * PL;                    // global bytes per row and 32-deep K block
};
constexpr int X6P_STAGE = PlaneGeo<3>::STAGE;

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

__device__ __forceinline__ void glds16(const void* src, char* lds_dst) {
  __builtin_amdgcn_global_load_lds((glb_void*)src, (lds_void*)lds_dst, 16, 0, 0);
}


// TM: timing-only probes for tools/gemm_bench (wrong results; production launches TM 0, the
// producer / consumer conv kernel TM 256): 2 = no LDS-DMA in the loop, 4 = no barrier in the
// loop, 8 = LDS-DMA always from stage 0's (L2-hot) addresses; beluga_fc_h3p also 16 / 32 = only
// the A / B pieces L2-hot; beluga_conv_h3p 2048 = no epilogue; the f16x3 conv kernels 8192 =
// round 2's per-column epilogue factor loads (epi_factors).
// 16x16x32 lane layout: A/B lane l holds row/col (l & 15), k = 8*(l >> 4)..+7; C lane l
// holds col (l & 15), rows 4*(l >> 4)..+3.  The 16 lanes of one ds_read_b128 lane group then
// read mixed chunks, so LDS-DMA pieces (lane-linear 1 KiB = 16 rows x 64 B) are placed with an
// XOR swizzle on the SOURCE offset, undone on the read: position = chunk ^ (-(row >> 2) & 3).
typedef float floatx4v __attribute__((ext_vector_type(4)));

// (window, position) of row mw + off from the wave's (w0, t0) = divmod(mw, s_in): rows of a
// tile span only a few windows, so stepping beats a 64-bit division per row.
__device__ __forceinline__ void row_wt(long long w0, int t0, int off, int s_in, long long& w, int& t) {
  t = t0 + off;
  w = w0;
  while (t >= s_in) {
    t -= s_in;
    ++w;
  }
}

template <int EPI, int FMT, int NB = 10, int MB = 4>
__device__ __forceinline__ void gemm_epilogue16(const GemmArgs& p, const floatx4v (&acc)[MB][NB], long long mw, int n0,
                                                int ks, int lane) {
  const int fr = lane & 15, fq = lane >> 4;
  const long long w0 = mw / p.s_in;
  const int t0 = (int)(mw - w0 * p.s_in);
  // the lane's per-column bias / scale, loaded together up front (clamped indices; columns past
  // n_store are skipped below) rather than one load + wait per use (see epi_factors)
  float bnv[NB], csv[NB];
  if constexpr (EPI != EPI_PARTIAL) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int n = min(n0 + nb * 16 + fr, p.n_store - 1);
      bnv[nb] = p.bias[n];
      csv[nb] = FMT == 2 ? p.col_scale[n] : 1.f;
    }
  }
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const long long m4 = mw + mb * 16 + 4 * fq;   // first of this lane's 4 rows (multiple of 4)
    if (EPI == EPI_PARTIAL) {
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const int n = n0 + nb * 16 + fr;
        if (n >= p.n_store) continue;
        float* cp = p.C + (long long)ks * p.split_stride + n;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (m4 + j < p.M) cp[(m4 + j) * p.ldc] = acc[mb][nb][j];
      }
    } else if (EPI == EPI_RELU_POOL4) {
      if (m4 >= p.M) continue;
      long long w;
      int t;
      row_wt(w0, t0, mb * 16 + 4 * fq, p.s_in, w, t);
      const int tp = t >> 2;
      if (tp >= p.t_valid) continue;
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const int n = n0 + nb * 16 + fr;
        if (n >= p.n_store) continue;
        const float bn = bnv[nb];
        // f16x3: acc * 2^-(s_in + s_w[n]) is exact (power of 2), so the value equals the unscaled sum
        const float cs = csv[nb];
        float mx = fmaxf(fmaxf(acc[mb][nb][0], acc[mb][nb][1]), fmaxf(acc[mb][nb][2], acc[mb][nb][3]));
        if (FMT == 2) mx *= cs;
        store_act<FMT>(p.C, w * p.s_out + tp, p.ldc, n, fmaxf(mx + bn, 0.f), p.out_scale, p.ovf);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const long long m = m4 + j;
        if (m >= p.M) continue;
        long long w;
        int tpos;
        row_wt(w0, t0, mb * 16 + 4 * fq + j, p.s_in, w, tpos);
        if (tpos >= p.t_valid) continue;
        const long long orow = p.c_rows ? p.c_rows[m] : (w * p.s_out + tpos);
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          const int n = n0 + nb * 16 + fr;
          if (n >= p.n_store) continue;
          const float bn = bnv[nb];
          const float cs = csv[nb];
          const float a = FMT == 2 ? acc[mb][nb][j] * cs : acc[mb][nb][j];
          const float v = a + bn;
          if (EPI == EPI_SIGMOID)
            p.C[orow * p.ldc + n] = 1.0f / (1.0f + expf(-v));
          else
            store_act<FMT>(p.C, orow, p.ldc, n, fmaxf(v, 0.f), p.out_scale, p.ovf);
        }
      }
    }
  }
}

// Products of one (16-row, 16-col, 32-deep) unit, smallest terms first, into one fp32 accumulator.
//   PL 3 (bf16x6): x = x0 + x1 + x2 (bf16), the six products of combined order <= 2;
//   PL 2 (f16x3):  x = hi + lo (fp16, operands pre-scaled), hi*hi + hi*lo + lo*hi (lo*lo, at
//                  2^-22 relative, dropped).  Every product is exact in fp32 in both forms.
template <int PL>
__device__ __forceinline__ floatx4v planes_mfma(floatx4v c, const bf16x8 (&a)[3], const bf16x8 (&b)[3]) {
  if constexpr (PL == 3) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], c, 0, 0, 0);
  } else {
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(halfx8, a[1]), __builtin_bit_cast(halfx8, b[0]), c,
                                               0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(halfx8, a[0]), __builtin_bit_cast(halfx8, b[1]), c,
                                               0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(halfx8, a[0]), __builtin_bit_cast(halfx8, b[0]), c,
                                               0, 0, 0);
  }
  return c;
}

// Body of the planes GEMM (PL operand planes per value; see beluga_gemm_x6q),
// NS-stage LDS ring: the loads of stage s + NS - 1 are in flight while stage s computes.
template <int LAYER, int EPI, int TM, int PL, int NS>
__device__ __forceinline__ void gemm_planes_body(const GemmArgs& p, char* smem) {
  static_assert(NS == 2 || (NS == 3 && PL == 2), "3-stage ring only fits the 2-plane stage in LDS");
  using G = PlaneGeo<PL>;
  constexpr int FMT = PL == 3 ? 1 : 2;
  const unsigned nblk = gridDim.x, bid = blockIdx.x;
  const unsigned xcd = bid & 7u, q = nblk >> 3, rr = nblk & 7u;
  const unsigned lin =
      p.linear_order ? bid : (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  long long mt;
  int nt, ks;
  if (p.m_fastest) {
    mt = lin % p.m_tiles;
    const long long rest = lin / p.m_tiles;
    nt = (int)(rest % p.n_tiles);
    ks = (int)(rest / p.n_tiles);
  } else {
    nt = (int)(lin % (unsigned)p.n_tiles);
    const long long rest = lin / (unsigned)p.n_tiles;
    mt = rest % p.m_tiles;
    ks = (int)(rest / p.m_tiles);
  }
  if (p.ks_mask && !((p.ks_mask[mt] >> ks) & 1u)) return;   // slab unchanged: partials already in C
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // uniform: LDS bases stay scalar
  const long long m0 = mt * X6P_BM;
  const int n0 = nt * GBN;
  const int kb_total = (int)(p.ldb / GBK);
  const int gs0 = ks * (p.kper / GBK);
  const long long lda_kb = p.lda / GBK;
  auto swz = [](int r) { return (-(r >> 2)) & 3; };
  // Sources = uniform 64-bit base + constant 32-bit lane offset (global_load_lds saddr form:
  // a stage only moves the scalar base).  FC1's row gather (a_rows) keeps 64-bit lane addresses.
  constexpr bool kGather = (LAYER == 7);
  const char* Ab = (const char*)p.A + (kGather ? 0 : m0 * lda_kb * G::ROW_KB);
  unsigned aoff[4];
  const char* aptr[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = wave * 64 + j * 16 + (lane >> 2);
    long long m = m0 + r;
    if (m > p.M - 1) m = p.M - 1;
    const int c = (lane & 3) ^ swz(r);
    if (kGather) {
      aptr[j] = (const char*)p.A + (p.a_rows ? p.a_rows[m] / GBK : m * lda_kb) * G::ROW_KB + 16 * c;
      aoff[j] = 0;
    } else {
      aptr[j] = nullptr;
      aoff[j] = (unsigned)((m - m0) * lda_kb * G::ROW_KB + 16 * c);
    }
  }
  const char* Bb = (const char*)p.Bp + ((long long)n0 * kb_total + gs0) * G::ROW_KB;
  unsigned boff[G::B_PER_WAVE];
#pragma unroll
  for (int j = 0; j < G::B_PER_WAVE; ++j) {
    const int g = min(wave + 4 * j, G::B_GROUPS - 1);
    const int pl = g / 10, r = 16 * (g % 10) + (lane >> 2);
    const int c = (lane & 3) ^ swz(r);
    boff[j] = (unsigned)((long long)r * kb_total * G::ROW_KB + pl * 64 + 16 * c);
  }
  // buffer_load ... lds: 128-bit resource from uniform values, the constant lane offset in
  // voffset and the stage offset in soffset (no per-stage vector address arithmetic)
  const __amdgpu_buffer_rsrc_t arsrc = __builtin_amdgcn_make_buffer_rsrc((void*)Ab, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t brsrc = __builtin_amdgcn_make_buffer_rsrc((void*)Bb, (short)0, 0x7fffffff, 0x00020000);
  auto issue_a = [&](int s, int buf, int i0, int ni) {
    if constexpr ((TM & 8) != 0) s = 0;
    const int gs = gs0 + s;
    const int chunk = gs / p.taps, tap = gs - chunk * p.taps;
    const long long ao = ((long long)tap * lda_kb + chunk) * G::ROW_KB;
    char* base = smem + buf * G::STAGE;
    for (int i = i0; i < i0 + ni; ++i) {
      char* dst = base + (i / 4) * X6P_A_PLANE + (wave * 4 + i % 4) * 1024;
      if (kGather)
        glds16(aptr[i % 4] + ao + (i / 4) * 64, dst);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(arsrc, (lds_void*)dst, 16, aoff[i % 4] + (i / 4) * 64, (unsigned)ao, 0,
                                                 0);
    }
  };
  auto issue_b = [&](int s, int buf, int j0, int nj) {
    if constexpr ((TM & 8) != 0) s = 0;
    char* base = smem + buf * G::STAGE + G::A_BYTES;
    for (int j = j0; j < j0 + nj; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(brsrc, (lds_void*)(base + (wave + 4 * j) * 1024), 16, boff[j],
                                               (unsigned)(s * G::ROW_KB), 0, 0);
  };

  floatx4v acc[4][10];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int nb = 0; nb < 10; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[mb][nb][r] = 0.f;

  const int fr = lane & 15, fq = lane >> 4;
  const int coff = 16 * (fq ^ swz(fr));            // swizzled chunk of this lane (row & 15 = fr)
  const int arow = (wave * 64 + fr) * 64 + coff;
  const int brow = G::A_BYTES + fr * 64 + coff;
  const int nk = p.kper / GBK;

  auto read_a = [&](const char* base, bf16x8 (&a)[4][3]) {
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
      const char* ar = base + arow + mb * 16 * 64;
#pragma unroll
      for (int pl = 0; pl < PL; ++pl) a[mb][pl] = *(const bf16x8*)(ar + pl * X6P_A_PLANE);
    }
  };
  auto read_b = [&](const char* base, int nb, bf16x8 (&b)[3]) {
    const char* br = base + brow + nb * 16 * 64;
#pragma unroll
    for (int pl = 0; pl < PL; ++pl) b[pl] = *(const bf16x8*)(br + pl * X6P_B_PLANE);
  };
  auto unit = [&](const bf16x8 (&a)[4][3], int nb, const bf16x8 (&b)[3]) {
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) acc[mb][nb] = planes_mfma<PL>(acc[mb][nb], a[mb], b);
  };
  // NM MFMAs (16 cycles each) per unit; up to 2 LDS-DMA pieces, 1 LDS read, 1 VALU per slot
  constexpr int NM = PL == 3 ? 24 : 12;
  auto pin = [&](int nv) {
#pragma unroll
    for (int i = 0; i < NM; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      if ((i % 6) == 0 && i < 6 * nv) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      if ((i & 1) == 0) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
    }
  };
  // per stage and wave: A_PIECES A pieces over the first units, then B_PER_WAVE B pieces
  constexpr int A_UNITS = G::A_PIECES / 2;          // 2 A pieces per unit: units 0 .. A_UNITS-1
  constexpr int B_PER_UNIT = (G::B_PER_WAVE + (10 - A_UNITS) - 1) / (10 - A_UNITS);

  issue_a(0, 0, 0, G::A_PIECES);
  issue_b(0, 0, 0, G::B_PER_WAVE);
  if constexpr (NS == 3) {
    issue_a(min(1, nk - 1), 1, 0, G::A_PIECES);
    issue_b(min(1, nk - 1), 1, 0, G::B_PER_WAVE);
    asm volatile("s_waitcnt vmcnt(13)" ::: "memory");   // stage 0 landed (13 = pieces per stage)
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  bf16x8 as[4][3];
  read_a(smem, as);
  int buf = 0;
  for (int s = 0; s < nk; ++s) {
    const int nbuf = buf + 1 == NS ? 0 : buf + 1;             // stage s + 1
    const int lbuf = NS == 2 ? nbuf : (nbuf + 1 == NS ? 0 : nbuf + 1);   // stage s + NS - 1
    const int sn = (TM & 2) ? s : min(s + NS - 1, nk - 1);
    const char* base = smem + buf * G::STAGE;
    const char* nbase = smem + nbuf * G::STAGE;
    const bool go = !(TM & 2);
    bf16x8 b0[3], b1[3];
    read_b(base, 0, b0);
#pragma unroll
    for (int nb = 0; nb < 10; ++nb) {
      int nv = 0;
      if (go && nb < A_UNITS) {
        issue_a(sn, lbuf, 2 * nb, 2);
        nv = 2;
      }
      if (go && nb >= A_UNITS) {
        const int j0 = (nb - A_UNITS) * B_PER_UNIT;
        const int nj = min(B_PER_UNIT, G::B_PER_WAVE - j0);
        if (nj > 0) {
          issue_b(sn, lbuf, j0, nj);
          nv = nj;
        }
      }
      if (nb + 1 < 10) read_b(base, nb + 1, (nb & 1) ? b0 : b1);
      unit(as, nb, (nb & 1) ? b1 : b0);
      pin(nv);
    }
    // A of stage s+1 (this wave's A pieces, older than its B pieces) replaces A(s) while the
    // last unit's MFMAs drain
    if constexpr (!(TM & 2)) {
      if constexpr (NS == 3)
        asm volatile("s_waitcnt vmcnt(13)" ::: "memory");   // all of stage s+1 (s+2 in flight)
      else if constexpr (G::B_PER_WAVE == 8)
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    }
    read_a(nbase, as);
    if constexpr (!(TM & 4)) {
      if constexpr (NS == 3)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    asm volatile("" ::: "memory");
    buf = nbuf;
  }
  gemm_epilogue16<EPI, FMT>(p, acc, m0 + wave * 64, n0, ks, lane);
}

// ---- f16x3 FC GEMM, producer / consumer waves ---------------------------------------------
// Tile 256 rows x 160 columns, 4 MFMA waves of 64 rows, with both operands staged through an
// LDS ring by 4 producer waves (one per SIMD beside its MFMA wave), so the MFMA waves issue only
// ds_reads and MFMAs.  A stage = one 32-deep K block: A 256 rows x 2 planes (32 pieces,
// per-lane 64-bit sources: a_rows gathers windows from anywhere in the activation buffer) + B
// 160 columns x 2 planes (20 pieces); 3 stages = 156 KB.  (A variant loading each wave's A
// fragments straight into registers, tools/gemm_probes.h beluga_fc_h3, ran 431 vs 356
// fp32-equivalent TF/s at 2000 rows.)  Same operands, products and k order per output as the
// planes GEMM: bitwise equal.
constexpr int H3E_ROW = 656;
constexpr int H3E_WAVE = 32 * H3E_ROW;                 // 20,992 B per wave

// Split-K partial epilogue through LDS: a wave's 64 x 160 fp32 tile is, per row, one contiguous
// 640-B run of the partial slab (row stride ldc).  The accumulator layout scatters it over 4-B
// pieces (16 lanes = 64 B per store); staged per 32-row half in the wave's LDS area (row stride
// H3E_ROW = 656 B: the 4 row groups of a ds_write_b32 land on distinct banks), it leaves as
// 16-B stores, 40 per row.  Same values and addresses as gemm_epilogue16<EPI_PARTIAL>.
__device__ __forceinline__ void epilogue_partial_lds(const GemmArgs& p, const floatx4v (&acc)[4][10], long long mw,
                                                     int n0, int ks, int lane, char* lds) {
  const int fr = lane & 15, fq = lane >> 4;
  float* const cbase = p.C + (long long)ks * p.split_stride;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
#pragma unroll
    for (int nb = 0; nb < 10; ++nb)
#pragma unroll
      for (int mh = 0; mh < 2; ++mh)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          *(float*)(lds + (mh * 16 + 4 * fq + j) * H3E_ROW + (nb * 16 + fr) * 4) = acc[2 * half + mh][nb][j];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll 4
    for (int i = 0; i < 20; ++i) {
      const int k = i * 64 + lane, row = k / 40, ch = k - row * 40;
      const long long m = mw + half * 32 + row;
      if (m < p.M && n0 + 4 * ch < p.n_store)
        *(floatx4v*)(cbase + m * p.ldc + n0 + 4 * ch) = *(const floatx4v*)(lds + row * H3E_ROW + ch * 16);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

constexpr int FCP_APLANE = 256 * 64;                   // 16 KB
constexpr int FCP_STAGE = 2 * FCP_APLANE + 2 * X6P_B_PLANE;   // 52 KB

template <int LAYER, int EPI, int TM, int NS>
__device__ __forceinline__ void gemm_fc_h3p_body(const GemmArgs& p, char* smem) {
  static_assert(NS == 3 || NS == 4, "ring depth");
  // PF: producers wait for ALL their pieces at each stage end (stage s+NS-1 landed at barrier s),
  // so the consumers read stage s+1's first fragments before barrier s and start it without an
  // LDS round trip; the loads get one stage less to land.
  constexpr bool PF = (TM & 256) != 0;
  constexpr int ROW_KB = 128;
  const unsigned nblk = gridDim.x, bid = blockIdx.x;
  const unsigned xcd = bid & 7u, q = nblk >> 3, rr = nblk & 7u;
  const unsigned lin =
      p.linear_order ? bid : (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  long long mt;
  int nt, ks;
  if (p.m_fastest == 2) {
    // split-K slab outermost over the whole chip (all XCDs sweep one weight slab together, so it
    // is read from HBM once and shared through the Infinity Cache), and within a slab XCD x owns
    // the M tiles mt = x mod 8, running each one's N tiles back to back (its A rows stay in the
    // XCD's L2).  Needs m_tiles % 8 == 0 (the host checks).
    const long long per_ks = p.m_tiles * p.n_tiles;
    ks = (int)(bid / per_ks);
    const unsigned j = (unsigned)((bid - ks * per_ks) >> 3);
    mt = (long long)(j / (unsigned)p.n_tiles) * 8 + (bid & 7u);
    nt = (int)(j % (unsigned)p.n_tiles);
  } else if (p.m_fastest == 3) {
    // grouped: per split-K slab, groups of m_group M tiles; inside a group N tiles outer and M
    // tiles inner, so the ~32 workgroups an XCD runs at once (the XCD remap keeps lin
    // contiguous per XCD) cover ~m_group M tiles x 32/m_group N tiles: a weight tile is read
    // by m_group concurrent M tiles instead of ~2.5 (N tiles fastest), an activation tile by
    // 32/m_group N tiles instead of all 13
    const long long per_ks = p.m_tiles * p.n_tiles;
    ks = (int)(lin / per_ks);
    const long long r = lin - ks * per_ks;
    const long long g = r / ((long long)p.m_group * p.n_tiles);
    const int i = (int)(r - g * p.m_group * p.n_tiles);
    const int gm = (int)min((long long)p.m_group, p.m_tiles - g * p.m_group);
    nt = i / gm;
    mt = g * p.m_group + i % gm;
  } else if (p.m_fastest) {
    mt = lin % p.m_tiles;
    const long long rest = lin / p.m_tiles;
    nt = (int)(rest % p.n_tiles);
    ks = (int)(rest / p.n_tiles);
  } else {
    nt = (int)(lin % (unsigned)p.n_tiles);
    const long long rest = lin / (unsigned)p.n_tiles;
    mt = rest % p.m_tiles;
    ks = (int)(rest / p.m_tiles);
  }
  if (p.ks_mask && !((p.ks_mask[mt] >> ks) & 1u)) return;   // slab unchanged: partials already in C
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const long long m0 = mt * X6P_BM;
  const int n0 = nt * GBN;
  const int kb_total = (int)(p.ldb / GBK);
  const int gs0 = ks * (p.kper / GBK);
  const long long lda_kb = p.lda / GBK;
  const int nk = p.kper / GBK;
  auto swz = [](int r) { return (-(r >> 2)) & 3; };

  if (wave >= 4) {
    // ---------------- producer ----------------
    const int pw = wave - 4;
    // A pieces P = pw + 4*i (i < 8) of 32: plane P & 1, rows 16*(P >> 1) + (lane >> 2)
    const char* asrc[8];
    unsigned adst[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int P = pw + 4 * i, g = P >> 1, pl = P & 1;
      const int r = 16 * g + (lane >> 2);
      long long m = m0 + r;
      if (m > p.M - 1) m = p.M - 1;
      const long long kb0 = (p.a_rows ? p.a_rows[m] / GBK : m * lda_kb) + gs0;
      const int c = (lane & 3) ^ swz(r);
      asrc[i] = (const char*)p.A + kb0 * ROW_KB + pl * 64 + 16 * c;
      adst[i] = (unsigned)(pl * FCP_APLANE + g * 1024);
    }
    const char* Bb = (const char*)p.Bp + ((long long)n0 * kb_total + gs0) * ROW_KB;
    unsigned boff[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const int g = pw + 4 * j;
      const int pl = g / 10, r = 16 * (g % 10) + (lane >> 2);
      const int c = (lane & 3) ^ swz(r);
      boff[j] = (unsigned)((long long)r * kb_total * ROW_KB + pl * 64 + 16 * c);
    }
    const __amdgpu_buffer_rsrc_t brsrc = __builtin_amdgcn_make_buffer_rsrc((void*)Bb, (short)0, 0x7fffffff, 0x00020000);
    auto issue = [&](int s, int slot) {
      if constexpr ((TM & 8) != 0) s = 0;
      // probes (tools/gemm_bench): 16 = A pieces always from stage 0 (L2-hot A), 32 = B hot
      const int sa = (TM & 16) ? 0 : s, sb = (TM & 32) ? 0 : s;
      char* base = smem + slot * FCP_STAGE;
#pragma unroll
      for (int i = 0; i < 8; ++i) glds16(asrc[i] + (long long)sa * ROW_KB, base + adst[i]);
#pragma unroll
      for (int j = 0; j < 5; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(brsrc, (lds_void*)(base + 2 * FCP_APLANE + (pw + 4 * j) * 1024), 16,
                                                 boff[j], (unsigned)(sb * ROW_KB), 0, 0);
    };
    for (int s = 0; s < NS - 1; ++s) issue(min(s, nk - 1), s);
    if constexpr (PF)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (NS == 3)
      asm volatile("s_waitcnt vmcnt(13)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(26)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    int slot = 0;
    for (int s = 0; s < nk; ++s) {
      const int lslot = slot == 0 ? NS - 1 : slot - 1;   // stage s+NS-1 goes where s-1 was
      if (!(TM & 2)) issue(min(s + NS - 1, nk - 1), lslot);
      // all but the pieces of the last NS-2 stages: stage s+1 landed (PF: all of them)
      if constexpr (PF)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else if constexpr (NS == 3)
        asm volatile("s_waitcnt vmcnt(13)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(26)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      slot = slot + 1 == NS ? 0 : slot + 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (EPI == EPI_PARTIAL)
      __builtin_amdgcn_s_barrier();   // tail pieces landed: the consumers' epilogue reuses the LDS
    return;
  }

  // ---------------- consumer ----------------
  floatx4v acc[4][10];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int nb = 0; nb < 10; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[mb][nb][r] = 0.f;
  const int fr = lane & 15, fq = lane >> 4;
  const int brow = fr * 64 + 16 * (fq ^ swz(fr));
  const int arow = (wave * 64 + fr) * 64 + 16 * (fq ^ swz(fr));   // swz(wave*64 + mb*16 + fr) = swz(fr)
  auto read_a = [&](const char* base, bf16x8 (&a)[4][3]) {
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
      a[mb][0] = *(const bf16x8*)(base + arow + mb * 1024);
      a[mb][1] = *(const bf16x8*)(base + arow + mb * 1024 + FCP_APLANE);
    }
  };
  auto read_b = [&](const char* base, int nb, bf16x8 (&b)[3]) {
    const char* br = base + 2 * FCP_APLANE + brow + nb * 1024;
    b[0] = *(const bf16x8*)(br);
    b[1] = *(const bf16x8*)(br + X6P_B_PLANE);
  };
  auto pin = [&]() {
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      if ((i & 1) == 0) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
    }
  };
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  bf16x8 as[4][3];
  bf16x8 b0[3], b1[3];
  if constexpr (PF) {
    read_b(smem, 0, b0);
    read_a(smem, as);
  }
  int slot = 0;
  for (int s = 0; s < nk; ++s) {
    const char* base = smem + slot * FCP_STAGE;
    const int nslot = slot + 1 == NS ? 0 : slot + 1;
    // the stage's first B fragment, then its A fragments in MFMA order: the first MFMAs wait for
    // 4 reads, not 10 (round 1 read A first)
    if constexpr (!PF) {
      read_b(base, 0, b0);
      read_a(base, as);
    }
#pragma unroll
    for (int nb = 0; nb < 10; ++nb) {
      if (nb + 1 < 10) read_b(base, nb + 1, (nb & 1) ? b0 : b1);
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) acc[mb][nb] = planes_mfma<2>(acc[mb][nb], as[mb], (nb & 1) ? b1 : b0);
      pin();
    }
    if constexpr (PF) {
      if (s + 1 < nk) {   // stage s+1 landed at barrier s-1
        read_b(smem + nslot * FCP_STAGE, 0, b0);
        read_a(smem + nslot * FCP_STAGE, as);
      }
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    slot = nslot;
  }
  if constexpr (EPI == EPI_PARTIAL) {
    __builtin_amdgcn_s_barrier();   // producers drained their tail pieces
    epilogue_partial_lds(p, acc, m0 + wave * 64, n0, ks, lane, smem + wave * H3E_WAVE);
  } else {
    gemm_epilogue16<EPI, 2, 10, 4>(p, acc, m0 + wave * 64, n0, ks, lane);
  }
}

template <int LAYER, int EPI, int TM = 0, int NS = 3>
__global__ __launch_bounds__(512, 1) void beluga_fc_h3p(GemmArgs p) {
  __shared__ __attribute__((aligned(1024))) char smem[NS * FCP_STAGE];
  gemm_fc_h3p_body<LAYER, EPI, TM, NS>(p, smem);
}

// ---- f16x3 FC GEMM, wide tiles: 256 rows x 336 columns, 8 MFMA waves ----------------------
// In the FC1 launch every weight (B) tile is re-fetched from beyond L2 once per ~2.5 M tiles an
// XCD runs at once (tools/gemm_bench fc1, 8192 rows: 7 of 10 GB of FETCH per launch are B; B
// served L2-hot ran 8.6 % faster, A L2-hot 4.4 %).  A 336-column tile (6 of them cover FC1's
// 2016 padded outputs with 0.6 % padding) holds twice the outputs per workgroup, so per MFMA it
// stages half the bytes, and an XCD's 32 concurrent workgroups cover ~5.3 M tiles x all 6 N
// tiles: each weight tile is read by 5.3 concurrent M tiles instead of 2.5.
// 8 waves, all MFMA (two per SIMD, 168 accumulators each): wave w owns rows 32w..32w+31 and all
// 21 column blocks.  A stage = one 32-deep K block: A 256 rows x 2 planes (32 LDS-DMA pieces of
// 1 KiB, per-lane 64-bit sources: a_rows gathers) + B 336 columns x 2 planes (42 pieces); every
// wave issues 4 A + 6 B pieces per stage (waves 2-7 repeat B piece 41: identical bytes to the
// same LDS address), one per MFMA unit, for the NEXT stage into the other half of a 2-stage
// ring (2 x 75,776 B), waits for its own pieces at the stage end and meets the others at one
// barrier per stage.  Epilogue (split-K partial slabs) staged per wave through LDS in 16-row x
// 176/160-column passes.  Same operands, products and k order per output as beluga_fc_h3p:
// bitwise equal.
constexpr int FCW_NB = 21;                             // 16-column blocks per tile
constexpr int FCW_BN = 16 * FCW_NB;                    // 336
constexpr int FCW_APLANE = 256 * 64;                   // 16 KB
constexpr int FCW_BPLANE = FCW_NB * 1024;              // 21 KB
constexpr int FCW_STAGE = 2 * FCW_APLANE + 2 * FCW_BPLANE;   // 75,776 B
constexpr int FCW_EROW = 176 * 4 + 16;                 // epilogue staging row stride (720 B)
constexpr int FCW_EWAVE = 16 * FCW_EROW;               // 11,520 B per wave

// s_waitcnt vmcnt(N) for compile-time piece counts (conv producers, the 3-stage FC ring)
template <int N>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N == 2)
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 4)
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 5)
    asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  else if constexpr (N == 10)
    asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  else
    static_assert(N == 2, "vmcnt value");
}

// One 256 x (16 NB) split-K partial tile of the wide FC GEMM: A row m (< M) starts at element
// (a_rows ? a_rows[m] + a_off : m * 32 * lda_kb) of A and is read for nk 32-deep K blocks from
// K block kb0; Bb = the weight planes of column n0 at the same first K block (kb_total K blocks
// per weight row); the fp32 partial row m goes to cbase + m * ldc (columns < n_store).  Shared by
// beluga_fc_h3w (one split-K GEMM) and beluga_fc_h3k (a group of GEMMs in one launch): the same
// pieces, products and k order per output.  NB = 21 (336 columns) everywhere but the grouped FC1 of
// small batches, which takes NB = 7 (112 columns, 3x the workgroups; fc_narrow in beluga.hip): an
// output's products and k order do not depend on the tile width, so both give the same bits.  A wave
// whose 32 rows all lie past M skips its MFMAs and fragment reads (it still issues its LDS-DMA
// pieces and meets every barrier): in a part-filled M tile the live waves then have their SIMDs
// to themselves.
template <int NB>
struct FcwGeo {
  static constexpr int BPLANE = NB * 1024;
  static constexpr int STAGE = 2 * FCW_APLANE + 2 * BPLANE;
  static constexpr int JB = (2 * NB + 7) / 8;           // B pieces per wave and stage
  static constexpr int NP = 4 + JB;                     // LDS-DMA pieces per wave and stage
  static_assert(2 * STAGE >= 8 * FCW_EWAVE, "epilogue staging inside the stage ring");
};

template <int TM, int NB = FCW_NB, int NS = 2>
__device__ __forceinline__ void fc_h3w_tile(const float* A, const long long* a_rows, long long a_off, long long lda_kb,
                                            int kb0a, long long M, const char* Bb, int kb_total, int nk, float* cbase,
                                            long long ldc, int n_store, long long m0, int n0, char* smem) {
  using G = FcwGeo<NB>;
  constexpr int ROW_KB = 128;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  auto swz = [](int r) { return (-(r >> 2)) & 3; };
  // this wave's LDS-DMA pieces: A pieces P = wave + 8i (i < 4) of 32 (plane P & 1, rows
  // 16 (P >> 1) ..), B pieces Q = min(wave + 8j, 2 NB - 1) (j < JB) of 2 NB (plane Q / NB, cols
  // 16 (Q % NB) ..)
  const char* asrc[4];
  unsigned adst[4];
  unsigned alive = 0;   // bit i: A piece i holds a row < M (a row group past M feeds only skipping waves)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int P = wave + 8 * i, g = P >> 1, pl = P & 1;
    if (m0 + 16 * g < M) alive |= 1u << i;
    const int r = 16 * g + (lane >> 2);
    long long m = m0 + r;
    if (m > M - 1) m = M - 1;
    const long long kb0 = (a_rows ? (a_rows[m] + a_off) / GBK : m * lda_kb) + kb0a;
    const int c = (lane & 3) ^ swz(r);
    asrc[i] = (const char*)A + kb0 * ROW_KB + pl * 64 + 16 * c;
    adst[i] = (unsigned)(pl * FCW_APLANE + g * 1024);
  }
  static_assert(G::JB <= 6, "B pieces per wave");
  unsigned boff[6], bdst[6];   // (a dependent bound here fails the host pass of hipcc's lambdas)
#pragma unroll
  for (int j = 0; j < G::JB; ++j) {
    const int Q = min(wave + 8 * j, 2 * NB - 1);
    const int pl = Q / NB, r = 16 * (Q % NB) + (lane >> 2);
    const int c = (lane & 3) ^ swz(r);
    boff[j] = (unsigned)((long long)r * kb_total * ROW_KB + pl * 64 + 16 * c);
    bdst[j] = (unsigned)(2 * FCW_APLANE + Q * 1024);
  }
  const __amdgpu_buffer_rsrc_t brsrc = __builtin_amdgcn_make_buffer_rsrc((void*)Bb, (short)0, 0x7fffffff, 0x00020000);
  auto issue_piece = [&](int s, char* base, int k) {   // piece k < NP of stage s: 0-3 A, then B
    if constexpr ((TM & 8) != 0) s = 0;
    if (k < 4) {
      // (the narrow tiles of small batches only: the wide kernel's schedule stays branch-free)
      if (NB == FCW_NB || ((alive >> k) & 1u))
        glds16(asrc[k] + (long long)((TM & 16) ? 0 : s) * ROW_KB, base + adst[k]);
    } else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(brsrc, (lds_void*)(base + bdst[k - 4]), 16, boff[k - 4],
                                               (unsigned)(((TM & 32) ? 0 : s) * ROW_KB), 0, 0);
  };

  floatx4v acc[2][NB];
#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[mb][nb][r] = 0.f;
  const int fr = lane & 15, fq = lane >> 4;
  const int brow = 2 * FCW_APLANE + fr * 64 + 16 * (fq ^ swz(fr));
  const int arow = (wave * 32 + fr) * 64 + 16 * (fq ^ swz(fr));   // swz(wave*32 + mb*16 + fr) = swz(fr)
  auto read_a = [&](const char* base, bf16x8 (&a)[2][3]) {
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
      a[mb][0] = *(const bf16x8*)(base + arow + mb * 1024);
      a[mb][1] = *(const bf16x8*)(base + arow + mb * 1024 + FCW_APLANE);
    }
  };
  auto read_b = [&](const char* base, int nb, bf16x8 (&b)[3]) {
    const char* br = base + brow + nb * 1024;
    b[0] = *(const bf16x8*)(br);
    b[1] = *(const bf16x8*)(br + G::BPLANE);
  };
  auto pin = [&](int nv) {   // one unit: 6 MFMAs, <= 1 LDS-DMA piece, the next unit's 2 B reads
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      if (i == 0 && nv) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      if (i < 2) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
    }
  };
  // NS stages in the ring: 2 (the wide tiles: 2 x 75,776 B), or 3 for the narrow tiles (3 x 47,104
  // B), whose part-filled M tiles leave a stage's loads less compute to hide behind (one live wave
  // per CU at batch 32).  Pieces of stage s + NS - 1 are issued during stage s; at its end a wave
  // waits until only those are outstanding (npw of them: its B pieces and its A pieces of live row
  // groups), i.e. for stage s + 1.
  static_assert(NS == 2 || NS == 3, "FC ring depth");
  static_assert(NS * G::STAGE <= 160 * 1024, "FC ring in LDS");
  static_assert(NS == 2 || NB != FCW_NB, "3-stage ring: narrow tiles (A pieces of dead row groups skipped)");
  constexpr int LOOK = NS - 1;
  const int npw = __builtin_popcount(alive) + G::JB;   // wave-uniform
  auto stage_end_wait = [&]() {
    if constexpr (NS == 2) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's pieces of stage s+1 landed
    } else {
      static_assert(G::JB == 2, "vmcnt cases");
      switch (npw) {
        case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
      }
    }
  };
  // prologue: stages 0 .. LOOK-1
#pragma unroll
  for (int st = 0; st < LOOK; ++st)
#pragma unroll
    for (int k = 0; k < G::NP; ++k) issue_piece(min(st, nk - 1), smem + st * G::STAGE, k);
  stage_end_wait();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  bf16x8 as[2][3];
  bf16x8 b0[3], b1[3];
  const bool live = m0 + 32 * wave < M;   // wave-uniform: some of this wave's rows are real
  if (live) {
    for (int s = 0; s < nk; ++s) {
      const char* base = smem + (s % NS) * G::STAGE;
      char* nbase = smem + ((s + LOOK) % NS) * G::STAGE;
      // the next stage's pieces are issued unconditionally (the last stages re-fetch the last K
      // block into the free buffer, drained before the epilogue): a runtime `more` test compiled to
      // a branch around every piece, and the block boundaries made the LDS-read waits lgkmcnt(0)
      const int s_next = min(s + LOOK, nk - 1);
      constexpr bool more = !(TM & 2);
      read_b(base, 0, b0);
      read_a(base, as);
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const int k = nb * G::NP / NB;                  // units spread the NP pieces
        const bool issue = more && (nb * G::NP % NB) < G::NP;
        if (issue) issue_piece(s_next, nbase, k);
        if (nb + 1 < NB) read_b(base, nb + 1, (nb & 1) ? b0 : b1);
        // nothing crosses this point: the next unit's fragment reads stay ahead of this unit's
        // MFMAs in their own registers.  Without it the scheduler (minimising registers) read
        // every fragment right before its MFMA into the previous unit's registers, and the
        // lgkmcnt(0) before each use exposed the full LDS latency (gemm_bench fc1 8192 rows:
        // 499 vs 474 fp32-eq TF/s; without LDS-DMA 630 vs 533)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int mb = 0; mb < 2; ++mb) acc[mb][nb] = planes_mfma<2>(acc[mb][nb], as[mb], (nb & 1) ? b1 : b0);
        pin(issue ? 1 : 0);
      }
      stage_end_wait();
      __builtin_amdgcn_s_barrier();                      // everyone's, and stage s fully read
      asm volatile("" ::: "memory");
    }
  } else {   // rows all past M: this wave's share of the pieces and the barriers only
    for (int s = 0; s < nk; ++s) {
      char* nbase = smem + ((s + LOOK) % NS) * G::STAGE;
      const int s_next = min(s + LOOK, nk - 1);
      if constexpr (!(TM & 2)) {
#pragma unroll
        for (int k = 0; k < G::NP; ++k) issue_piece(s_next, nbase, k);
      }
      stage_end_wait();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
  }
  if constexpr (NS > 2) {   // the last re-fetches still in flight: drained before the LDS is reused
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  if (!live) return;   // no stores: every row of this wave is >= M
  // split-K partial epilogue: 16-row x (176 | 160)-column passes through the wave's LDS area
  char* const lds = smem + wave * FCW_EWAVE;
#pragma unroll
  for (int mb = 0; mb < 2; ++mb) {
#pragma unroll
    for (int h = 0; h < (NB > 11 ? 2 : 1); ++h) {
      const int nb0 = h ? 11 : 0, nbn = NB > 11 ? (h == 0 ? 11 : NB - 11) : NB, cols = 16 * nbn;
#pragma unroll
      for (int nb = 0; nb < 11; ++nb) {
        if (nb >= nbn) break;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          *(float*)(lds + (4 * fq + j) * FCW_EROW + (nb * 16 + fr) * 4) = acc[mb][nb0 + nb][j];
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const int chunks = cols / 4;                      // 16-B chunks per row (44 | 40 | 28)
      for (int i = lane; i < 16 * chunks; i += 64) {
        const int row = i / chunks, ch = i - row * chunks;
        const long long m = m0 + wave * 32 + mb * 16 + row;
        const int n = n0 + nb0 * 16 + 4 * ch;
        if (m < M && n < n_store)
          *(floatx4v*)(cbase + m * ldc + n) = *(const floatx4v*)(lds + row * FCW_EROW + ch * 16);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
}

template <int LAYER, int EPI, int TM, int NB = FCW_NB, int NS = 2>
__device__ __forceinline__ void gemm_fc_h3w_body(const GemmArgs& p, char* smem) {
  static_assert(EPI == EPI_PARTIAL, "split-K partial slabs only");
  const unsigned nblk = gridDim.x, bid = blockIdx.x;
  const unsigned xcd = bid & 7u, q = nblk >> 3, rr = nblk & 7u;
  const unsigned lin =
      p.linear_order ? bid : (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  long long mt;
  int nt, ks;
  if (p.m_fastest == 3) {
    const long long per_ks = p.m_tiles * p.n_tiles;
    ks = (int)(lin / per_ks);
    const long long r = lin - ks * per_ks;
    const long long g = r / ((long long)p.m_group * p.n_tiles);
    const int i = (int)(r - g * p.m_group * p.n_tiles);
    const int gm = (int)min((long long)p.m_group, p.m_tiles - g * p.m_group);
    nt = i / gm;
    mt = g * p.m_group + i % gm;
  } else if (p.m_fastest) {
    mt = lin % p.m_tiles;
    const long long rest = lin / p.m_tiles;
    nt = (int)(rest % p.n_tiles);
    ks = (int)(rest / p.n_tiles);
  } else {
    nt = (int)(lin % (unsigned)p.n_tiles);
    const long long rest = lin / (unsigned)p.n_tiles;
    mt = rest % p.m_tiles;
    ks = (int)(rest / p.m_tiles);
  }
  if (p.ks_mask && !((p.ks_mask[mt] >> ks) & 1u)) return;   // slab unchanged: partials already in C
  const long long m0 = mt * X6P_BM;
  const int n0 = nt * 16 * NB;
  const int kb_total = (int)(p.ldb / GBK);
  const int gs0 = ks * (p.kper / GBK);
  constexpr int ROW_KB = 128;
  fc_h3w_tile<TM, NB, NS>(p.A, p.a_rows, 0, p.lda / GBK, gs0, p.M, (const char*)p.Bp + ((long long)n0 * kb_total + gs0) * ROW_KB,
                  kb_total, p.kper / GBK, p.C + (long long)ks * p.split_stride, p.ldc, p.n_store, m0, n0, smem);
}

template <int LAYER, int EPI, int TM = 0>
__global__ __launch_bounds__(512, 1) void beluga_fc_h3w(GemmArgs p) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * FCW_STAGE];
  gemm_fc_h3w_body<LAYER, EPI, TM>(p, smem);
}

// the same split-K GEMM on 112-column tiles and a 3-stage ring (the direct FC1 / FC2 of small
// per-window batches: 3x the workgroups at a third of the work each; an output's products and k
// order do not depend on the tile width, so the same bits)
template <int LAYER, int EPI>
__global__ __launch_bounds__(512, 1) void beluga_fc_h3w_narrow(GemmArgs p) {
  __shared__ __attribute__((aligned(1024))) char smem[3 * FcwGeo<7>::STAGE];
  gemm_fc_h3w_body<LAYER, EPI, 0, 7, 3>(p, smem);
}

// The same split-K GEMM for batches of <= 32 rows (the reference's per-window batch of 32): a
// weight stream with almost no MFMA work per byte, so the time is how many bytes each CU keeps in
// flight.  The 256-row tiles above stage 32 KB of A planes per K block for 32 live rows and run a
// 3-stage ring on 144 workgroups (FC1: 160 us, 3.4 TB/s of weights); here a tile is 32 rows x 16 NB
// columns, a stage (A 32 rows + B 16 NB columns, two planes each) 4 + 2 NB KB and the ring NS
// stages deep: NB 2, NS 9 = FC1 in 504 workgroups, two per CU, 128 KB of pieces in flight per CU
// (125 us; NB 3, NS 7: 336 workgroups, 145 us).  The wait for a stage is the memory latency over
// the ring depth: the weights arrive at ~35 GB/s per CU either way.  2 NB waves, one 16 x 16 output block each (rows 16 (w / NB), columns 16 (w % NB)):
// the same pieces, swizzle, fragments, products and k order per output as fc_h3w_tile -- the same
// bits.
template <int NB>
struct FcsGeo {
  static constexpr int APLANE = 32 * 64;                 // 2 KB
  static constexpr int BPLANE = NB * 1024;
  static constexpr int STAGE = 2 * APLANE + 2 * BPLANE;
  static constexpr int WAVES = 2 * NB;
  static constexpr int PIECES = 4 + 2 * NB;              // 4 A, then 2 NB B pieces per stage
};
constexpr int FCS_NB = 2;   // 32 columns: FC1 63 N tiles x 8 slabs = 504 workgroups, two per CU
constexpr int FCS_NS = 9;   // ring stages (2 x 9 x 8 KB of LDS per CU)
template <int N>
__device__ __forceinline__ void wait_vmn() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int LAYER, int EPI, int NB = FCS_NB, int NS = FCS_NS>
__global__ __launch_bounds__(64 * 2 * NB, 2) void beluga_fc_h3s(GemmArgs p) {
  static_assert(EPI == EPI_PARTIAL, "split-K partial slabs only");
  using G = FcsGeo<NB>;
  static_assert(2 * NS * G::STAGE <= 160 * 1024, "two workgroups per CU");
  __shared__ __attribute__((aligned(1024))) char smem[NS * G::STAGE];
  constexpr int ROW_KB = 128;
  constexpr int LOOK = NS - 1;
  // N tiles fastest: the tiles of a slab share its A rows
  const int nt = (int)(blockIdx.x % (unsigned)p.n_tiles), ks = (int)(blockIdx.x / (unsigned)p.n_tiles);
  const int n0 = nt * 16 * NB;
  const int kb_total = (int)(p.ldb / GBK), nk = (int)(p.kper / GBK), kb0a = ks * nk;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int mb = wave / NB, nb = wave % NB;
  auto swz = [](int r) { return (-(r >> 2)) & 3; };
  // wave w issues pieces w and w + WAVES (if any): piece k < 4 is A piece k (plane k & 1, rows
  // 16 (k >> 1) ..), piece k >= 4 B piece Q = k - 4 (plane Q / NB, columns 16 (Q % NB) ..)
  const char* gsrc[2] = {nullptr, nullptr};   // A pieces: global source
  unsigned boff[2] = {0, 0}, dst[2] = {0, 0};
  bool isa[2] = {false, false};
  constexpr int NPW1 = G::PIECES > G::WAVES ? 1 : 0;   // waves with a second piece: w < PIECES - WAVES
  const int npw = 1 + (wave < G::PIECES - G::WAVES ? 1 : 0);
#pragma unroll
  for (int i = 0; i < 1 + NPW1; ++i) {
    const int k = wave + i * G::WAVES;
    if (k >= G::PIECES) break;
    if (k < 4) {
      const int g = k >> 1, pl = k & 1, r = 16 * g + (lane >> 2);
      const long long m = min((long long)r, p.M - 1);
      const long long kb0 = (p.a_rows ? p.a_rows[m] / GBK : m * (p.lda / GBK)) + kb0a;
      gsrc[i] = (const char*)p.A + kb0 * ROW_KB + pl * 64 + 16 * ((lane & 3) ^ swz(r));
      dst[i] = (unsigned)(pl * G::APLANE + g * 1024);
      isa[i] = true;
    } else {
      const int Q = k - 4, pl = Q / NB, r = 16 * (Q % NB) + (lane >> 2);
      boff[i] = (unsigned)((long long)r * kb_total * ROW_KB + pl * 64 + 16 * ((lane & 3) ^ swz(r)));
      dst[i] = (unsigned)(2 * G::APLANE + Q * 1024);
    }
  }
  const __amdgpu_buffer_rsrc_t brsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((const char*)p.Bp + ((long long)n0 * kb_total + kb0a) * ROW_KB), (short)0, 0x7fffffff, 0x00020000);
  auto issue = [&](int s, char* base) {   // this wave's pieces of stage s (wave-uniform branches)
#pragma unroll
    for (int i = 0; i < 1 + NPW1; ++i) {
      if (i == 1 && npw == 1) break;
      if (isa[i])
        glds16(gsrc[i] + (long long)s * ROW_KB, base + dst[i]);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(brsrc, (lds_void*)(base + dst[i]), 16, boff[i], (unsigned)(s * ROW_KB),
                                                 0, 0);
    }
  };
  // at a stage end a wave waits until only its pieces of the LOOK - 1 later stages are in flight
  auto stage_end_wait = [&]() {
    if (npw == 2)
      wait_vmn<2 * (LOOK - 1)>();
    else
      wait_vmn<LOOK - 1>();
  };
#pragma unroll
  for (int st = 0; st < LOOK; ++st) issue(min(st, nk - 1), smem + st * G::STAGE);
  stage_end_wait();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  const bool live = 16 * mb < p.M;   // wave-uniform
  const int fr = lane & 15, fq = lane >> 4;
  const int arow = (mb * 16 + fr) * 64 + 16 * (fq ^ swz(fr));
  const int brow = 2 * G::APLANE + nb * 1024 + fr * 64 + 16 * (fq ^ swz(fr));
  floatx4v acc = {0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < nk; ++s) {
    const char* base = smem + (s % NS) * G::STAGE;
    issue(min(s + LOOK, nk - 1), smem + ((s + LOOK) % NS) * G::STAGE);   // (the last re-fetch the last block)
    if (live) {
      bf16x8 a[3], b[3];
      a[0] = *(const bf16x8*)(base + arow);
      a[1] = *(const bf16x8*)(base + arow + G::APLANE);
      b[0] = *(const bf16x8*)(base + brow);
      b[1] = *(const bf16x8*)(base + brow + G::BPLANE);
      acc = planes_mfma<2>(acc, a, b);
    }
    stage_end_wait();
    __builtin_amdgcn_s_barrier();   // everyone's pieces of stage s + 1 landed, stage s fully read
    asm volatile("" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the re-fetches, before the workgroup's LDS is released
  if (!live) return;
  const int n = n0 + nb * 16 + fr;
  if (n >= p.n_store) return;
  float* cp = p.C + (long long)ks * p.split_stride + n;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const long long m = mb * 16 + 4 * fq + j;
    if (m < p.M) cp[m * p.ldc] = acc[j];
  }
}

// ---- grouped wide FC GEMM: several split-K partial GEMMs in one launch ----------------------
// FC1's block Karatsuba (beluga.hip, "FC1 as a block-Karatsuba convolution") runs up to 9
// products x 2 K slabs + the tail per window group as separate GEMMs with their own A rows,
// weight planes and partial rows; one launch over all of them fills the chip's rounds as one
// GEMM would (the r04 probe ran them as 4 launches and lost most of the saving to part-filled
// rounds).  Descriptor d covers launch blocks [blk0, blk0 + m_tiles * n_tiles), N tiles fastest
// (the 6 N tiles of an M tile run together; an XCD's ~32 concurrent workgroups share ~5 M tiles'
// weight tiles, as beluga_fc_h3w's N-fastest order).
constexpr int FCK_MAX = 24;
struct FcDesc {
  const float* A;            // activation rows (f16x3 planes)
  const long long* a_rows;   // element offset of each of the M rows
  long long a_off;           // + this element offset (the product's block, the K slab)
  const char* Bp;            // weight planes of column 0 at the first K block
  float* C;                  // partial row m at C + m * ldc
  const unsigned* mask;      // optional: mask[m_tile] & 1 = compute (else the partials stay)
  int M, m_tiles, nk, blk0;
};
struct FcGroup {
  FcDesc d[FCK_MAX];
  int n, kb_total, n_tiles, n_store;
  long long ldc;
  int rr;                    // 1: M tiles dealt round robin to the XCDs (grid 8 * ceil(M tiles / 8) * n_tiles)
};

// rr: work is dealt to the XCDs by M tile, round robin over the descriptors' M tiles in order (a
// workgroup's XCD is blockIdx mod 8): XCD x runs M tiles x, x + 8, x + 16, ... each with its N tiles
// back to back (the A rows of an M tile are read on one XCD, its ~32 concurrent workgroups share ~5
// M tiles' weight tiles, as the N-fastest order of beluga_fc_h3w).  Contiguous lin ranges per XCD
// (the other kernels' remap, rr 0) give the last XCDs only the short tail GEMM (120 K blocks against
// 250): they idle for the rest of the launch (SQ busy 3.48 of 4 per cycle against 3.89 in the direct
// FC1; FC1 13.0 -> 12.2 ms per step with rr).  Blocks past the last M tile exit.  The masked in-place
// alt launches keep rr 0 (measured slower with rr: 1.44 -> 1.90 ms per step).
template <int TM, int NB, int NS = 2>
__device__ __forceinline__ void fc_h3k_body(const FcGroup& g, char* smem) {
  const unsigned nblk = gridDim.x, bid = blockIdx.x;
  int k = 0, mt, nt;
  if (g.rr) {
    const int slot = (int)(bid >> 3);
    const int T = (slot / g.n_tiles) * 8 + (int)(bid & 7u);   // global M tile (descriptor order)
    nt = slot % g.n_tiles;
    while (k + 1 < g.n && T >= g.d[k + 1].blk0 / g.n_tiles) ++k;
    mt = T - g.d[k].blk0 / g.n_tiles;
    if (mt >= g.d[k].m_tiles) return;                 // past the last descriptor's M tiles
  } else {
    const unsigned xcd = bid & 7u, q = nblk >> 3, rr = nblk & 7u;
    const int lin = (int)((xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3));
    while (k + 1 < g.n && lin >= g.d[k + 1].blk0) ++k;
    const int r = lin - g.d[k].blk0;
    nt = r % g.n_tiles;
    mt = r / g.n_tiles;
  }
  const FcDesc& d = g.d[k];
  if (d.mask && !(d.mask[mt] & 1u)) return;
  const int n0 = nt * 16 * NB;
  constexpr int ROW_KB = 128;
  fc_h3w_tile<TM, NB, NS>(d.A, d.a_rows, d.a_off, 0, 0, d.M, d.Bp + (long long)n0 * g.kb_total * ROW_KB, g.kb_total,
                          d.nk, d.C, g.ldc, g.n_store, (long long)mt * X6P_BM, n0, smem);
}

template <int TM = 0>
__global__ __launch_bounds__(512, 1) void beluga_fc_h3k(FcGroup g) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * FcwGeo<FCW_NB>::STAGE];
  fc_h3k_body<TM, FCW_NB>(g, smem);
}

// the same grouped launch on 112-column tiles (per-window forwards of small batches; same bits)
__global__ __launch_bounds__(512, 1) void beluga_fc_h3k_narrow(FcGroup g) {
  __shared__ __attribute__((aligned(1024))) char smem[3 * FcwGeo<7>::STAGE];
  fc_h3k_body<0, 7, 3>(g, smem);
}

// ---- f16x3 conv GEMM with the Toeplitz A tile staged once per channel chunk -------------
// For a k=8 conv the 8 taps of one 32-channel chunk read A rows m0+tap .. m0+tap+255: the same
// 263 rows shifted by one.  gemm_planes_body re-stages them for every tap (8x the A traffic);
// here the chunk's 288-row A slab (2 planes, 36 KB) is staged ONCE into a double-buffered slab
// and the 8 tap stages read it at row offset +tap, while B (the weights of one (chunk, tap)
// K-block, 20 KB) streams through a 3-deep ring.  A of chunk c+1 is fetched during chunk c
// (9 pieces per wave, one or two per tap, issued before that stage's B pieces so a uniform
// vmcnt(5) at every stage end covers it).  Same operands, products and k order as
// gemm_planes_body<PL=2>: results are bitwise identical.
// LDS: 2 x 36,864 (A slabs) + 3 x 20,480 (B ring) = 135,168 B.
constexpr int H3C_AROWS = 288;                         // 256 + 7 rows needed, 18 groups of 16
constexpr int H3C_APLANE = H3C_AROWS * 64;             // 18,432 B
constexpr int H3C_ASLAB = 2 * H3C_APLANE;              // 36,864 B
constexpr int H3C_BSTAGE = 2 * X6P_B_PLANE;            // 20,480 B
template <int NSB>
constexpr int h3c_lds() { return 2 * H3C_ASLAB + NSB * H3C_BSTAGE; }

// Slab geometry of the chunk-slab kernel for MB 16-row blocks per wave (tile BM = 64 * MB rows):
//   MB 4: 256-row tile, 288-row slab (18 groups, 9 LDS-DMA pieces per wave and chunk);
//   MB 6: 384-row tile, 400-row slab (25 groups = 50 pieces, 13 per wave: waves 2 and 3 repeat
//         piece 49, identical bytes to the same LDS address), LDS 2 x 51,200 + 3 x 20,480 =
//         163,840 B = all of a CU's LDS.  Each B (weight) piece then feeds 1.5x the MFMAs, and
//         a K-block stage (one barrier) is 180 instead of 120 MFMAs per wave.
template <int MB>
struct SlabGeo {
  static constexpr int BM = 64 * MB;
  static constexpr int GROUPS = MB == 4 ? 18 : (BM + 7 + 15) / 16;
  static constexpr int AROWS = 16 * GROUPS;
  static constexpr int APLANE = AROWS * 64;
  static constexpr int ASLAB = 2 * APLANE;
  static constexpr int PIECES = 2 * GROUPS;
  static constexpr int NA = (PIECES + 3) / 4;          // slab pieces per wave and chunk
  static constexpr int EXTRA = NA - 8;                 // taps 0 .. EXTRA-1 issue 2 pieces, the rest 1
  static_assert(AROWS >= BM + 7 && NA >= 8 && NA <= 16, "slab geometry");
};
template <int NSB, int MB>
constexpr int h3c_lds_mb() { return 2 * SlabGeo<MB>::ASLAB + NSB * H3C_BSTAGE; }

// ReLU epilogue of the f16x3 conv kernel through LDS.  A wave's 64 x 160 tile is, per output
// row, ONE contiguous 640-B run of the planes layout (5 blocks x [hi 64 B | lo 64 B]); the
// accumulator layout scatters it over 2-byte pieces.  Each half of the tile (32 rows) is split
// into the wave's private LDS area (row stride 656 B: the 4 row groups of a ds_write_b16 land
// on distinct banks), then written out as 16-B chunks (20 per lane), each row fully coalesced.

// (Measured and not kept, tools/gemm_bench + the same-box pipeline A/B tools/ab_bench.sh:
// streamed (nontemporal) stores and the plain split gained 1.6-4.1 % on conv3 / conv5 / conv6
// alone but moved no layer time of the 200-window pipeline; streamed stores cost conv1 6 %.)
// Per-column epilogue factors of a lane's 10 columns n0 + 16 nb + (lane & 15): the column scale
// and the bias, each x out_scale (0 past n_store).  All 20 loads are issued before the first use
// (clamped, unconditional indices), so the wave waits for them ONCE.  Round 2 loaded them per
// column block under an n < n_store branch, right before use: 20-40 loads per tile each followed
// by s_waitcnt vmcnt(0) -- which also waited for the epilogue's own earlier global stores --
// i.e. 20-40 serialized memory latencies per tile (BATCH false: that form, a timing probe).
template <bool BATCH = true, int NB = 10>
__device__ __forceinline__ void epi_factors(const GemmArgs& p, int n0, int fr, float (&cso)[NB], float (&bo)[NB]) {
  float c[NB], b[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const int n = n0 + nb * 16 + fr;
    if constexpr (BATCH) {
      const int nc = min(n, p.n_store - 1);
      c[nb] = p.col_scale[nc];
      b[nb] = p.bias[nc];
    } else {
      c[nb] = n < p.n_store ? p.col_scale[n] : 0.f;
      b[nb] = n < p.n_store ? p.bias[n] : 0.f;
    }
  }
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const bool in = n0 + nb * 16 + fr < p.n_store;
    // fmaxf(acc*cs + b, 0) * osc with the power-of-2 scales folded: the same value
    cso[nb] = in ? c[nb] * p.out_scale : 0.f;
    bo[nb] = in ? b[nb] * p.out_scale : 0.f;
  }
}

// NOSTORE: timing probe (tools/ck_bench direct_nostore, wrong results): everything but the global stores
template <int MB = 4, bool BATCH = true, int NB = 10, bool NOSTORE = false>
__device__ __forceinline__ void epilogue_relu_h2_lds(const GemmArgs& p, const floatx4v (&acc)[MB][NB], long long mw,
                                                     int n0, int lane, char* lds) {
  static_assert(NB % 2 == 0, "whole 32-column blocks");
  constexpr int CPR = 4 * NB;                          // 16-B chunks per staged row (40 | 16)
  const int fr = lane & 15, fq = lane >> 4;
  const long long w0 = mw / p.s_in;
  const int t0 = (int)(mw - w0 * p.s_in);
  float csov[NB], bov[NB];
  epi_factors<BATCH, NB>(p, n0, fr, csov, bov);
  // overflow: a running max per lane and ONE flag store at the end (a per-value conditional
  // store compiled to a branch and exec-mask juggling around every value: ~4 instructions each)
  float vmax = 0.f;
#pragma unroll
  for (int half = 0; half < MB / 2; ++half) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const float cso = csov[nb], bo = bov[nb];
#pragma unroll
      for (int mh = 0; mh < 2; ++mh) {
        const int mb = 2 * half + mh;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float x = fmaxf(fmaf(acc[mb][nb][j], cso, bo), 0.f);
          vmax = fmaxf(vmax, x);
          _Float16 hi, lo;
          split_h2p(x, hi, lo);
          char* d = lds + (mh * 16 + 4 * fq + j) * H3E_ROW + (nb >> 1) * 128 + ((nb & 1) * 16 + fr) * 2;
          *(_Float16*)d = hi;
          *(_Float16*)(d + 64) = lo;
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const long long ldb = p.ldc >> 5;
#pragma unroll 4
    for (int i = 0; i < CPR / 2; ++i) {
      const int k = i * 64 + lane, row = k / CPR, ch = k - row * CPR;
      const long long m = mw + half * 32 + row;
      if (m < p.M) {
        long long w;
        int tpos;
        row_wt(w0, t0, half * 32 + row, p.s_in, w, tpos);
        if (tpos < p.t_valid && n0 + (ch >> 3) * 32 < p.n_store) {
          const long long orow = w * p.s_out + tpos;
          char* g = (char*)p.C + (orow * ldb + (n0 >> 5)) * 128 + ch * 16;
          const floatx4v v = *(const floatx4v*)(lds + row * H3E_ROW + ch * 16);
          if constexpr (NOSTORE)
            vmax = fmaxf(vmax, v[0]);
          else
            *(floatx4v*)g = v;
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if (!(vmax < 65504.f)) *p.ovf = 1;   // overflow: the call is recomputed (bf16x6)
}

// LDS swizzle of the conv kernels' A slab and B stages: the 16-B chunk c of row r sits at
// position c ^ swz(r).  The 16x16x32 fragment reads of tap t read rows t..t+15 (A) and 0..15 (B);
// a ds_read_b128 lane group then holds, per row residue mod 4 (= the bank quarter), four rows in
// consecutive quads with chunk pattern (f, f^1, f^1, f) (the group's fq values).  swz(r) = 2 *
// ((r >> 2) & 1) gives those four lanes distinct positions for EVERY t, i.e. conflict-free
// reads at all 8 tap offsets; round 1's (-(r >> 2)) & 3 is conflict-free at t = 0 mod 4 only
// (2-way conflicts otherwise: SQ_LDS_BANK_CONFLICT 25 % of SQ_LDS_IDX_ACTIVE on conv2).
template <int TM>
__device__ __forceinline__ int conv_swz(int r) {
  return ((r >> 2) & 1) << 1;
}


// Pool epilogue of the f16x3 conv kernels through LDS.  A lane's 4 accumulator rows of a
// 16-row block are one pool group (rows 4*fq..4*fq+3; m0 and s_in are multiples of 4), so the
// pooled value needs no shuffle: maxpool(relu(x*cs + b)) = relu(max(x)*cs + b) (monotone maps).
// The wave's 4*MB pooled rows x 160 columns are split into its private LDS area in the planes
// layout, then stored as 16-B chunks (one contiguous 640-B run per pooled row) instead of two
// 2-byte stores per value.  Same values as gemm_epilogue16<EPI_RELU_POOL4, 2>.
template <int MB, bool CANON = false, bool BATCH = true, int NB = 10>
__device__ __forceinline__ void epilogue_pool_h2_lds(const GemmArgs& p, const floatx4v (&acc)[MB][NB], long long mw,
                                                     int n0, int lane, char* lds) {
  static_assert(4 * MB <= 32, "pooled rows per wave exceed the LDS area");
  static_assert(NB % 2 == 0, "whole 32-column blocks");
  constexpr int CPR = 4 * NB;                          // 16-B chunks per staged row (40 | 32 | 16)
  const int fr = lane & 15, fq = lane >> 4;
  float csov[NB], bov[NB];
  epi_factors<BATCH, NB>(p, n0, fr, csov, bov);
  float vmax = 0.f;   // overflow: running max, one flag store at the end
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const float cso = csov[nb], bo = bov[nb];
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const float mx = fmaxf(fmaxf(acc[mb][nb][0], acc[mb][nb][1]), fmaxf(acc[mb][nb][2], acc[mb][nb][3]));
      const float x = fmaxf(fmaf(mx, cso, bo), 0.f);
      vmax = fmaxf(vmax, x);
      _Float16 hi, lo;
      if constexpr (CANON)
        split_h2(x, hi, lo);
      else
        split_h2p(x, hi, lo);
      char* d = lds + (mb * 4 + fq) * H3E_ROW + (nb >> 1) * 128 + ((nb & 1) * 16 + fr) * 2;
      *(_Float16*)d = hi;
      *(_Float16*)(d + 64) = lo;
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const long long ldb = p.ldc >> 5;
  const long long w0 = mw / p.s_in;
  const int t0 = (int)(mw - w0 * p.s_in);
#pragma unroll 5
  for (int i = 0; i < (4 * MB * CPR) / 64; ++i) {
    const int k = i * 64 + lane, row = k / CPR, ch = k - row * CPR;
    const long long m4 = mw + 4 * row;                  // first conv row of pooled row `row`
    if (m4 < p.M) {
      long long w;
      int t;
      row_wt(w0, t0, 4 * row, p.s_in, w, t);
      const int tp = t >> 2;
      if (tp < p.t_valid && n0 + (ch >> 3) * 32 < p.n_store) {
        char* g = (char*)p.C + ((w * p.s_out + tp) * ldb + (n0 >> 5)) * 128 + ch * 16;
        *(floatx4v*)g = *(const floatx4v*)(lds + row * H3E_ROW + ch * 16);
      }
    }
  }
  if (!(vmax < 65504.f)) *p.ovf = 1;   // overflow: the call is recomputed (bf16x6)
}

// Pool2 of conv4's rows in the epilogue for the segment path's two pool phases 0 and 2 (the 200-bp
// shift sweeps): the same values as EPI_RELU's plain-split rows pooled by pool4_phases_h2m --
// x = relu(acc * cs + b) per row; the phase-p row of group rows t..t+3 (t = p mod 4) is the
// canonical split of max(x), and split_h2(max x) = canon(r(max x)) = canon(max r(x)) with r(x) =
// hi + lo of the plain split (r is monotone and r(r(x)) = r(x)).  A lane holds rows 4 fq .. 4 fq + 3
// of each 16-row block, i.e. a phase-0 group; a phase-2 group takes this lane's rows 2, 3 and the
// next lane group's rows 0, 1 (ds_bpermute by 16 lanes; across a 16-row block the next block's
// register, across waves an LDS exchange).  The group across the tile's end is left to
// pool2_tile_seams, which pools it from the two tiles' edge rows written unpooled (c_seam).  Rows
// of a segment start 4-aligned in M (the caller's segment stride s_in is a multiple of 4), so t and
// the tile-local row agree mod 4.  Pooled rows are staged per wave in LDS (rows 0..15 phase 0,
// 16..31 phase 2) and stored as 16-B chunks like epilogue_pool_h2_lds.
template <bool BATCH>
__device__ __forceinline__ void epilogue_pool_ph02(const GemmArgs& p, floatx4v (&acc)[4][10], long long mw, int n0,
                                                   int lane, int wave, char* smem) {
  constexpr int NB = 10, CPR = 40;
  const int fr = lane & 15, fq = lane >> 4;
  float csov[NB], bov[NB];
  epi_factors<BATCH, NB>(p, n0, fr, csov, bov);
  float vmax = 0.f;
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float x = fmaxf(fmaf(acc[mb][nb][j], csov[nb], bov[nb]), 0.f);
        vmax = fmaxf(vmax, x);
        acc[mb][nb][j] = x;
      }
  const long long w0 = mw / p.s_in;
  const int t0 = (int)(mw - w0 * p.s_in);
  const long long ldb = p.ldc >> 5;
  // unpooled rows others read (plain split, as EPI_RELU stores them)
  auto put_row = [&](char* base, long long drow, const floatx4v (&a)[NB], int j) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      if (n0 + nb * 16 + fr >= p.n_store) continue;
      _Float16 hi, lo;
      split_h2p(a[nb][j], hi, lo);
      char* d = base + drow * ldb * 128 + ((n0 >> 5) + (nb >> 1)) * 128 + ((nb & 1) * 16 + fr) * 2;
      *(_Float16*)d = hi;
      *(_Float16*)(d + 64) = lo;
    }
  };
  // the tile's edge rows: wave 0's rows 0, 1 and wave 3's rows 62, 63 (pool2_tile_seams)
  const long long mt = (mw - wave * 64) >> 8;
  if (wave == 0 && fq == 0) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
      if (mw + j < p.M) put_row((char*)p.c_seam, mt * 4 + j, acc[0], j);
  } else if (wave == 3 && fq == 3) {
#pragma unroll
    for (int j = 2; j < 4; ++j)
      if (mw + 60 + j < p.M) put_row((char*)p.c_seam, mt * 4 + j, acc[3], j);
  }
  // seg_delta_pool's ref rows: only waves whose 64 rows meet a segment's range (wave-uniform test;
  // the rows span at most two segments)
  if (p.unp_tab && mw < p.M) {
    auto range = [&](long long w, int& lo_, int& hi_) {
      const int* tb = p.unp_tab + w * p.unp_ld;   // phase 0 pooled rows from tb[5], phase 2 from tb[6]
      lo_ = min(4 * tb[5], 2 + 4 * tb[6]);
      hi_ = max(4 * (tb[5] + p.unp_dw), 2 + 4 * (tb[6] + p.unp_dw));
    };
    long long wl;
    int tl;
    row_wt(w0, t0, 63, p.s_in, wl, tl);
    int lo0, hi0, lo1 = 0, hi1 = 0;
    range(w0, lo0, hi0);
    bool hit = t0 < hi0 && (wl == w0 ? tl : p.s_in - 1) >= lo0;
    if (wl != w0 && wl * p.s_in < p.M) {   // (a segment past the launch's rows has no table entry)
      range(wl, lo1, hi1);
      hit = hit || (0 < hi1 && tl >= lo1);
    }
    if (hit) {
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int ro = mb * 16 + 4 * fq + j;
          if (mw + ro >= p.M) continue;
          long long w;
          int t;
          row_wt(w0, t0, ro, p.s_in, w, t);
          const int ulo = w == w0 ? lo0 : lo1, uhi = w == w0 ? hi0 : hi1;
          if (t >= ulo && t < uhi && t - ulo < 32) put_row((char*)p.c_edge, w * 32 + (t - ulo), acc[mb], j);
        }
    }
  }
  // phase-2 partners: h01 = max of a lane's rows 0, 1; rot = the next lane group's h01
  float* xch = (float*)(smem + 4 * H3E_WAVE);   // [wave][nb][fr]: h01 of block 0, lane group 0
  if (wave > 0 && fq == 0) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) xch[(wave * NB + nb) * 16 + fr] = fmaxf(acc[0][nb][0], acc[0][nb][1]);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();   // (the producers meet it before they end)
  asm volatile("" ::: "memory");
  char* const lds = smem + wave * H3E_WAVE;
  const int src = ((lane + 16) & 63) * 4;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    float rot[4];
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
      rot[mb] = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src, __builtin_bit_cast(int, fmaxf(acc[mb][nb][0], acc[mb][nb][1]))));
    const float nxt = wave < 3 ? xch[((wave + 1) * NB + nb) * 16 + fr] : 0.f;
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
      const float m0v = fmaxf(fmaxf(acc[mb][nb][0], acc[mb][nb][1]), fmaxf(acc[mb][nb][2], acc[mb][nb][3]));
      const float part = fq < 3 ? rot[mb] : (mb < 3 ? rot[mb + 1] : nxt);
      const float m2v = fmaxf(fmaxf(acc[mb][nb][2], acc[mb][nb][3]), part);
      _Float16 hi, lo;
      split_h2(m0v, hi, lo);
      char* d = lds + (mb * 4 + fq) * H3E_ROW + (nb >> 1) * 128 + ((nb & 1) * 16 + fr) * 2;
      *(_Float16*)d = hi;
      *(_Float16*)(d + 64) = lo;
      split_h2(m2v, hi, lo);
      d += 16 * H3E_ROW;
      *(_Float16*)d = hi;
      *(_Float16*)(d + 64) = lo;
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll 4
  for (int i = 0; i < (32 * CPR) / 64; ++i) {
    const int k = i * 64 + lane, row = k / CPR, ch = k - row * CPR;
    const int ph = row >> 4, g = row & 15;   // phase index (0: phase 0, 1: phase 2), group
    const int ro = 4 * g + 2 * ph;          // first row of the group in the wave's 64
    if (ph == 1 && wave == 3 && g == 15) continue;   // across the tile's end: pool2_tile_seams
    const long long m = mw + ro;
    if (m + 3 >= p.M) continue;
    long long w;
    int t;
    row_wt(w0, t0, ro, p.s_in, w, t);
    if (t + 3 >= p.t_valid || n0 + (ch >> 3) * 32 >= p.n_store) continue;   // group past its segment's rows
    const long long prow = (2 * w + ph) * p.s_out + (t >> 2);
    char* gp = (char*)p.C + (prow * ldb + (n0 >> 5)) * 128 + ch * 16;
    *(floatx4v*)gp = *(const floatx4v*)(lds + row * H3E_ROW + ch * 16);
  }
  if (!(vmax < 65504.f)) *p.ovf = 1;   // overflow: the call is recomputed (bf16x6)
}

// NSB: depth of the B ring (3: loads of stage s+2 in flight during stage s; 4: s+3).
template <int LAYER, int EPI, int TM, int NSB, int MB = 4>
__device__ __forceinline__ void gemm_conv_h3_body(const GemmArgs& p, char* smem) {
  static_assert(NSB == 3 || (NSB == 4 && MB == 4), "B ring depth");
  using G = SlabGeo<MB>;
  constexpr int ROW_KB = 128;                         // global bytes per row and 32-channel block
  const unsigned nblk = gridDim.x, bid = blockIdx.x;
  const unsigned xcd = bid & 7u, q = nblk >> 3, rr = nblk & 7u;
  const unsigned lin = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  const int nt = (int)(lin % (unsigned)p.n_tiles);
  const long long mt = (long long)(lin / (unsigned)p.n_tiles) % p.m_tiles;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const long long m0 = mt * G::BM;
  const int n0 = nt * GBN;
  const int kb_total = (int)(p.ldb / GBK);
  const long long lda_kb = p.lda / GBK;
  const int nchunk = (int)lda_kb;                     // Cin / 32
  const int nk = nchunk * 8;
  auto swz = [](int r) { return conv_swz<TM>(r); };
  // A slab pieces: P = wave + 4*i (i < NA) of G::PIECES = row groups x 2 planes
  const char* Ab = (const char*)p.A + m0 * lda_kb * ROW_KB;
  const long long last_row = p.M - 1 + 7;             // Toeplitz rows read by the last output row
  unsigned aoff[G::NA];
#pragma unroll
  for (int i = 0; i < G::NA; ++i) {
    const int P = min(wave + 4 * i, G::PIECES - 1), g = P >> 1, pl = P & 1;
    const int r = 16 * g + (lane >> 2);
    const long long m = min(m0 + r, last_row);
    const int c = (lane & 3) ^ swz(r);
    aoff[i] = (unsigned)((m - m0) * lda_kb * ROW_KB + pl * 64 + 16 * c);
  }
  const char* Bb = (const char*)p.Bp + (long long)n0 * kb_total * ROW_KB;
  unsigned boff[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const int g = wave + 4 * j;                        // 20 pieces: plane g / 10, cols 16*(g % 10)
    const int pl = g / 10, r = 16 * (g % 10) + (lane >> 2);
    const int c = (lane & 3) ^ swz(r);
    boff[j] = (unsigned)((long long)r * kb_total * ROW_KB + pl * 64 + 16 * c);
  }
  const __amdgpu_buffer_rsrc_t arsrc = __builtin_amdgcn_make_buffer_rsrc((void*)Ab, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t brsrc = __builtin_amdgcn_make_buffer_rsrc((void*)Bb, (short)0, 0x7fffffff, 0x00020000);
  char* const aslab = smem;
  char* const bring = smem + 2 * G::ASLAB;
  auto issue_a = [&](int chunk, int i0, int ni) {      // pieces i0.. of chunk's slab
    char* base = aslab + (chunk & 1) * G::ASLAB;
    for (int i = i0; i < i0 + ni; ++i) {
      const int P = min(wave + 4 * i, G::PIECES - 1);
      char* dst = base + (P & 1) * G::APLANE + (P >> 1) * 1024;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(arsrc, (lds_void*)dst, 16, aoff[i], (unsigned)(chunk * ROW_KB), 0, 0);
    }
  };
  auto issue_b = [&](int s, int slot) {
    if constexpr ((TM & 8) != 0) s = 0;
    char* base = bring + slot * H3C_BSTAGE;
#pragma unroll
    for (int j = 0; j < 5; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(brsrc, (lds_void*)(base + (wave + 4 * j) * 1024), 16, boff[j],
                                               (unsigned)(s * ROW_KB), 0, 0);
  };
  auto issue_b1 = [&](int s, int slot, int j) {         // one of the 5 B pieces
    if constexpr ((TM & 8) != 0) s = 0;
    char* base = bring + slot * H3C_BSTAGE;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(brsrc, (lds_void*)(base + (wave + 4 * j) * 1024), 16, boff[j],
                                             (unsigned)(s * ROW_KB), 0, 0);
  };

  floatx4v acc[MB][10];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int nb = 0; nb < 10; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[mb][nb][r] = 0.f;
  const int fr = lane & 15, fq = lane >> 4;
  const int brow = fr * 64 + 16 * (fq ^ swz(fr));
  // A fragment of (row group mb, tap t): slab row wave*16*MB + mb*16 + fr + t
  auto read_a = [&](const char* slab, int t, bf16x8 (&a)[MB][3]) {
    const int rr2 = fr + t;
    const int off = (wave * 16 * MB + rr2) * 64 + 16 * (fq ^ swz(rr2));
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      a[mb][0] = *(const bf16x8*)(slab + off + mb * 1024);
      a[mb][1] = *(const bf16x8*)(slab + off + mb * 1024 + G::APLANE);
    }
  };
  auto read_b = [&](const char* base, int nb, bf16x8 (&b)[3]) {
    const char* br = base + brow + nb * 1024;
    b[0] = *(const bf16x8*)(br);
    b[1] = *(const bf16x8*)(br + X6P_B_PLANE);
  };
  auto unit = [&](const bf16x8 (&a)[MB][3], int nb, const bf16x8 (&b)[3]) {
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) acc[mb][nb] = planes_mfma<2>(acc[mb][nb], a[mb], b);
  };
  auto pin = [&](int nv) {
#pragma unroll
    for (int i = 0; i < 3 * MB; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      if ((i % 6) == 0 && i < 6 * nv) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      if ((i & 1) == 0) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
    }
  };

  // prologue: slab 0, B stages 0 .. NSB-2
  issue_a(0, 0, G::NA);
  issue_b(0, 0);
  issue_b(min(1, nk - 1), 1);
  if constexpr (NSB == 4) {
    issue_b(min(2, nk - 1), 2);
    asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  bf16x8 as[MB][3];
  read_a(aslab, 0, as);
  int slot = 0;
  for (int c = 0; c < nchunk; ++c) {
    const char* slab = aslab + (c & 1) * G::ASLAB;
    const bool more_a = (c + 1 < nchunk) && !(TM & 2);
    for (int t = 0; t < 8; ++t) {
      const int s = c * 8 + t;
      const int nslot = slot + 1 == NSB ? 0 : slot + 1;
      const int lslot = slot == 0 ? NSB - 1 : slot - 1;     // stage s + NSB - 1 (the slot read at s - 1)
      const char* base = bring + slot * H3C_BSTAGE;
      bf16x8 b0[3], b1[3];
      read_b(base, 0, b0);
      // slab c+1, NA pieces: NSB 3 -> taps 0..EXTRA-1 two pieces, the others one (MB 4:
      // 2,1,1,1,1,1,1,1; MB 6: 2,2,2,2,2,1,1,1); NSB 4 (MB 4) -> taps 0..5 as 2,2,2,1,1,1
      // (the last two taps issue B only, so vmcnt(10) at tap 7 covers the slab)
      constexpr int E = G::EXTRA;
      const int i0 = NSB == 3 ? (t < E ? 2 * t : E + t) : (t < 3 ? 2 * t : t + 3);
      const int ni = !more_a ? 0 : NSB == 3 ? (t < E ? 2 : 1) : (t < 3 ? 2 : (t < 6 ? 1 : 0));
#pragma unroll
      for (int nb = 0; nb < 10; ++nb) {
        int nv = 0;
        // one LDS-DMA piece per unit, slab pieces first (units 0-1) so the stage-end vmcnt(5) =
        // "all but this stage's 5 B pieces" still covers them: an isolated piece among MFMAs
        // costs its wave ~60 issue cycles, one inside a burst 100-185 (MI355X_MICROARCH.md,
        // LDS-DMA issue-cost row; round 1's burst schedule measured slower)
        if (nb < 2 && nb < ni) {
          issue_a(c + 1, i0 + nb, 1);
          nv = 1;
        }
        if (nb >= 2 && nb < 7 && !(TM & 2)) {
          issue_b1(min(s + NSB - 1, nk - 1), lslot, nb - 2);
          nv = 1;
        }
        if (nb + 1 < 10) read_b(base, nb + 1, (nb & 1) ? b0 : b1);
        unit(as, nb, (nb & 1) ? b1 : b0);
        pin(nv);
      }
      if (t < 7) read_a(slab, t + 1, as);     // same slab: already resident
      if constexpr (!(TM & 4)) {
        // all but the B pieces of the last NSB-2 stages: B(s+1), and slab c+1 by its last tap.
        // The next tap's A fragment reads (from the slab, which no DMA touches before the
        // chunk after next) stay in flight across the barrier: the MFMAs that use them wait.
        if constexpr (NSB == 4)
          asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
        else
          asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      }
      asm volatile("" ::: "memory");
      slot = nslot;
    }
    if (c + 1 < nchunk) read_a(aslab + ((c + 1) & 1) * G::ASLAB, 0, as);
  }
  if constexpr (EPI == EPI_RELU || EPI == EPI_RELU_POOL4) {
    // the ring's last (duplicate) B pieces may still be landing: drain before reusing LDS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if constexpr (EPI == EPI_RELU)
      epilogue_relu_h2_lds<MB, (TM & 8192) == 0>(p, acc, m0 + wave * 16 * MB, n0, lane, smem + wave * H3E_WAVE);
    else
      epilogue_pool_h2_lds<MB, LAYER == 4, (TM & 8192) == 0>(p, acc, m0 + wave * 16 * MB, n0, lane,
                                                             smem + wave * H3E_WAVE);
  } else {
    gemm_epilogue16<EPI, 2, 10, MB>(p, acc, m0 + wave * 16 * MB, n0, 0, lane);
  }
}

// ---- the library's bf16x6 GEMM (16x16x32 MFMAs, LDS-DMA staged) ---------------------------
// beluga_gemm_x6q: bf16x6 (3 bf16 planes, 6 products): fp32-faithful over fp32's whole range.
// (The f16x3 layers -- 2 fp16 planes of pre-scaled operands, 3 products -- run the conv / FC
// kernels below; the same body at PL 2, beluga_gemm_h3q, is a probe in tools/gemm_probes.h.)
template <int LAYER, int EPI, int TM = 0>
__global__ __launch_bounds__(256, 1) void beluga_gemm_x6q(GemmArgs p) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * PlaneGeo<3>::STAGE];
  gemm_planes_body<LAYER, EPI, TM, 3, 2>(p, smem);
}

// f16x3 conv layers (taps == 8, no split-K): the chunk-slab body above with 384-row tiles (6
// row blocks per wave): 1.5x the MFMAs per weight piece and per stage barrier of the 256-row
// form (beluga_conv_h3q, tools/gemm_probes.h); bitwise equal (same products and k order)
template <int LAYER, int EPI, int TM = 0>
__global__ __launch_bounds__(256, 1) void beluga_conv_h3r(GemmArgs p) {
  __shared__ __attribute__((aligned(1024))) char smem[h3c_lds_mb<3, 6>()];
  gemm_conv_h3_body<LAYER, EPI, TM, 3, 6>(p, smem);
}

// ---- f16x3 conv GEMM, producer / consumer waves ------------------------------------------
// gemm_conv_h3_body (256 x 160 tile, 4 waves of 64 x 160) with every LDS-DMA issue moved to 4
// extra "producer" waves, one per SIMD beside its MFMA wave.  An LDS-DMA piece costs the wave
// that issues it 60-185 issue cycles among MFMAs, but a partner wave's load segment costs the
// MFMA wave only ~40 cycles (MI355X_MICROARCH.md "Two waves per SIMD" item 7 and the LDS-DMA
// issue-cost row), and the A-slab + B-ring pieces of one stage are ~6.6 per MFMA wave.
// Producers issue the B pieces of stage s+2 and the next chunk's slab pieces right after
// barrier s-1, wait for everything but this stage's B pieces, and meet the consumers at barrier
// s.  Two waves per SIMD cap a wave at 256 registers: the consumer's 160 accumulators + A and B
// fragments fit at 64 rows per wave.  Same products and k order per output as every f16x3 conv
// kernel: bitwise equal.
// NSB: B ring depth; 4 gives the producers' pieces two stages to land (slab pieces then go out
// at taps 0-5 only, so the vmcnt that leaves the last two stages' B pieces in flight covers them).
// Producer waves of conv2 with conv1 FUSED (TM & H3P_FUSE_CONV1; f16x3).  Instead of LDS-DMA
// copies of conv1's stored planes, the producers compute each 32-channel chunk's A slab (288 conv1
// rows x 32 channels, hi and lo planes) from base codes -- conv1's 2 x 5 GB of plane writes and
// re-reads per 200-window step never reach HBM.  Conv1 is the K = 32 one-hot GEMM of
// beluga_conv1_h3 (k = tap*4 + channel) issued TRANSPOSED: A = the chunk's weight planes (rows =
// channels), B = the one-hot fragment of 16 slab rows (a lane's positions t+2fq, t+2fq+1), so the
// 16x16 result gives a lane 4 consecutive CHANNELS of one row = one 8-byte piece of the slab row
// per plane.  The dot products are those of beluga_conv1_h3 over the same k (products x*w_lo
// into 0, then x*w_hi), followed by its epilogue (fmaf(acc, cs*osc, b*osc), ReLU, plain split):
// bitwise the planes beluga_conv1_h3 stores, so conv2's output is bitwise the unfused one
// (tests/test_gpu_forward.py).  Work per chunk and workgroup: 18 groups of 16 rows x 2 channel
// blocks x 2 MFMAs (72 MFMAs beside the consumers' 3,840, +1.9 %) and 36 values per producer lane.
// Schedule: the one-hot fragments of the producer's <= 5 groups (groups pw + 4i) are built once
// per tile from codes (global byte loads); chunk c+1's weights are loaded at tap 0 of chunk c and
// its slab groups computed at taps 1..5, written with ds_write_b64 and drained (lgkmcnt(0)) before
// those taps' barriers -- slab c+1 is complete at barrier 5, before the consumers read it (tap 7's
// PF read, after barrier 6).  The B ring is issued exactly as in the unfused producer.
template <int NSB, bool PF>
__device__ __forceinline__ void conv12_producer(const GemmArgs& p, char* smem, long long m0, int n0, int pw,
                                                int lane) {
  using G = SlabGeo<4>;
  constexpr int ROW_KB = 128;
  constexpr int NG = 5;                               // slab groups per producer wave (18 over 4 waves)
  const int kb_total = (int)(p.ldb / GBK);
  const int nchunk = (int)(p.lda / GBK);
  const int nk = nchunk * 8;
  char* const aslab = smem;
  char* const bring = smem + 2 * G::ASLAB;
  auto swz = [](int r) { return conv_swz<0>(r); };
  // B ring pieces: as gemm_conv_h3p_body's producers
  const char* Bb = (const char*)p.Bp + (long long)n0 * kb_total * ROW_KB;
  unsigned boff[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const int g = pw + 4 * j;
    const int pl = g / 10, r = 16 * (g % 10) + (lane >> 2);
    const int c = (lane & 3) ^ swz(r);
    boff[j] = (unsigned)((long long)r * kb_total * ROW_KB + pl * 64 + 16 * c);
  }
  const __amdgpu_buffer_rsrc_t brsrc = __builtin_amdgcn_make_buffer_rsrc((void*)Bb, (short)0, 0x7fffffff, 0x00020000);
  auto issue_b = [&](int s, int slot) {
    char* base = bring + slot * H3C_BSTAGE;
#pragma unroll
    for (int j = 0; j < 5; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(brsrc, (lds_void*)(base + (pw + 4 * j) * 1024), 16, boff[j],
                                               (unsigned)(s * ROW_KB), 0, 0);
  };
  // one-hot B fragments of the wave's slab rows (built once per tile)
  const int fr = lane & 15, fq = lane >> 4;
  halfx8 oh[NG];
  bool rvalid[NG];
#pragma unroll
  for (int i = 0; i < NG; ++i) {
    const int g = pw + 4 * i;
    unsigned c0 = 4, c1 = 4;
    rvalid[i] = false;
    if (g < G::GROUPS) {
      const long long m = m0 + 16 * g + fr;
      const long long w = m / p.s_in;
      const int t = (int)(m - w * p.s_in);
      if (w < p.c1_n_win) {
        long long src = p.c1_row0 + w;
        bool rc = p.c1_mode == 1;
        if (p.c1_mode == 2 && src >= p.c1_n_src) {
          src -= p.c1_n_src;
          rc = true;
        }
        const unsigned char* row = p.c1_codes + src * p.c1_stride;
        const int pos = t + 2 * fq;
        if (pos < p.c1_len) c0 = row[rc ? p.c1_len - 1 - pos : pos];
        if (pos + 1 < p.c1_len) c1 = row[rc ? p.c1_len - 2 - pos : pos + 1];
        if (rc) {
          c0 = c0 < 4 ? 3 - c0 : c0;
          c1 = c1 < 4 ? 3 - c1 : c1;
        }
        rvalid[i] = t < p.c1_len - 7;
      }
    }
    const u32x4 u = {onehot_h2(c0, 0), onehot_h2(c0, 1), onehot_h2(c1, 0), onehot_h2(c1, 1)};
    oh[i] = __builtin_bit_cast(halfx8, u);
  }
  // chunk weights: A fragments of channels 32c + 16cb + fr, factors of channels 32c + 16cb + 4fq + j
  halfx8 wh[2], wl[2];
  floatx4 sc[2], bb[2];
  auto load_w = [&](int c) {
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      const _Float16* w = p.c1_w + (32 * c + 16 * cb + fr) * 64 + 8 * fq;
      wh[cb] = *(const halfx8*)w;
      wl[cb] = *(const halfx8*)(w + 32);
      sc[cb] = *(const floatx4*)(p.c1_cs + 32 * c + 16 * cb + 4 * fq);
      bb[cb] = *(const floatx4*)(p.c1_b + 32 * c + 16 * cb + 4 * fq);
    }
  };
  auto scale_w = [&]() {   // cs * osc and b * osc, as beluga_conv1_h3 forms them (once per chunk)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      sc[cb] *= p.c1_osc;
      bb[cb] *= p.c1_osc;
    }
  };
  float vmax = 0.f;
  auto slab_group = [&](char* base, int i) {
    const int g = pw + 4 * i;
    if (g >= G::GROUPS) return;
    const int r = 16 * g + fr;
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      floatx4v c = {0.f, 0.f, 0.f, 0.f};
      c = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl[cb], oh[i], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[cb], oh[i], c, 0, 0, 0);
      floatx4 v;
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = fmaxf(fmaf(c[j], sc[cb][j], bb[cb][j]), 0.f);
      const float vm = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
      vmax = fmaxf(vmax, rvalid[i] ? vm : 0.f);
      // split_h2p of the 4 values, converted in pairs (v_cvt_pk_f16_f32: the same RNE conversion)
      const halfx4 hv = __builtin_convertvector(v, halfx4);
      const halfx4 lv = __builtin_convertvector(v - __builtin_convertvector(hv, floatx4), halfx4);
      const int off = r * 64 + 16 * ((2 * cb + (fq >> 1)) ^ swz(r)) + 8 * (fq & 1);
      *(halfx4*)(base + off) = hv;
      *(halfx4*)(base + G::APLANE + off) = lv;
    }
  };
  load_w(0);
  scale_w();
  issue_b(0, 0);
  issue_b(min(1, nk - 1), 1);
  if constexpr (NSB == 4) issue_b(min(2, nk - 1), 2);
#pragma unroll
  for (int i = 0; i < NG; ++i) slab_group(aslab, i);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if constexpr (NSB == 4) {
    if constexpr (PF)
      asm volatile("s_waitcnt vmcnt(5)" ::: "memory");    // stages 0 and 1 landed
    else
      asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  int slot = 0;
  for (int c = 0; c < nchunk; ++c) {
    const bool more = c + 1 < nchunk;
    char* const nslab = aslab + ((c + 1) & 1) * G::ASLAB;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int s = c * 8 + t;
      const int lslot = slot == 0 ? NSB - 1 : slot - 1;
      if (t == 0 && more) load_w(c + 1);
      if (t == 1 && more) scale_w();
      if (t >= 1 && t <= NG && more) slab_group(nslab, t - 1);
      issue_b(min(s + NSB - 1, nk - 1), lslot);
      if constexpr (NSB == 4 && !PF)
        asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      if (t >= 1 && t <= NG) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      slot = slot + 1 == NSB ? 0 : slot + 1;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (!(vmax < 65504.f)) *p.ovf = 1;   // conv1 value out of fp16 range: recomputed (bf16x6)
}

template <int LAYER, int EPI, int TM, int NSB, int NB = 10>
__device__ __forceinline__ void gemm_conv_h3p_body(const GemmArgs& p, char* smem) {
  static_assert(NSB == 3 || NSB == 4, "B ring depth");
  // NB 16-column blocks per tile: 10 (160 columns), 8 (128: conv3 / conv4 of small batches, 4 N
  // tiles of 480 outputs -- the weight planes carry 32 zero rows -- so 62 M tiles x 4 fit one round
  // of 256 CUs at batch 32 where 3 N tiles left 70 idle) or 4 (64: conv5 / conv6 of small batches,
  // 2.5x the workgroups); an output's products and k order do not depend on the tile width: same bits
  static_assert(NB == 10 || ((NB == 4 || NB == 8) && (TM & H3P_FUSE_CONV1) == 0 &&
                             (EPI == EPI_RELU || EPI == EPI_RELU_POOL4)), "conv tile width");
  constexpr int JB = NB / 2;                          // B pieces per producer wave and stage (of 2 NB)
  // PF (NSB 4): producers keep one stage less in flight, so at the end of stage s the consumers
  // can already read stage s+1's first B fragments (and, at a chunk's last tap, the next slab's
  // A fragments) and start it right after the barrier without an LDS round trip.
  constexpr bool PF = NSB == 4 && (TM & 256) != 0;
  using G = SlabGeo<4>;
  constexpr int ROW_KB = 128;
  constexpr int NAP = (G::PIECES + 3) / 4;            // slab pieces per producer wave and chunk (9)
  const unsigned nblk = gridDim.x, bid = blockIdx.x;
  const unsigned xcd = bid & 7u, q = nblk >> 3, rr = nblk & 7u;
  const unsigned lin = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  const int nt = (int)(lin % (unsigned)p.n_tiles);
  const long long mt = (long long)(lin / (unsigned)p.n_tiles) % p.m_tiles;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const long long m0 = mt * G::BM;
  const int n0 = nt * 16 * NB;
  const int kb_total = (int)(p.ldb / GBK);
  const long long lda_kb = p.lda / GBK;
  const int nchunk = (int)lda_kb;
  const int nk = nchunk * 8;
  auto swz = [](int r) { return conv_swz<TM>(r); };
  char* const aslab = smem;
  char* const bring = smem + 2 * G::ASLAB;

  if (wave >= 4) {
    if constexpr ((TM & H3P_FUSE_CONV1) != 0) {   // conv2 with conv1 fused: slabs from base codes
      conv12_producer<NSB, PF>(p, smem, m0, n0, wave - 4, lane);
      if constexpr (EPI == EPI_RELU || EPI == EPI_RELU_POOL4) __builtin_amdgcn_s_barrier();
      return;
    }
    // ---------------- producer: all LDS-DMA issue ----------------
    const int pw = wave - 4;
    const char* Ab = (const char*)p.A + m0 * lda_kb * ROW_KB;
    const long long last_row = p.M - 1 + 7;
    unsigned aoff[NAP];
#pragma unroll
    for (int i = 0; i < NAP; ++i) {
      const int P = min(pw + 4 * i, G::PIECES - 1), g = P >> 1, pl = P & 1;
      const int r = 16 * g + (lane >> 2);
      const long long m = min(m0 + r, last_row);
      const int c = (lane & 3) ^ swz(r);
      aoff[i] = (unsigned)((m - m0) * lda_kb * ROW_KB + pl * 64 + 16 * c);
    }
    const char* Bb = (const char*)p.Bp + (long long)n0 * kb_total * ROW_KB;
    unsigned boff[5], bdst[5];
#pragma unroll
    for (int j = 0; j < JB; ++j) {
      const int g = pw + 4 * j;
      const int pl = g / NB, r = 16 * (g % NB) + (lane >> 2);
      const int c = (lane & 3) ^ swz(r);
      boff[j] = (unsigned)((long long)r * kb_total * ROW_KB + pl * 64 + 16 * c);
      bdst[j] = (unsigned)((pl * 10 + g % NB) * 1024);   // plane pl at X6P_B_PLANE whatever NB
    }
    const __amdgpu_buffer_rsrc_t arsrc = __builtin_amdgcn_make_buffer_rsrc((void*)Ab, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t brsrc = __builtin_amdgcn_make_buffer_rsrc((void*)Bb, (short)0, 0x7fffffff, 0x00020000);
    auto issue_a = [&](int chunk, int i0, int ni) {
      char* base = aslab + (chunk & 1) * G::ASLAB;
      const int src_chunk = (TM & (8 | 16)) ? 0 : chunk;   // timing probes: A L2-hot
      for (int i = i0; i < i0 + ni; ++i) {
        const int P = min(pw + 4 * i, G::PIECES - 1);
        char* dst = base + (P & 1) * G::APLANE + (P >> 1) * 1024;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(arsrc, (lds_void*)dst, 16, aoff[i], (unsigned)(src_chunk * ROW_KB), 0, 0);
      }
    };
    auto issue_b = [&](int s, int slot) {
      if constexpr ((TM & (8 | 32)) != 0) s = 0;          // timing probes: B L2-hot
      char* base = bring + slot * H3C_BSTAGE;
#pragma unroll
      for (int j = 0; j < JB; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(brsrc, (lds_void*)(base + bdst[j]), 16, boff[j],
                                                 (unsigned)(s * ROW_KB), 0, 0);
    };
    issue_a(0, 0, NAP);
    issue_b(0, 0);
    issue_b(min(1, nk - 1), 1);
    if constexpr (NSB == 4) {
      issue_b(min(2, nk - 1), 2);
      if constexpr (PF)
        wait_vm<JB>();    // stages 0 and 1 landed
      else
        wait_vm<2 * JB>();
    } else {
      wait_vm<JB>();
    }
    __builtin_amdgcn_s_barrier();
    constexpr bool ST = (TM & H3P_STAMP) != 0;
    unsigned long long st_loop = 0, st_bar = 0, st_vm = 0;
    if constexpr (ST) st_loop = h3p_stamp();
    int slot = 0;
    for (int c = 0; c < nchunk; ++c) {
      const bool more_a = (c + 1 < nchunk) && !(TM & 2);
      for (int t = 0; t < 8; ++t) {
        const int s = c * 8 + t;
        const int lslot = slot == 0 ? NSB - 1 : slot - 1;   // stage s+NSB-1's slot (read at s-1)
        if constexpr (NSB == 3) {     // slab pieces 2,1,1,1,1,1,1,1
          if (more_a) issue_a(c + 1, t == 0 ? 0 : t + 1, t == 0 ? 2 : (t + 1 < NAP ? 1 : 0));
        } else {                      // 2,2,2,1,1,1,0,0
          if (more_a && t < 6) issue_a(c + 1, t < 3 ? 2 * t : t + 3, t < 3 ? 2 : 1);
        }
        if (!(TM & 2)) issue_b(min(s + NSB - 1, nk - 1), lslot);
        unsigned long long t0 = 0, t1 = 0;
        if constexpr (ST) t0 = h3p_stamp();
        // everything but the B pieces of the last NSB-2 stages: B(s+1), and slab c+1 by tap 7
        // (PF: all but this stage's pieces, so B(s+2) has landed at barrier s and the
        // consumers read stage s+1's first fragments before that barrier)
        if constexpr (NSB == 4 && !PF)
          wait_vm<2 * JB>();
        else
          wait_vm<JB>();
        if constexpr (ST) t1 = h3p_stamp();
        __builtin_amdgcn_s_barrier();
        if constexpr (ST) {
          const unsigned long long t2 = h3p_stamp();
          st_vm += t1 - t0;
          st_bar += t2 - t1;
        }
        slot = slot + 1 == NSB ? 0 : slot + 1;
      }
    }
    if constexpr (ST) {
      if (lane == 0) {
        unsigned long long* d = p.stamps + ((long long)blockIdx.x * 8 + wave) * 4;
        d[0] = h3p_stamp() - st_loop;
        d[1] = st_bar;
        d[2] = st_vm;
        d[3] = 0;
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (EPI == EPI_RELU || EPI == EPI_RELU_POOL4 || EPI == EPI_POOL_PH02) {
      __builtin_amdgcn_s_barrier();                    // consumers' epilogue reuses the LDS
    }
    if constexpr (EPI == EPI_POOL_PH02) __builtin_amdgcn_s_barrier();   // the epilogue's wave exchange
    return;
  }

  // ---------------- consumer: LDS reads and MFMAs ----------------
  floatx4v acc[4][NB];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[mb][nb][r] = 0.f;
  const int fr = lane & 15, fq = lane >> 4;
  const int brow = fr * 64 + 16 * (fq ^ swz(fr));
  auto read_a = [&](const char* slab, int t, bf16x8 (&a)[4][3]) {
    const int rr2 = fr + t;
    const int off = (wave * 64 + rr2) * 64 + 16 * (fq ^ swz(rr2));
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
      a[mb][0] = *(const bf16x8*)(slab + off + mb * 1024);
      a[mb][1] = *(const bf16x8*)(slab + off + mb * 1024 + G::APLANE);
    }
  };
  auto read_b = [&](const char* base, int nb, bf16x8 (&b)[3]) {
    const char* br = base + brow + nb * 1024;
    b[0] = *(const bf16x8*)(br);
    b[1] = *(const bf16x8*)(br + X6P_B_PLANE);
  };
  auto pin = [&]() {
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      if ((i & 1) == 0) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
    }
  };
  // EA (TM & 64, PF only): the next stage's operands are read INSIDE the stage's last unit -- B
  // fragment 0 of stage s+1 first (b0 is free there: the last unit, NB - 1 odd, runs on b1), then
  // row block mb's A fragments of the next tap right after mb's 3 MFMAs -- instead of all 10 reads
  // after the last MFMA, where the 4 waves' 40 KB of LDS reads met the next stage's first MFMAs
  // across the barrier (tools/ck_bench stamp build: 2,210 cycles per 1,920-cycle stage, unchanged
  // with no loads at all).  The reads go to the same registers, branch-free (past the tile's last
  // stage they re-read resident LDS into registers nothing uses); same MFMAs in the same order.
  constexpr bool EA = PF && (TM & 64) != 0;
  static_assert(!EA || (NB % 2) == 0, "EA: the last unit runs on b1");
  auto read_a1 = [&](const char* slab, int t, int mb, bf16x8 (&a)[3]) {
    const int rr2 = fr + t;
    const int off = (wave * 64 + rr2) * 64 + 16 * (fq ^ swz(rr2));
    a[0] = *(const bf16x8*)(slab + off + mb * 1024);
    a[1] = *(const bf16x8*)(slab + off + mb * 1024 + G::APLANE);
  };
  auto pin_last = [&]() {
    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);   // next stage's b0
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
      __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);   // row block mb's 3 products
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);   // its next-tap A fragments
    }
  };
  __builtin_amdgcn_s_barrier();                       // slab 0 and B stage 0 landed
  asm volatile("" ::: "memory");
  bf16x8 as[4][3];
  bf16x8 b0[3], b1[3];
  read_a(aslab, 0, as);
  if constexpr (PF) read_b(bring, 0, b0);
  constexpr bool ST = (TM & H3P_STAMP) != 0;
  unsigned long long st_loop = 0, st_bar = 0;
  if constexpr (ST) st_loop = h3p_stamp();
  int slot = 0;
  for (int c = 0; c < nchunk; ++c) {
    const char* slab = aslab + (c & 1) * G::ASLAB;
    for (int t = 0; t < 8; ++t) {
      const char* base = bring + slot * H3C_BSTAGE;
      const int nslot = slot + 1 == NSB ? 0 : slot + 1;
      if constexpr (!PF) read_b(base, 0, b0);
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        if (nb + 1 < NB) read_b(base, nb + 1, (nb & 1) ? b0 : b1);
        if (EA && nb == NB - 1) {
          // next tap of this slab, or tap 0 of the next chunk's slab (landed by tap 6's barrier)
          const char* nsl = t < 7 ? slab : aslab + ((c + 1) & 1) * G::ASLAB;
          const int ntap = t < 7 ? t + 1 : 0;
          read_b(bring + nslot * H3C_BSTAGE, 0, b0);   // stage s+1 landed at barrier s-1
#pragma unroll
          for (int mb = 0; mb < 4; ++mb) {
            acc[mb][nb] = planes_mfma<2>(acc[mb][nb], as[mb], b1);
            read_a1(nsl, ntap, mb, as[mb]);
          }
          pin_last();
          continue;
        }
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) acc[mb][nb] = planes_mfma<2>(acc[mb][nb], as[mb], (nb & 1) ? b1 : b0);
        pin();
      }
      if constexpr (!EA) {
        if (t < 7)
          read_a(slab, t + 1, as);   // slab reads stay in flight across the barrier
        else if (PF && c + 1 < nchunk)
          read_a(aslab + ((c + 1) & 1) * G::ASLAB, 0, as);   // next slab landed by tap 6's barrier
        if constexpr (PF) {
          if (c * 8 + t + 1 < nk) read_b(bring + nslot * H3C_BSTAGE, 0, b0);   // stage s+1 landed at barrier s-1
        }
      }
      unsigned long long t1 = 0;
      if constexpr (ST) t1 = h3p_stamp();
      __builtin_amdgcn_s_barrier();
      if constexpr (ST) st_bar += h3p_stamp() - t1;
      asm volatile("" ::: "memory");
      slot = nslot;
    }
    if (!PF && c + 1 < nchunk) read_a(aslab + ((c + 1) & 1) * G::ASLAB, 0, as);
  }
  unsigned long long st_end = 0;
  if constexpr (ST) st_end = h3p_stamp();
  if constexpr ((TM & 2048) != 0) {   // timing probe (wrong results): no epilogue, one store per lane
    __builtin_amdgcn_s_barrier();
    float t = 0.f;
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) t += acc[mb][nb][0] + acc[mb][nb][1] + acc[mb][nb][2] + acc[mb][nb][3];
    p.C[(m0 + wave * 64 + lane) % p.M] = t;
    return;
  }
  if constexpr (EPI == EPI_POOL_PH02) {
    static_assert(NB == 10 && (TM & H3P_FUSE_CONV1) == 0, "pool phases epilogue: wide conv4 tiles");
    __builtin_amdgcn_s_barrier();                     // producers drained their tail pieces
    epilogue_pool_ph02<(TM & 8192) == 0>(p, acc, m0 + wave * 64, n0, lane, wave, smem);
  } else if constexpr (EPI == EPI_RELU || EPI == EPI_RELU_POOL4) {
    __builtin_amdgcn_s_barrier();                     // producers drained their tail pieces
    if constexpr (EPI == EPI_RELU)
      epilogue_relu_h2_lds<4, (TM & 8192) == 0, NB, (TM & 512) != 0>(p, acc, m0 + wave * 64, n0, lane,
                                                                    smem + wave * H3E_WAVE);
    else
      epilogue_pool_h2_lds<4, LAYER == 4, (TM & 8192) == 0, NB>(p, acc, m0 + wave * 64, n0, lane,
                                                                 smem + wave * H3E_WAVE);
    if constexpr (ST) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned long long t = h3p_stamp();
      if (lane == 0) {
        unsigned long long* d = p.stamps + ((long long)blockIdx.x * 8 + wave) * 4;
        d[0] = st_end - st_loop;
        d[1] = st_bar;
        d[2] = 0;
        d[3] = t - st_end;
      }
    }
  } else {
    if constexpr (NB == 10) gemm_epilogue16<EPI, 2, 10, 4>(p, acc, m0 + wave * 64, n0, 0, lane);
  }
}

template <int LAYER, int EPI, int TM = 0, int NSB = 3>
__global__ __launch_bounds__(512, 1) void beluga_conv_h3p(GemmArgs p) {
  __shared__ __attribute__((aligned(1024))) char smem[h3c_lds<NSB>()];
  gemm_conv_h3p_body<LAYER, EPI, TM, NSB>(p, smem);
}

// the same kernel on 64-column (NB 4: conv5 / conv6) or 128-column (NB 8: conv3 / conv4) tiles for
// small per-window batches (same bits)
template <int LAYER, int EPI, int NB = 4>
__global__ __launch_bounds__(512, 1) void beluga_conv_h3p_narrow(GemmArgs p) {
  __shared__ __attribute__((aligned(1024))) char smem[h3c_lds<4>()];
  gemm_conv_h3p_body<LAYER, EPI, 256 | 64, 4, NB>(p, smem);   // early next-stage reads (EA)
}

// B planes for beluga_gemm_x6q from a K-contiguous fp32 B [rows][K] (K % 32 == 0).
__global__ void split_planes(const float* __restrict__ W, long long rows, int K, __bf16* __restrict__ Bp) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * K / 4) return;
  const long long e = 4 * i, n = e / K;
  const int k = (int)(e - n * K), kb = k / GBK, j = k % GBK;
  bf16x4 h, m, l;
  split3(*(const floatx4*)(W + e), h, m, l);
  __bf16* d = Bp + ((n * (K / GBK) + kb) * 3) * GBK + j;
  *(bf16x4*)d = h;
  *(bf16x4*)(d + GBK) = m;
  *(bf16x4*)(d + 2 * GBK) = l;
}

// f16x3 B planes: row n scaled by 2^s_w[n] (s_w from row_scale_exp), then split into fp16
// hi/lo planes [n][K/32][2][32].
__global__ void split_planes_h2(const float* __restrict__ W, long long rows, int K, const int* __restrict__ sw,
                                _Float16* __restrict__ Bp) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * K / 4) return;
  const long long e = 4 * i, n = e / K;
  const int k = (int)(e - n * K), kb = k / GBK, j = k % GBK;
  const floatx4 x = *(const floatx4*)(W + e);
  _Float16* d = Bp + ((n * (K / GBK) + kb) * 2) * GBK + j;
#pragma unroll
  for (int t = 0; t < 4; ++t) split_h2(ldexpf(x[t], sw[n]), d[t], d[GBK + t]);
}

}  // namespace expecto
