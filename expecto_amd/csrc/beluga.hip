// Beluga forward for MI355X (gfx950 / CDNA4): conv1 one-hot kernel + MFMA implicit-GEMM
// kernels (fp32 MFMA, or the fp32-faithful bf16x6 split) with fused bias/ReLU/MaxPool/
// Sigmoid epilogues.
//
// Replaces the ATen ops launched by Beluga.forward (reference Beluga.py:18-51,
// SURVEY.md 2.2).  Layout in HBM (per window, channel-last; fp32 rows on the fp32 path,
// bf16 planes [row][C/32][3][32] on the bf16x6 path, gemm_kernel.h store_act):
//   act0 [1996][320]  conv1 out (1993 valid)          -> buffer P
//   act1 [ 496][320]  conv2+pool (496 valid)          -> buffer Q
//   act2 [ 492][480]  conv3 (489 valid)               -> buffer P
//   act3 [ 120][480]  conv4+pool (120 valid)          -> buffer Q
//   act4 [ 113][640]  conv5 (113 valid)               -> buffer P
//   act5 [ 106][640]  conv6 (106 valid)               -> buffer Q
// With channel-last rows the im2col row of output position t of a k=8 conv is the
// CONTIGUOUS slice X[t*Cin : (t+8)*Cin], so every conv is a GEMM with an overlapping
// (Toeplitz) A operand: A[m][tap,ci] = X[(m+tap)*Cin + ci], K = 8*Cin, taken in the order
// [ci/32][tap][ci%32] (B = W repacked [Cout][ci/32][tap][ci%32]).
// FC1 reads the 106 rows of act5 as one 67840-long row (weights permuted from the
// reference flatten order c*106+t to t*640+c).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cassert>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>
#include <string>
#include <vector>

#include "common.h"
#include "gemm_kernel.h"

namespace expecto {

constexpr int kLen = 2000;         // input window (chromatin.py:35-36, fixed by FC1)
constexpr int kNFeat = 2002;
constexpr int kFc1In = 67840;      // 640 * 106
constexpr int kFc1Out = 2003;
constexpr int kHidLd = 2016;       // FC1 output row stride = FC2 K (2003 padded to 32)
constexpr int kWM = 4;             // GEMM waves per block (stacked along M)
constexpr int kMinBlocks = 2;      // resident blocks per CU the register budget targets
constexpr int kPipe = 1;           // MFMA / ds_read interleave pinned (tools/gemm_bench A/B: +6-8 %)
constexpr int GBM = 32 * kWM;      // GEMM tile rows

// conv1 (4 -> 320, k=8): 32 FMAs per output; one window x 128 positions per block,
// one output channel per thread (coalesced channel-last stores).  The input tile is built
// in LDS either from one-hot floats ([B][4][1][2000], Beluga.py:23) or from base codes
// with the encodeSeqs mapping A,G,C,T -> channel 0..3 (chromatin.py:155-160) and the
// reverse complement [:, ::-1, ::-1] (chromatin.py:170) generated on the fly.
constexpr int C1_T = 128;
__global__ __launch_bounds__(320) void beluga_conv1(const float* __restrict__ x, const uint8_t* __restrict__ codes,
                                                    long long code_stride, int n_src, int mode, long long row0,
                                                    const float* __restrict__ w1, const float* __restrict__ b1,
                                                    float* __restrict__ out, int out_rows, int len, int fmt,
                                                    float osc, int* __restrict__ ovf) {
  __shared__ floatx4 xs[C1_T + 8];
  const int t0 = blockIdx.x * C1_T;
  const long long win = blockIdx.y;
  const long long r = row0 + win;
  const int tid = threadIdx.x;
  for (int j = tid; j < C1_T + 7; j += 320) {
    const int pos = t0 + j;
    floatx4 v = {0.f, 0.f, 0.f, 0.f};
    if (pos < len) {
      if (x) {
        const float* xr = x + r * (4LL * len);
        v[0] = xr[pos];
        v[1] = xr[len + pos];
        v[2] = xr[2 * len + pos];
        v[3] = xr[3 * len + pos];
      } else {
        long long src = r;
        bool rc = (mode == EXPECTO_STRAND_RC);
        if (mode == EXPECTO_STRAND_BOTH && r >= n_src) {
          src = r - n_src;
          rc = true;
        }
        const int pp = rc ? (len - 1 - pos) : pos;
        const unsigned c = codes[src * code_stride + pp];
        if (c < 4) {
          const unsigned ch = rc ? 3 - c : c;
          v[0] = ch == 0 ? 1.f : 0.f;
          v[1] = ch == 1 ? 1.f : 0.f;
          v[2] = ch == 2 ? 1.f : 0.f;
          v[3] = ch == 3 ? 1.f : 0.f;
        }
      }
    }
    xs[j] = v;
  }
  __syncthreads();
  const int co = tid;
  float w[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) w[i] = w1[co * 32 + i];  // [ci*8 + k] as in the reference
  const float bco = b1[co];
  const int tmax = min(C1_T, len - 7 - t0);
  const long long orow = win * out_rows + t0;
  for (int t = 0; t < tmax; ++t) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const floatx4 v = xs[t + k];
      s = fmaf(w[k], v[0], s);
      s = fmaf(w[8 + k], v[1], s);
      s = fmaf(w[16 + k], v[2], s);
      s = fmaf(w[24 + k], v[3], s);
    }
    store_act_rt(fmt, out, orow + t, 320, co, fmaxf(s + bco, 0.f), osc, ovf);
  }
}

// conv1 on MFMA (f16x3 path).  One-hot inputs are exact in fp16, so conv1 is a K = 32 GEMM
// (k = tap*4 + channel) whose A row t is the 32 halves of positions t..t+7: per 16-row block a
// lane builds its A fragment (positions t + 2fq and t + 2fq + 1, 4 channels each) from two base
// codes in registers -- no im2col, no LDS read for A.  B = the conv1 weights as per-row scaled
// fp16 planes (hi, lo), held in registers: wave w owns output channels 64w..64w+63 (two 32-channel
// plane groups, 4 MFMA column blocks).  Products x_lo*w_hi (float inputs only: the 22-bit split
// of a one-hot value has x_lo = 0), x*w_lo, x*w_hi accumulate in fp32 -- the same arithmetic
// class as every other f16x3 layer, so codes and one-hot floats give the same bits.  Epilogue:
// unscale, bias, ReLU and the conv2-input scale in one FMA + max (the scales are powers of 2),
// canonical split, staged per wave through LDS so each row's two 128-B plane groups leave as
// 16-B stores (the VALU kernel's 2-byte stores and 32 FMAs per output were its limit).
// 5 waves; 256 output rows per workgroup in 32-row steps.
constexpr int C1H_ROWS = 256, C1H_STEP = 32;
constexpr int C1H_WROW = 2 * 128 + 16;   // staged bytes per row and wave (2 plane groups + pad)

__global__ __launch_bounds__(320) void beluga_conv1_h3(const float* __restrict__ x, const uint8_t* __restrict__ codes,
                                                       long long code_stride, int n_src, int mode, long long row0,
                                                       const _Float16* __restrict__ wpl, const float* __restrict__ cs1,
                                                       const float* __restrict__ b1, float* __restrict__ out,
                                                       int out_rows, int len, float osc, int* __restrict__ ovf) {
  __shared__ unsigned char cl[C1H_ROWS + 8];
  __shared__ __attribute__((aligned(16))) char stg[5][C1H_STEP * C1H_WROW];
  const int t0 = blockIdx.x * C1H_ROWS;
  const long long win = blockIdx.y;
  const long long r = row0 + win;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int T = len - 7;
  long long src = r;
  bool rc = (mode == EXPECTO_STRAND_RC);
  if (mode == EXPECTO_STRAND_BOTH && r >= n_src) {
    src = r - n_src;
    rc = true;
  }
  if (!x) {
    for (int j = tid; j < C1H_ROWS + 7; j += 320) {
      const int pos = t0 + j;
      unsigned c = 4;
      if (pos < len) {
        c = codes[src * code_stride + (rc ? len - 1 - pos : pos)];
        if (rc && c < 4) c = 3 - c;
      }
      cl[j] = (unsigned char)c;
    }
  }
  const int fr = lane & 15, fq = lane >> 4;
  halfx8 bh[4], bl[4];
  float sc[4], bb[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    const int n = 64 * wave + 16 * cb + fr;
    bh[cb] = *reinterpret_cast<const halfx8*>(wpl + n * 64 + 8 * fq);
    bl[cb] = *reinterpret_cast<const halfx8*>(wpl + n * 64 + 32 + 8 * fq);
    sc[cb] = cs1[n] * osc;
    bb[cb] = b1[n] * osc;
  }
  __syncthreads();
  char* const sw = stg[wave];
  float vmax = 0.f;
  bool bad = false;
  const int tend = min(C1H_ROWS, T - t0);
  for (int s = 0; s < tend; s += C1H_STEP) {
    floatx4v acc[2][4];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const int tr = s + 16 * rb + fr + 2 * fq;     // first of the lane's two positions (tile-relative)
      halfx8 ah, al;
      if (!x) {
        const unsigned c0 = cl[tr], c1 = cl[tr + 1];
        const u32x4 u = {onehot_h2(c0, 0), onehot_h2(c0, 1), onehot_h2(c1, 0), onehot_h2(c1, 1)};
        ah = __builtin_bit_cast(halfx8, u);
        al = halfx8{};
      } else {
        const float* xr = x + r * (4LL * len);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int pos = t0 + tr + (e >> 2);
          const float v = pos < len ? xr[(e & 3) * (long long)len + pos] : 0.f;
          bad |= !(fabsf(v) < 65504.f);   // out of fp16 range (or NaN): recomputed in bf16x6
          _Float16 h, l;
          split_h2(v, h, l);
          ah[e] = h;
          al[e] = l;
        }
      }
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        floatx4v c = {0.f, 0.f, 0.f, 0.f};
        if (x) c = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[cb], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[cb], c, 0, 0, 0);
        acc[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[cb], c, 0, 0, 0);
      }
    }
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float v = fmaxf(fmaf(acc[rb][cb][j], sc[cb], bb[cb]), 0.f);
          vmax = fmaxf(vmax, v);
          _Float16 h, l;
          split_h2p(v, h, l);
          char* d = sw + (16 * rb + 4 * fq + j) * C1H_WROW + (cb >> 1) * 128 + ((cb & 1) * 16 + fr) * 2;
          *reinterpret_cast<_Float16*>(d) = h;
          *reinterpret_cast<_Float16*>(d + 64) = l;
        }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < (C1H_STEP * 16) / 64; ++i) {   // 32 rows x 16 chunks of 16 B
      const int k = i * 64 + lane, row = k >> 4, ch = k & 15;
      if (s + row < tend) {
        char* g = reinterpret_cast<char*>(out) + ((win * out_rows + t0 + s + row) * 10 + 2 * wave) * 128 + ch * 16;
        *reinterpret_cast<floatx4*>(g) = *reinterpret_cast<const floatx4*>(sw + row * C1H_WROW + ch * 16);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if ((bad || !(vmax < 65504.f)) && ovf) *ovf = 1;
}

__global__ void fc1_reduce(const float* __restrict__ part, int splits, long long split_stride, long long count,
                           const float* __restrict__ bias, float* __restrict__ h1, int fmt,
                           const float* __restrict__ col_scale, float osc, int* __restrict__ ovf) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const long long row = i / kHidLd;
  const int n = (int)(i - row * kHidLd);
  float s = 0.f;
  for (int k = 0; k < splits; ++k) s += part[k * split_stride + i];
  if (col_scale) s *= col_scale[n];   // f16x3: exact power-of-2 unscaling of the split-K sum
  const float v = n < kFc1Out ? fmaxf(s + bias[n], 0.f) : 0.f;
  store_act_rt(fmt, h1, row, kHidLd, n, v, osc, ovf);
}

// fc1_reduce for f16x3 hidden rows, 4 columns per thread: float4 loads of the split-K slabs,
// 8-byte stores of the 4 hi and 4 lo halves (4 columns never straddle a 32-column plane group).
// Same per-element sum order, unscaling, bias, ReLU and split: bitwise equal to fc1_reduce.
typedef _Float16 halfx4 __attribute__((ext_vector_type(4)));
__global__ void fc1_reduce_h2(const float* __restrict__ part, int splits, long long split_stride, long long count4,
                              const float* __restrict__ bias, float* __restrict__ h1,
                              const float* __restrict__ col_scale, float osc, int* __restrict__ ovf) {
  const long long i4 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i4 >= count4) return;
  const long long i = i4 * 4;
  const long long row = i / kHidLd;
  const int n = (int)(i - row * kHidLd);
  floatx4 s = {0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < splits; ++k) {
    const floatx4 v = *reinterpret_cast<const floatx4*>(part + k * split_stride + i);
#pragma unroll
    for (int e = 0; e < 4; ++e) s[e] += v[e];
  }
  halfx4 hv, lv;
  bool bad = false;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float t = s[e];
    if (col_scale) t *= col_scale[n + e];
    const float v = n + e < kFc1Out ? fmaxf(t + bias[min(n + e, kFc1Out - 1)], 0.f) : 0.f;
    const float x = v * osc;
    bad |= !(fabsf(x) < 65504.f);
    _Float16 hh, ll;
    split_h2p(x, hh, ll);   // FC2 reads the planes as stored (no re-split): the plain split
    hv[e] = hh;
    lv[e] = ll;
  }
  if (bad && ovf) *ovf = 1;
  _Float16* d = reinterpret_cast<_Float16*>(h1) + act_index<2>(row, kHidLd, n);
  *reinterpret_cast<halfx4*>(d) = hv;
  *reinterpret_cast<halfx4*>(d + 32) = lv;
}

// FC2 output: y[c_rows[m] or m][n] = sigmoid(sum_k part[k][m][n] * col_scale[n] + bias[n]) (Beluga.py:46-48)
// HBM-bound (splits x 8 KB read per 8 KB row written).  Grid (kNFeat/512, row blocks): a
// thread takes 2 adjacent features (8-B loads and store, no 64-bit division for m / n) and
// issues a chunk's split loads before summing them; per value the same k-order sum, unscale,
// bias and sigmoid as the one-value-per-thread kernel it replaces.
constexpr int kFc2Chunk = 8;
__device__ __forceinline__ float fc2_value(float s, const float* __restrict__ col_scale, const float* __restrict__ bias,
                                           int n) {
  if (col_scale) s *= col_scale[n];   // f16x3: exact power-of-2 unscaling of the split-K sum
  const float v = s + bias[n];
  return 1.0f / (1.0f + expf(-v));
}
__global__ __launch_bounds__(256) void fc2_reduce(const float* __restrict__ part, int splits, long long split_stride,
                                                  int M, const float* __restrict__ bias,
                                                  const float* __restrict__ col_scale,
                                                  const long long* __restrict__ c_rows, float* __restrict__ y) {
  static_assert(kNFeat % 2 == 0 && kHidLd % 2 == 0, "2 features per thread");
  const int n = 2 * (blockIdx.x * blockDim.x + threadIdx.x);
  if (n >= kNFeat) return;
  for (long long m = blockIdx.y; m < M; m += gridDim.y) {
    const float* src = part + m * kHidLd + n;
    float s0 = 0.f, s1 = 0.f;
    for (int k0 = 0; k0 < splits; k0 += kFc2Chunk) {
      float2 v[kFc2Chunk];
#pragma unroll
      for (int u = 0; u < kFc2Chunk; ++u)
        v[u] = *reinterpret_cast<const float2*>(src + (long long)min(k0 + u, splits - 1) * split_stride);
#pragma unroll
      for (int u = 0; u < kFc2Chunk; ++u)
        if (k0 + u < splits) {
          s0 += v[u].x;
          s1 += v[u].y;
        }
    }
    float2 o;
    o.x = fc2_value(s0, col_scale, bias, n);
    o.y = fc2_value(s1, col_scale, bias, n + 1);
    *reinterpret_cast<float2*>(y + (c_rows ? c_rows[m] : m) * kNFeat + n) = o;
  }
}
// One value per thread, for an output pointer that is not 8-byte aligned (same values).
__global__ void fc2_reduce1(const float* __restrict__ part, int splits, long long split_stride, int M,
                            const float* __restrict__ bias, const float* __restrict__ col_scale,
                            const long long* __restrict__ c_rows, float* __restrict__ y) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)M * kNFeat) return;
  const int m = (int)(i / kNFeat), n = (int)(i - (long long)m * kNFeat);
  const long long src = (long long)m * kHidLd + n;
  float s = 0.f;
  for (int k = 0; k < splits; ++k) s += part[k * split_stride + src];
  y[(c_rows ? c_rows[m] : m) * kNFeat + n] = fc2_value(s, col_scale, bias, n);
}

// MaxPool(1,4) floor mode at pool phases p (segment path, SURVEY.md 5 "trunk sharing"):
// out[(seg*n_ph + i)*s_out + g][c] = max_{j<4} in[seg*s_in + ph[i] + 4g + j][c],
// g < (t_in - ph[i]) / 4.  ReLU was applied by the producing conv (Beluga.py:32-34 order).
// One thread per channel; on the bf16x6 path the values are recovered exactly from their
// planes, pooled, and re-split (so the planes equal those of the pooled fp32 value).
__global__ void pool4_phases(const float* __restrict__ in, int n_seg, int s_in, int t_in, int C,
                             int n_ph, int4 ph, int s_out, float* __restrict__ out, int fmt) {
  const int c = threadIdx.x;
  const int g = blockIdx.x;
  const int i = blockIdx.y % n_ph;
  const long long seg = blockIdx.y / n_ph;
  const int p = i == 0 ? ph.x : i == 1 ? ph.y : i == 2 ? ph.z : ph.w;
  if (c >= C || g >= (t_in - p) / 4) return;
  const long long r0 = seg * s_in + p + 4LL * g, orow = (seg * n_ph + i) * s_out + g;
  float m = load_act_rt(fmt, in, r0, C, c);
#pragma unroll
  for (int j = 1; j < 4; ++j) m = fmaxf(m, load_act_rt(fmt, in, r0 + j, C, c));
  store_act_rt(fmt, out, orow, C, c, m);   // fmt 2: values stay in the (shared) scaled domain
}

// pool4_phases for f16x3 rows (fmt 2), 16-byte accesses: a row of C channels is C/32 groups of
// [32 hi | 32 lo] fp16, so one thread takes 8 channels (16 B of hi + the matching 16 B of lo)
// of 4 input rows and writes 8 pooled channels; 4 pooled rows per 256-thread block.  The same
// decode (hi + lo), fmaxf order and canonical re-split as pool4_phases: bitwise equal.
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));
__global__ __launch_bounds__(256) void pool4_phases_h2(const float* __restrict__ in, int s_in, int t_in, int C,
                                                        int n_ph, int4 ph, int s_out, float* __restrict__ out) {
  const int c8 = threadIdx.x & 63;
  const int g = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int i = blockIdx.y % n_ph;
  const long long seg = blockIdx.y / n_ph;
  const int p = i == 0 ? ph.x : i == 1 ? ph.y : i == 2 ? ph.z : ph.w;
  if (c8 >= C / 8 || g >= (t_in - p) / 4) return;
  const long long rb = (long long)C * 4;   // bytes per row
  const int cofs = (c8 >> 2) * 128 + (c8 & 3) * 16;
  const char* src = reinterpret_cast<const char*>(in) + (seg * s_in + p + 4LL * g) * rb + cofs;
  halfx8 hi[4], lo[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    hi[j] = *reinterpret_cast<const halfx8*>(src + j * rb);
    lo[j] = *reinterpret_cast<const halfx8*>(src + j * rb + 64);
  }
  halfx8 oh, ol;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float m = (float)hi[0][e] + (float)lo[0][e];
#pragma unroll
    for (int j = 1; j < 4; ++j) m = fmaxf(m, (float)hi[j][e] + (float)lo[j][e]);
    _Float16 h, l;
    split_h2(m, h, l);
    oh[e] = h;
    ol[e] = l;
  }
  char* dst = reinterpret_cast<char*>(out) + ((seg * n_ph + i) * s_out + g) * rb + cofs;
  *reinterpret_cast<halfx8*>(dst) = oh;
  *reinterpret_cast<halfx8*>(dst + 64) = ol;
}

// pool4_phases_h2 for all n_ph phases of a segment in ONE pass: a thread takes pooled row g of
// every phase, so it reads the union of the phases' input rows once -- rows 4g + pmin ..
// 4g + pmax + 3 (the 200-bp shift sweep has phases {0, 2}: 6 rows instead of 2 x 4) -- and
// pools each phase from those registers with the same decode, fmaxf order and canonical re-split
// as pool4_phases_h2 (bitwise equal).  ph: the present phases, ascending (ph.x = pmin).
__global__ __launch_bounds__(256) void pool4_phases_h2m(const float* __restrict__ in, int s_in, int t_in, int C,
                                                         int n_ph, int4 ph, int s_out, float* __restrict__ out) {
  const int c8 = threadIdx.x & 63;
  const int g = blockIdx.x * 4 + (threadIdx.x >> 6);
  const long long seg = blockIdx.y;
  const int pmin = ph.x;
  const int pmax = n_ph == 1 ? ph.x : n_ph == 2 ? ph.y : n_ph == 3 ? ph.z : ph.w;
  if (c8 >= C / 8 || g >= (t_in - pmin) / 4) return;
  const long long rb = (long long)C * 4;   // bytes per row
  const int cofs = (c8 >> 2) * 128 + (c8 & 3) * 16;
  const char* src = reinterpret_cast<const char*>(in) + (seg * s_in + pmin + 4LL * g) * rb + cofs;
  const int nr = min(pmax - pmin + 4, t_in - pmin - 4 * g);   // rows of the union inside the layer
  halfx8 hi[7], lo[7];
#pragma unroll
  for (int j = 0; j < 7; ++j) {
    if (j < nr) {
      hi[j] = *reinterpret_cast<const halfx8*>(src + j * rb);
      lo[j] = *reinterpret_cast<const halfx8*>(src + j * rb + 64);
    }
  }
  float fv[7][8];                          // decoded union rows
#pragma unroll
  for (int j = 0; j < 7; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) fv[j][e] = j < nr ? (float)hi[j][e] + (float)lo[j][e] : 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (i >= n_ph) break;
    const int p = i == 0 ? ph.x : i == 1 ? ph.y : i == 2 ? ph.z : ph.w;
    if (g >= (t_in - p) / 4) continue;
    const int o = p - pmin;                // first union row of this phase's window (0..3)
    halfx8 oh, ol;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float m = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        // union row o + j (o is wave-uniform: selects, not a register-indexed read)
        const float v = o == 0 ? fv[j][e] : o == 1 ? fv[j + 1][e] : o == 2 ? fv[j + 2][e] : fv[j + 3][e];
        m = j == 0 ? v : fmaxf(m, v);
      }
      _Float16 h, l;
      split_h2(m, h, l);
      oh[e] = h;
      ol[e] = l;
    }
    char* dst = reinterpret_cast<char*>(out) + ((seg * n_ph + i) * s_out + g) * rb + cofs;
    *reinterpret_cast<halfx8*>(dst) = oh;
    *reinterpret_cast<halfx8*>(dst + 64) = ol;
  }
}

// FC1 row table of the windows of one segment chunk: window m of the chunk reads conv6
// rows [off6, off6+106) of block (segment, pool2 phase).
// (widx: optional list of window indices; row m then serves window widx[m].)
__global__ void seg_a_rows(const int* __restrict__ win_seg, const int* __restrict__ win_off,
                           const int* __restrict__ win_row, const int* __restrict__ widx, int w0, int m_count,
                           int seg_base, int rc, int seg_len, int n_ph, int4 ph_idx, int s7, long long row_base,
                           long long* __restrict__ a_rows, long long* __restrict__ c_rows) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= m_count) return;
  const int w = widx ? widx[m] : w0 + m;
  c_rows[m] = row_base + (win_row ? win_row[w] : w);
  const int o = rc ? seg_len - 2000 - win_off[w] : win_off[w];
  const int q = o >> 2, p = q & 3, off6 = (q - p) >> 2;
  const int pi = p == 0 ? ph_idx.x : p == 1 ? ph_idx.y : p == 2 ? ph_idx.z : ph_idx.w;
  const long long blk = (long long)(win_seg[w] - seg_base) * n_ph + pi;
  a_rows[m] = (blk * s7 + off6) * 640;
}

// ---- alt-cone reuse for SNV ref/alt window pairs (per-layer deltas) ---------------------
// An SNV at window index p changes only a few rows of each layer.  With the ref window's
// layer l-1 activations at hand (the ping-pong buffer holds them while layer l is computed
// for the ref windows) the alt window's layer l is obtained by recomputing a fixed-size run
// of W_l rows starting at r_l, from an "assembled" input patch: the ref rows of layer l-1
// with the alt's own recomputed rows of layer l-1 spliced in.  Rows outside [r_l, r_l+W_l)
// are unchanged (they see only unchanged inputs), so the alt conv6 output is the ref's with
// rows [r6, r6+20) replaced.  Every recomputed row uses the same operands, kernel and K order
// as the full forward -> bit-identical alt outputs (tests/test_gpu_pipelines.py).
//   layer    changed rows (from the previous run)          W     input rows (A patch)
//   conv1    [p-7, p]                                      8     15 codes
//   conv2+p  pooled [floor((r1-7)/4), floor((r1+7)/4)]     5     4*5+7 -> 28
//   conv3    [r2-7, r2+4]                                  12    19
//   conv4+p  pooled [floor((r3-7)/4), floor((r3+11)/4)]    6     4*6+7 -> 32
//   conv5    [r4-7, r4+5]                                  13    20
//   conv6    [r5-7, r5+12]                                 20    27
// Each start is clamped to [0, T_l - W_l] (T_l = valid rows of layer l), which keeps the run
// inside the layer and still covers every changed row.
constexpr int kDW[7] = {0, 8, 5, 12, 6, 13, 20};         // W_l, l = 1..6
constexpr int kDA[7] = {0, 15, 28, 19, 32, 20, 27};      // input rows of the layer-l patch
constexpr int kDT[7] = {0, 1993, 496, 489, 120, 113, 106};
constexpr int kDC[7] = {4, 320, 320, 480, 480, 640, 640};  // channels of layer l's output

struct DeltaRows {
  int r[7];    // r[l]: first recomputed row of layer l
  int base[7]; // base[l]: first row of layer l-1 in layer l's input patch
};

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
__device__ __forceinline__ int floor4(int v) { return v >= 0 ? v >> 2 : -((3 - v) >> 2); }

__device__ __forceinline__ DeltaRows delta_rows(int p) {
  DeltaRows d;
  d.r[0] = p;
  d.r[1] = clampi(p - 7, 0, kDT[1] - kDW[1]);
  d.r[2] = clampi(floor4(d.r[1] - 7), 0, kDT[2] - kDW[2]);
  d.r[3] = clampi(d.r[2] - 7, 0, kDT[3] - kDW[3]);
  d.r[4] = clampi(floor4(d.r[3] - 7), 0, kDT[4] - kDW[4]);
  d.r[5] = clampi(d.r[4] - 7, 0, kDT[5] - kDW[5]);
  d.r[6] = clampi(d.r[5] - 7, 0, kDT[6] - kDW[6]);
  d.base[0] = 0;
  d.base[1] = d.r[1];
  d.base[2] = 4 * d.r[2];
  d.base[3] = d.r[3];
  d.base[4] = 4 * d.r[4];
  d.base[5] = d.r[5];
  d.base[6] = d.r[6];
  return d;
}

// window m = strand * nv + (v - v0); SNV index in that strand's window coordinates
__device__ __forceinline__ int pair_pos(const int* var_pos, int m, int nv, int v0) {
  const int s = m / nv, v = v0 + m % nv;
  const int pv = min(max(var_pos[v], 0), kLen - 1);
  return s ? kLen - 1 - pv : pv;
}

// conv1 input of the alt run: 16 codes starting at r1 of the alt window (15 used).
__global__ void delta_codes(const uint8_t* __restrict__ alt, long long stride, int nv, int v0,
                            const int* __restrict__ var_pos, uint8_t* __restrict__ out, int R) {
  const int i = threadIdx.x & 15;
  const int m = blockIdx.x * (blockDim.x >> 4) + (threadIdx.x >> 4);
  if (m >= R) return;
  const int s = m / nv, v = v0 + m % nv;
  const int start = delta_rows(pair_pos(var_pos, m, nv, v0)).r[1];
  const uint8_t* a = alt + (long long)v * stride;
  const int pos = min(start + i, kLen - 1);
  uint8_t c;
  if (s) {
    const uint8_t f = a[kLen - 1 - pos];
    c = f < 4 ? (uint8_t)(3 - f) : f;
  } else {
    c = a[pos];
  }
  out[(long long)m * 16 + i] = c;
}

// Input patch of layer l (l = 2..6) for alt window m: rows base_l + i (i < kDA[l]) of the ref
// layer l-1 (row stride ref_rows per window), except rows inside [r_{l-1}, r_{l-1}+W_{l-1})
// which come from the alt run of layer l-1 (dprev, kDW[l-1] rows per window).  Rows are
// row16 16-byte lanes (fp32 rows or bf16 planes of the same channels).
// One block per alt window (all kDA[l] rows: 20-70 KB), so the copy runs near HBM rate.
__global__ __launch_bounds__(256) void delta_assemble(const float* __restrict__ ref, int ref_rows,
                                                      const float* __restrict__ dprev, int l, int row16, int nv, int v0,
                                                      const int* __restrict__ var_pos, float* __restrict__ out) {
  const int m = blockIdx.x;
  const DeltaRows d = delta_rows(pair_pos(var_pos, m, nv, v0));
  const int rp = d.r[l - 1], wp = kDW[l - 1];
  floatx4* to = reinterpret_cast<floatx4*>(out) + (long long)m * kDA[l] * row16;
  for (int k = threadIdx.x; k < kDA[l] * row16; k += blockDim.x) {
    const int i = k / row16, c = k - i * row16;
    const int src = min(d.base[l] + i, ref_rows - 1);   // rows past the window feed only invalid rows
    const floatx4* from = (src >= rp && src < rp + wp)
                              ? reinterpret_cast<const floatx4*>(dprev) + ((long long)m * wp + src - rp) * row16
                              : reinterpret_cast<const floatx4*>(ref) + ((long long)m * ref_rows + src) * row16;
    to[k] = from[c];
  }
}

// FC1 split-K slabs the alt run changes: alt window m differs from its ref window only in conv6
// rows [r6, r6+20), i.e. FC1 K range [640*r6, 640*(r6+20)); bit ks of mask[m / tile_rows] is
// set for every slab (slab_k wide) that range touches.  Slabs outside it have the same A rows
// as the ref windows, so their split-K partials (still in the partial buffer after the ref
// FC1 of the same rows and tiling) are already the alt ones, bit for bit.
__global__ void fc1_slab_mask(const int* __restrict__ var_pos, int nv, int v0, int R, int tile_rows, int slab_k,
                              unsigned* __restrict__ mask) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= R) return;
  const int r6 = delta_rows(pair_pos(var_pos, m, nv, v0)).r[6];
  const int k0 = r6 * 640, k1 = (r6 + kDW[6]) * 640 - 1;
  unsigned bits = 0;
  for (int ks = k0 / slab_k; ks <= k1 / slab_k; ++ks) bits |= 1u << ks;
  atomicOr(mask + m / tile_rows, bits);
}

// profiling: executed MACs of a masked FC1 = set slab bits x MACs per (tile, slab), summed into
// acc on the device (one wave; the host reads acc when the layer times are collected)
__global__ __launch_bounds__(64) void slab_macs(const unsigned* __restrict__ mask, int tiles, double per_bit,
                                                double* __restrict__ acc) {
  int bits = 0;
  for (int i = threadIdx.x; i < tiles; i += 64) bits += __popc(mask[i]);
  for (int o = 32; o > 0; o >>= 1) bits += __shfl_down(bits, o);
  if (threadIdx.x == 0) atomicAdd(acc, bits * per_bit);
}

// alt conv6 = ref conv6 (act6, 106 rows per window) with rows [r6, r6+20) from the alt run
__global__ __launch_bounds__(256) void pair_patch_apply(const float* __restrict__ d6, float* __restrict__ act6, int nv,
                                                        int v0, const int* __restrict__ var_pos, int row16) {
  const int m = blockIdx.x;
  const int r6 = delta_rows(pair_pos(var_pos, m, nv, v0)).r[6];
  const floatx4* src = reinterpret_cast<const floatx4*>(d6) + (long long)m * kDW[6] * row16;
  floatx4* dst = reinterpret_cast<floatx4*>(act6) + ((long long)m * 106 + r6) * row16;
  for (int k = threadIdx.x; k < kDW[6] * row16; k += blockDim.x) dst[k] = src[k];
}

// ---- alt deltas on the segment path (shift sweeps) -------------------------------------
// Same idea as the pair path, in segment coordinates: the alt segment differs from the ref
// segment at one base q (q' = L-1-q on the reverse-complement strand).  conv1..conv3 runs as
// above; conv4 is unpooled on the segment path, so its run is the 19 rows [r4u, r4u+19); each
// pool2 phase p then changes <= 6 pooled rows [r4p, r4p+6) and conv5 / conv6 runs follow per
// (segment, phase) block.  Starts are clamped with the phase-0 (longest) geometry, like the
// ref blocks; rows past a phase's valid length are never read by any window.
// Per-segment table (kSegTab ints): q', r1, r2, r3, r4u, r4p[4], r5[4], r6[4].
constexpr int kSegTab = 20;
constexpr int kW4u = 19, kA4u = 26;   // conv4 run [r3 - 7, r3 + 12): the 12 changed conv3 rows' reach
struct SegDims {
  int L, T1, P1, T3, T4, S5, T5, T6;
};

__global__ void seg_delta_table(const int* __restrict__ var_pos, int s0, int ns, int rc, SegDims g, int n_ph, int4 ph,
                                int* __restrict__ tab) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= ns) return;
  int q = min(max(var_pos[s0 + m], 0), g.L - 1);
  if (rc) q = g.L - 1 - q;
  int* t = tab + m * kSegTab;
  const int r1 = clampi(q - 7, 0, g.T1 - kDW[1]);
  const int r2 = clampi(floor4(r1 - 7), 0, g.P1 - kDW[2]);
  const int r3 = clampi(r2 - 7, 0, g.T3 - kDW[3]);
  const int r4 = clampi(r3 - 7, 0, g.T4 - kW4u);
  t[0] = q;
  t[1] = r1;
  t[2] = r2;
  t[3] = r3;
  t[4] = r4;
  for (int i = 0; i < n_ph; ++i) {
    const int p = i == 0 ? ph.x : i == 1 ? ph.y : i == 2 ? ph.z : ph.w;
    // pooled rows g of phase p read conv4 rows p+4g .. p+4g+3: the changed ones meet [r4, r4+19)
    const int r4p = clampi(floor4(r4 - p), 0, g.S5 - kDW[4]);
    const int r5 = clampi(r4p - 7, 0, g.T5 - kDW[5]);
    t[5 + i] = r4p;
    t[9 + i] = r5;
    t[13 + i] = clampi(r5 - 7, 0, g.T6 - kDW[6]);
  }
}

// 16 codes from r1 of the alt segment, in the strand's orientation (rc: mirrored, complemented)
__global__ void seg_delta_codes(const uint8_t* __restrict__ codes, long long stride, const uint8_t* __restrict__ alt_code,
                                int s0, int ns, int rc, int L, const int* __restrict__ tab, uint8_t* __restrict__ out) {
  const int i = threadIdx.x & 15;
  const int m = blockIdx.x * (blockDim.x >> 4) + (threadIdx.x >> 4);
  if (m >= ns) return;
  const int q = tab[m * kSegTab], x = min(tab[m * kSegTab + 1] + i, L - 1);
  uint8_t c = x == q ? alt_code[s0 + m] : codes[(long long)(s0 + m) * stride + (rc ? L - 1 - x : x)];
  if (rc && c < 4) c = (uint8_t)(3 - c);
  out[(long long)m * 16 + i] = c;
}

// conv1 fused into conv2 (f16x3): the ref conv1 planes are never stored, so the alt conv2 patch
// (kDA[2] conv1 rows from 4*r2) is conv1 of the alt codes [4*r2, 4*r2 + kDA[2] + 7) -- every row
// computed from the alt sequence, which is the ref row where the SNV is outside its 8 taps, bit
// for bit (conv1 is row-local).  kC1Pat codes per block at a kC1PatStride stride, code 4 (N) past
// the segment end; seg_delta_codes2 for segments (strand orientation, as seg_delta_codes),
// delta_codes2 for the pair path's alt windows (as delta_codes).
constexpr int kC1Pat = kDA[2] + 7, kC1PatStride = 48;
__global__ void seg_delta_codes2(const uint8_t* __restrict__ codes, long long stride, const uint8_t* __restrict__ alt_code,
                                 int s0, int ns, int rc, int L, const int* __restrict__ tab, uint8_t* __restrict__ out) {
  const int i = threadIdx.x % kC1PatStride;
  const int m = blockIdx.x * (blockDim.x / kC1PatStride) + threadIdx.x / kC1PatStride;
  if (m >= ns) return;
  const int q = tab[m * kSegTab], x = 4 * tab[m * kSegTab + 2] + i;
  uint8_t c = 4;
  if (i < kC1Pat && x < L) {
    c = x == q ? alt_code[s0 + m] : codes[(long long)(s0 + m) * stride + (rc ? L - 1 - x : x)];
    if (rc && c < 4) c = (uint8_t)(3 - c);
  }
  out[(long long)m * kC1PatStride + i] = c;
}

__global__ void delta_codes2(const uint8_t* __restrict__ alt, long long stride, int nv, int v0,
                             const int* __restrict__ var_pos, uint8_t* __restrict__ out, int R) {
  const int i = threadIdx.x % kC1PatStride;
  const int m = blockIdx.x * (blockDim.x / kC1PatStride) + threadIdx.x / kC1PatStride;
  if (m >= R) return;
  const int s = m / nv, v = v0 + m % nv;
  const int pos = 4 * delta_rows(pair_pos(var_pos, m, nv, v0)).r[2] + i;
  const uint8_t* a = alt + (long long)v * stride;
  uint8_t c = 4;
  if (i < kC1Pat && pos < kLen) {
    if (s) {
      const uint8_t f = a[kLen - 1 - pos];
      c = f < 4 ? (uint8_t)(3 - f) : f;
    } else {
      c = a[pos];
    }
  }
  out[(long long)m * kC1PatStride + i] = c;
}

// Input patch of one alt run: rows base + i (i < arows) of ref block m (ref_rows rows per
// block), except rows inside [rp, rp + wprev), taken from the previous alt run.  Blocks are
// segments (nb = 1) or (segment, phase) pairs (nb = n_ph, per-phase table entries).
// base = mult * tab[ib (+ phase)], rp = tab[irp (+ phase)].
__global__ __launch_bounds__(256) void seg_delta_assemble(const float* __restrict__ ref, int ref_rows,
                                                          const float* __restrict__ dprev, int wprev,
                                                          const int* __restrict__ tab, int nb, int ib, int mult, int irp,
                                                          int arows, int row16, float* __restrict__ out) {
  const int m = blockIdx.x;
  const int seg = m / nb, off = nb > 1 ? m % nb : 0;
  const int base = mult * tab[seg * kSegTab + ib + off], rp = tab[seg * kSegTab + irp + off];
  floatx4* to = reinterpret_cast<floatx4*>(out) + (long long)m * arows * row16;
  for (int k = threadIdx.x; k < arows * row16; k += blockDim.x) {
    const int i = k / row16, c = k - i * row16;
    const int src = min(base + i, ref_rows - 1);   // rows past the block feed only invalid rows
    const floatx4* from = (src >= rp && src < rp + wprev)
                              ? reinterpret_cast<const floatx4*>(dprev) + ((long long)m * wprev + src - rp) * row16
                              : reinterpret_cast<const floatx4*>(ref) + ((long long)m * ref_rows + src) * row16;
    to[k] = from[c];
  }
}

// pool2 of the alt run for each phase: pooled rows [r4p, r4p+6) of block (seg, phase) from the
// ref's unpooled conv4 rows and the alt conv4 run (exact max, as pool4_phases)
// (edge != 0: conv4 holds only the ref rows this kernel reads, kSegEdge per segment from the first
// one, the fused conv4 + pool2 epilogue's layout, gemm_kernel.h epilogue_pool_ph02)
constexpr int kSegEdge = 32;
__device__ __forceinline__ int seg_edge_lo(const int* t) { return min(4 * t[5], 2 + 4 * t[6]); }
__global__ void seg_delta_pool(const float* __restrict__ conv4, int t4, const float* __restrict__ d4, int n_ph,
                               int4 ph, const int* __restrict__ tab, int fmt, float* __restrict__ out, int edge = 0) {
  const int c = threadIdx.x;
  if (c >= 480) return;
  const int gi = blockIdx.x, m = blockIdx.y;
  const int seg = m / n_ph, i = m % n_ph;
  const int p = i == 0 ? ph.x : i == 1 ? ph.y : i == 2 ? ph.z : ph.w;
  const int r4 = tab[seg * kSegTab + 4];
  const int row0 = p + 4 * (tab[seg * kSegTab + 5 + i] + gi);
  const int elo = edge ? seg_edge_lo(tab + seg * kSegTab) : 0;
  float mx = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = row0 + j;
    const bool alt = row >= r4 && row < r4 + kW4u;
    const float* b = alt ? d4 : conv4;
    const long long r = alt    ? (long long)seg * kW4u + row - r4
                        : edge ? (long long)seg * kSegEdge + row - elo
                               : (long long)seg * t4 + row;
    const float v = load_act_rt(fmt, b, r, 480, c);
    mx = j == 0 ? v : fmaxf(mx, v);
  }
  store_act_rt(fmt, out, (long long)m * kDW[4] + gi, 480, c, mx);
}

// The phase-2 pooled row whose 4 conv4 rows straddle two 256-row tiles of the fused conv4 + pool2
// launch (epilogue_pool_ph02 leaves it): from the two tiles' edge rows (seam: 4 rows per tile, its
// rows 0, 1, 254, 255, plain split), pooled as pool4_phases_h2m does (decode, fmaxf in row order,
// canonical split).  One workgroup per tile boundary b = 256 k, rows b - 2 .. b + 1.
__global__ void pool2_tile_seams(const float* __restrict__ seam, long long M, int s_in, int t4, int s5,
                                 float* __restrict__ out) {
  const int c8 = threadIdx.x;   // 60 eight-channel pieces
  if (c8 >= 60) return;
  const long long k = blockIdx.x + 1, b = 256 * k;
  if (b + 1 >= M) return;
  const long long w = (b - 2) / s_in;   // segment blocks of s_in rows (4-aligned), t4 of them valid
  const int t = (int)(b - 2 - w * s_in), g = (t - 2) >> 2;
  if (t + 3 >= t4) return;   // the group would leave its segment's valid rows: no such pooled row
  constexpr long long rb = 480 * 4;
  const int cofs = (c8 >> 2) * 128 + (c8 & 3) * 16;
  const char* sb = reinterpret_cast<const char*>(seam);
  const char* src[4] = {sb + ((k - 1) * 4 + 2) * rb, sb + ((k - 1) * 4 + 3) * rb, sb + (k * 4 + 0) * rb,
                        sb + (k * 4 + 1) * rb};
  halfx8 oh, ol;
  float m[8];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const halfx8 hv = *reinterpret_cast<const halfx8*>(src[j] + cofs), lv = *reinterpret_cast<const halfx8*>(src[j] + cofs + 64);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float v = (float)hv[e] + (float)lv[e];
      m[e] = j == 0 ? v : fmaxf(m[e], v);
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    _Float16 h, l;
    split_h2(m[e], h, l);
    oh[e] = h;
    ol[e] = l;
  }
  char* dst = reinterpret_cast<char*>(out) + ((2 * w + 1) * s5 + g) * rb + cofs;
  *reinterpret_cast<halfx8*>(dst) = oh;
  *reinterpret_cast<halfx8*>(dst + 64) = ol;
}

// alt conv6 phase blocks: the ref block (t6 rows) with rows [r6, r6+20) from the alt run.  Only
// the rows some alt window reads are written: a window at offset o (strand orientation) holds the
// SNV at q iff o <= q < o + 2000, and reads rows [o/16, o/16 + 106) of its phase block, so every
// alt window lies in [(q-1999)/16, q/16 + 106) -- at most kAltRows6 rows (was: the whole block,
// 2 x 425 MB per chunk of the 200-window workload).
constexpr int kAltRows6 = 232;   // ceil(1999/16) + 106 + 1
__global__ void seg_alt_blocks(const float* __restrict__ ref6, const float* __restrict__ d6, int n_ph, int t6,
                               const int* __restrict__ tab, int row16, float* __restrict__ out) {
  const int m = blockIdx.y;
  const int q = tab[(m / n_ph) * kSegTab];
  const int t = (q >= 1999 ? (q - 1999) >> 4 : 0) + blockIdx.x;
  if (t >= t6 || t >= (q >> 4) + 106) return;
  const int r6 = tab[(m / n_ph) * kSegTab + 13 + m % n_ph];
  const floatx4* src = (t >= r6 && t < r6 + kDW[6])
                           ? reinterpret_cast<const floatx4*>(d6) + ((long long)m * kDW[6] + t - r6) * row16
                           : reinterpret_cast<const floatx4*>(ref6) + ((long long)m * t6 + t) * row16;
  floatx4* dst = reinterpret_cast<floatx4*>(out) + ((long long)m * t6 + t) * row16;
  for (int c = threadIdx.x; c < row16; c += blockDim.x) dst[c] = src[c];
}

// FC1 split-K slabs the alt windows of a segment chunk change (FC row m = window widx[m]; cf.
// fc1_slab_mask): the window reads conv6 rows [off6, off6+106) of block (segment, pool2
// phase), whose alt run replaced block rows [r6, r6+20) (seg_delta_table), so its FC1 K range
// that changed is 640 x that intersection.
__global__ void fc1_slab_mask_seg(const int* __restrict__ widx, int n_alt, const int* __restrict__ win_seg,
                                  const int* __restrict__ win_off, int seg_base, int rc, int seg_len, int4 ph_idx,
                                  const int* __restrict__ tab, int tile_rows, int slab_k, unsigned* __restrict__ mask) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n_alt) return;
  const int w = widx[m];
  const int o = rc ? seg_len - 2000 - win_off[w] : win_off[w];
  const int q = o >> 2, p = q & 3, off6 = (q - p) >> 2;
  const int pi = p == 0 ? ph_idx.x : p == 1 ? ph_idx.y : p == 2 ? ph_idx.z : ph_idx.w;
  const int r6 = tab[(win_seg[w] - seg_base) * kSegTab + 13 + pi];
  const int lo = max(r6 - off6, 0), hi = min(r6 + kDW[6] - off6, 106);
  if (lo >= hi) return;
  unsigned bits = 0;
  for (int ks = lo * 640 / slab_k; ks <= (hi * 640 - 1) / slab_k; ++ks) bits |= 1u << ks;
  atomicOr(mask + m / tile_rows, bits);
}

// y_alt rows of windows whose alt sequence equals the ref one (the SNV lies outside them)
__global__ void copy_rows(const float* __restrict__ src, float* __restrict__ dst, const int* __restrict__ widx,
                          const int* __restrict__ win_row, long long row_base) {
  const int w = widx[blockIdx.x];
  const long long r = (row_base + (win_row ? win_row[w] : w)) * kNFeat;
  for (int i = threadIdx.x; i < kNFeat; i += blockDim.x) dst[r + i] = src[r + i];
}

__global__ void pair_rows(long long* __restrict__ c_rows, int M, int nv, int v0, long long strand_stride) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m < M) c_rows[m] = (long long)(m / nv) * strand_stride + v0 + m % nv;
}

// ---- FC1 as a block-Karatsuba convolution (f16x3, round 5) ---------------------------------
// FC1 (Beluga.py:43-44) of a window reads its 106 conv6 rows x[0..105] as y = sum_{q<4} V_q X_q +
// T x[100..105], with X_q the 25-row block x[25q .. 25q+24] and V_q the matching 2003 x 16000
// slice of the weights.  On a 200-bp shift sweep, windows 400 bp apart in one pool2-phase block
// are 25 conv6 rows apart, so 4 such windows y_a (a = 0..3, blocks X_{a..a+3} of one sequence) are
// a 4-tap convolution over blocks, and two nested Karatsuba steps (F(2,2) x F(2,2)) give them
// from 9 block products instead of 16 (-41 % of FC1's multiply-adds on the headline):
//   m0 = V0 DD@0        m1 = (V0+V1) D2@1       m2 = -V1 DD@1
//   m3 = (V0+V2) D1@2   m4 = (V0+V1+V2+V3) X@3  m5 = -(V1+V3) D1@3
//   m6 = -V2 DD@2       m7 = -(V2+V3) D2@3      m8 = V3 DD@3
//   y0 = m0+m1+m3+m4   y1 = m1+m2+m4+m5   y2 = m3+m4+m6+m7   y3 = m4+m5+m7+m8   (+ the tail each)
// with S@b the rows 25b .. 25b+24 (from the group's first window) of the row sequences
//   D1[r] = x[r] - x[r+25],  D2[r] = x[r] - x[r+50],  DD[r] = (x[r] - x[r+25]) - (x[r+50] - x[r+75]).
// Every product of window a's sum reads only rows of window a itself, so a window can be computed
// alone in its role a (its position in the group: (conv6 offset / 25) mod 4): the per-window
// forwards use role 0 (EXPECTO_FC1_ROLE), the segment path gives each window the role of its
// offset and shares each group's products, and every path computes a window's FC1 as the same
// sum of the same partial products -- bitwise equal (tests/test_gpu_fc1_karatsuba.py).  Weights
// of the 9 products are formed once per handle in fp64 and rounded to fp32 once; the sequences
// are formed in fp32 from the stored f16x3 planes and stored as planes (22-bit) like any
// activation.  tests/test_fc1_karatsuba_identity.py checks the algebra in float64.
constexpr int kFkK = 16000;                        // one 25-row block of conv6 rows (25 x 640)
constexpr int kFkKb = kFkK / GBK;                  // 500 K blocks
constexpr int kFkSlabs = 2;                        // K slabs per product (250 K blocks, as FC1's 265)
constexpr int kFkTailK = kFc1In - 4 * kFkK;        // 3840: rows 100..105
constexpr int kFkKbTotal = 9 * kFkKb + kFkTailK / GBK;   // 4620 K blocks per weight row
constexpr long long kFkKTotal = 9LL * kFkK + kFkTailK;   // 147,840
constexpr int kFkSeq[9] = {3, 2, 3, 1, 0, 1, 3, 2, 3};   // product g reads sequence (0 x, 1 D1, 2 D2, 3 DD)
constexpr int kFkBlk[9] = {0, 1, 1, 2, 3, 3, 2, 3, 3};   //   at block kFkBlk[g] of its group
constexpr int kFkRole[4][4] = {{0, 1, 3, 4}, {1, 2, 4, 5}, {3, 4, 6, 7}, {4, 5, 7, 8}};
constexpr int kFkW[9][4] = {{1, 0, 0, 0}, {1, 1, 0, 0}, {0, -1, 0, 0}, {1, 0, 1, 0}, {1, 1, 1, 1},
                            {0, -1, 0, -1}, {0, 0, -1, 0}, {0, 0, -1, -1}, {0, 0, 0, 1}};   // V_q coefficients
constexpr int kFkParts = 4 * kFkSlabs + 1;         // partial rows a window's FC1 sums (8 + the tail)

// Karatsuba FC1 weights (fp32, K = 9 x 16000 + 3840 per row) from the repacked FC1 weights
// (w1 [rows][67840], K = t*640 + c): product g's row = sum_q kFkW[g][q] V_q in fp64, then the tail.
__global__ void fk_weights(const float* __restrict__ w1, long long rows, float* __restrict__ wk) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * kFkKTotal) return;
  const long long n = i / kFkKTotal;
  const int k = (int)(i - n * kFkKTotal);
  const float* wr = w1 + n * kFc1In;
  if (k >= 9 * kFkK) {
    wk[i] = wr[4 * kFkK + (k - 9 * kFkK)];
    return;
  }
  const int g = k / kFkK, kk = k - g * kFkK;
  double s = 0.0;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (kFkW[g][q]) s += kFkW[g][q] * (double)wr[q * kFkK + kk];
  wk[i] = (float)s;
}

// The row sequences D1, D2, DD of f16x3 conv6 rows (x: blocks of `s` rows, the first T valid):
// row r of a block gets D1 / D2 / DD where its last input row r + 25 / 50 / 75 is in [lo, hi).
// (gres: only the rows the block's groups read.)  Values from the stored planes (x = hi + lo), fp32 arithmetic in a fixed order, plain split (the
// planes are consumed as stored), the overflow flag as any f16x3 store.  [lo, hi) = [0, T), or
// with `tab` (segment pairs: the alt blocks seg_alt_blocks filled, n_ph blocks per segment) the
// rows that alt block holds.  320 threads = 4 rows x 80 eight-channel pieces (16 B of hi + 16 B of lo).
__global__ __launch_bounds__(320) void fk_seq_h2(const float* __restrict__ x, int T, int s, const int* __restrict__ tab,
                                                 int n_ph, const int* __restrict__ gres, float* __restrict__ d1,
                                                 float* __restrict__ d2, float* __restrict__ dd, int* __restrict__ ovf) {
  // a thread walks one residue class k of a block's rows (k, k + 25, k + 50, ...) for one
  // eight-channel piece, holding x[r .. r + 75 step 25] in registers: every row is loaded once
  // (workgroup: 4 residues x 80 pieces; 7 workgroups cover the 25 residues of a block)
  const int c8 = threadIdx.x % 80;
  const long long blk = blockIdx.x / 7;
  const int k = (int)(blockIdx.x - blk * 7) * 4 + threadIdx.x / 80;
  if (k >= 25) return;
  int lo = 0, hi = T;
  if (tab) {
    const int q = tab[(blk / n_ph) * kSegTab];
    lo = q >= 1999 ? (q - 1999) >> 4 : 0;
    hi = min(T, (q >> 4) + 106);
  }
  // gres (optional): the block's group starts are all = gres[blk] mod 100 (>= 0; -1: unknown; -2: the
  // block has no windows), so the products read D1 only at group rows 50..99 and D2 at 25..49 and
  // 75..99 (DD at all rows)
  const int g = gres ? gres[blk] : -1;
  if (g == -2) return;
  int r = k;
  if (r < lo) r += (lo - r + 24) / 25 * 25;
  if (r + 25 >= hi) return;
  constexpr long long rb = 640 * 4;   // bytes per row (20 groups of [32 hi | 32 lo] fp16)
  const long long base = blk * s * rb + (c8 >> 2) * 128 + (c8 & 3) * 16;
  auto ld = [&](int row, float (&v)[8]) {
    const char* p = reinterpret_cast<const char*>(x) + base + row * rb;
    const halfx8 h = *reinterpret_cast<const halfx8*>(p);
    const halfx8 l = *reinterpret_cast<const halfx8*>(p + 64);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (float)h[e] + (float)l[e];
  };
  bool bad = false;
  auto put = [&](float* dst, int row, const float (&y)[8]) {
    halfx8 h, l;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      bad |= !(fabsf(y[e]) < 65504.f);
      _Float16 a, b;
      split_h2p(y[e], a, b);
      h[e] = a;
      l[e] = b;
    }
    // Full-line stores: the 8 lanes of a lane octet (c8 = 8m .. 8m+7, one row) own channel groups
    // 2m' and 2m'+1 (4 eight-channel quarters each).  Each keeps one plane and trades the other with
    // its mirror lane j <-> 7 - j (DPP row_half_mirror): the low half keeps hi, the high half keeps
    // lo.  Then one store instruction writes group 2m' as whole 128-B lines [hi q0..q3 | lo q0..q3]
    // and the next group 2m'+1 -- instead of two half-line stores per group (the same bytes).
    const int j = c8 & 7;
    const bool low = j < 4;
    u32x4 send = __builtin_bit_cast(u32x4, low ? l : h), recv;
#pragma unroll
    for (int w = 0; w < 4; ++w) recv[w] = (unsigned)__builtin_amdgcn_update_dpp(0, (int)send[w], 0x141, 0xf, 0xf, false);
    const u32x4 keep = __builtin_bit_cast(u32x4, low ? h : l);
    char* d = reinterpret_cast<char*>(dst) + blk * s * rb + row * rb + (c8 >> 3) * 256;
    auto st = [](char* p, const u32x4& v) { *reinterpret_cast<u32x4*>(p) = v; };
    if (low) {   // hi quarter j of group 2m' (own), hi quarter 3 - j of group 2m'+1 (mirror's)
      st(d + j * 16, keep);
      st(d + 128 + (3 - j) * 16, recv);
    } else {     // lo quarter 7 - j of group 2m' (mirror's), lo quarter j - 4 of group 2m'+1 (own)
      st(d + 64 + (7 - j) * 16, recv);
      st(d + 128 + 64 + (j - 4) * 16, keep);
    }
  };
  float v0[8], v1[8], v2[8] = {}, v3[8] = {};
  ld(r, v0);
  ld(r + 25, v1);
  if (r + 50 < hi) ld(r + 50, v2);
  if (r + 75 < hi) ld(r + 75, v3);
  for (; r + 25 < hi; r += 25) {
    float nv[8] = {};
    if (r + 100 < hi) ld(r + 100, nv);   // the next row of the walk, in flight while this one is stored
    bool need1 = true, need2 = true;
    if (g >= 0) {
      const int rel = ((r - g) % 100 + 100) % 100;
      need1 = rel >= 50;
      need2 = (rel >= 25 && rel < 50) || rel >= 75;
    }
    float a[8], y[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] = v0[e] - v1[e];
    if (need1) put(d1, r, a);
    if (r + 50 < hi && need2) {
#pragma unroll
      for (int e = 0; e < 8; ++e) y[e] = v0[e] - v2[e];
      put(d2, r, y);
    }
    if (r + 75 < hi) {
#pragma unroll
      for (int e = 0; e < 8; ++e) y[e] = a[e] - (v2[e] - v3[e]);
      put(dd, r, y);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v0[e] = v1[e];
      v1[e] = v2[e];
      v2[e] = v3[e];
      v3[e] = nv[e];
    }
  }
  if (bad) *ovf = 1;
}

// FC1 output rows of the block Karatsuba: row m = sum of its kFkParts partial rows prow[m][j] (its
// 4 products x 2 K slabs in product order, then the tail), unscaled, + bias, ReLU, f16x3 planes
// for FC2 (the same per-element steps as fc1_reduce_h2).  4 columns per thread.
__global__ void fk_reduce_h2(const float* __restrict__ part, const int* __restrict__ prow, long long count4,
                             const float* __restrict__ bias, float* __restrict__ h1, const float* __restrict__ col_scale,
                             float osc, int* __restrict__ ovf) {
  const long long i4 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i4 >= count4) return;
  const long long row = i4 / (kHidLd / 4);
  const int n = (int)(i4 - row * (kHidLd / 4)) * 4;
  floatx4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < kFkParts; ++j) {
    const floatx4 v = *reinterpret_cast<const floatx4*>(part + (long long)prow[row * kFkParts + j] * kHidLd + n);
#pragma unroll
    for (int e = 0; e < 4; ++e) s[e] += v[e];
  }
  halfx4 hv, lv;
  bool bad = false;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float t = s[e] * col_scale[n + e];
    const float v = n + e < kFc1Out ? fmaxf(t + bias[min(n + e, kFc1Out - 1)], 0.f) : 0.f;
    const float x = v * osc;
    bad |= !(fabsf(x) < 65504.f);
    _Float16 hh, ll;
    split_h2p(x, hh, ll);
    hv[e] = hh;
    lv[e] = ll;
  }
  if (bad && ovf) *ovf = 1;
  _Float16* d = reinterpret_cast<_Float16*>(h1) + act_index<2>(row, kHidLd, n);
  *reinterpret_cast<halfx4*>(d) = hv;
  *reinterpret_cast<halfx4*>(d + 32) = lv;
}

// Per-window block Karatsuba (every window alone in role `role`, its 106 rows at m * rstride rows):
// group starts g_rows[m] = (m * rstride - 25 role) * 640, window starts w_rows[m] = m * rstride * 640,
// partial rows of window m: (2j + s) * M + m for its j-th product and slab s, then 8 M + m.
__global__ void fk_window_tables(int M, int rstride, int role, long long* __restrict__ g_rows,
                                 long long* __restrict__ w_rows, int* __restrict__ prow) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  g_rows[m] = ((long long)m * rstride - 25LL * role) * 640;
  w_rows[m] = (long long)m * rstride * 640;
#pragma unroll
  for (int j = 0; j < kFkParts; ++j) prow[(long long)m * kFkParts + j] = j * M + m;
}

// Alt masks of the per-window block Karatsuba (pair path): window m's alt conv6 differs from its
// ref rows only in [r6, r6 + 20) (window rows), so partial (product j, slab s) -- sequence rows
// 25 (blk - role) + [13 s - (s ? 1 : 0), 13 s + 12] with their lags -- and the tail (rows 100..105)
// are recomputed only where a dependency row falls in that run: bit 0 of mask[d * tiles + m / 256]
// for descriptor d = 2j + s (8 = the tail).  Unset descriptors keep the ref partials in place.
__global__ void fk_window_mask(const int* __restrict__ var_pos, int nv, int v0, int R, int role, int tiles,
                               unsigned* __restrict__ mask) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= R) return;
  const int r6 = delta_rows(pair_pos(var_pos, m, nv, v0)).r[6], r6e = r6 + kDW[6];
  for (int j = 0; j < 4; ++j) {
    const int g = kFkRole[role][j], sq = kFkSeq[g];
    const int nl = sq == 0 ? 1 : sq == 3 ? 4 : 2;
    const int lag1 = sq == 2 ? 50 : 25;
    for (int s = 0; s < kFkSlabs; ++s) {
      // K elements [s * 8000, (s + 1) * 8000) of the product = its rows [12.5 s, 12.5 (s + 1))
      const int i0 = 25 * (kFkBlk[g] - role) + (s * 8000) / 640, i1 = 25 * (kFkBlk[g] - role) + ((s + 1) * 8000 - 1) / 640;
      bool hit = false;
      for (int l = 0; l < nl; ++l) {
        const int lag = l == 0 ? 0 : (nl == 2 ? lag1 : 25 * l);
        hit |= i0 + lag < r6e && i1 + lag >= r6;
      }
      if (hit) atomicOr(mask + (2 * j + s) * tiles + m / 256, 1u);
    }
  }
  if (100 < r6e && 105 >= r6) atomicOr(mask + 8 * tiles + m / 256, 1u);
}

// Alt masks of the segment path's in-place alt FC1 (segment pairs): descriptor slot d of the ref
// layout (product g, slab s: rows i < cnt are groups rgrp[off + i], each (block, start row) in ginfo;
// the last slot: the tail over windows i < nw, (block, conv6 offset) in winfo) is recomputed for the
// M tiles holding a row whose partial reads -- the product's rows with its sequence's lags, or the
// tail's rows 100..105 -- meet its block's changed conv6 rows [r6, r6 + 20) (seg_delta_table).
struct FkMaskDesc {
  int n;
  int g[18], s[18], off[18], cnt[18];
  int nw;
};
__global__ void fk_seg_mask(FkMaskDesc md, const int* __restrict__ rgrp, const int* __restrict__ ginfo,
                            const int* __restrict__ winfo, const int* __restrict__ tab, int n_ph, int4 ph_unused,
                            int tiles, unsigned* __restrict__ mask) {
  const int d = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  auto r6_of = [&](int blk) { return tab[(blk / n_ph) * kSegTab + 13 + blk % n_ph]; };
  if (d == md.n) {   // the tail
    if (i >= md.nw) return;
    const int r6 = r6_of(winfo[2 * i]), o = winfo[2 * i + 1];
    if (o + 100 < r6 + kDW[6] && o + 105 >= r6) atomicOr(mask + (size_t)d * tiles + i / 256, 1u);
    return;
  }
  if (i >= md.cnt[d]) return;
  const int g = md.g[d], s = md.s[d], k = rgrp[md.off[d] + i];
  const int r6 = r6_of(ginfo[2 * k]), r6e = r6 + kDW[6];
  const int base = ginfo[2 * k + 1] + 25 * kFkBlk[g];
  const int i0 = base + (s * 8000) / 640, i1 = base + ((s + 1) * 8000 - 1) / 640;
  const int sq = kFkSeq[g], nl = sq == 0 ? 1 : sq == 3 ? 4 : 2, lag1 = sq == 2 ? 50 : 25;
  bool hit = false;
  for (int l = 0; l < nl; ++l) {
    const int lag = l == 0 ? 0 : (nl == 2 ? lag1 : 25 * l);
    hit |= i0 + lag < r6e && i1 + lag >= r6;
  }
  if (hit) atomicOr(mask + (size_t)d * tiles + i / 256, 1u);
}

// ---- weight repacking (reference layouts -> kernel layouts) --------------------------
__global__ void repack_conv(const float* __restrict__ W, int cout, int cin, int npad, float* __restrict__ Wt) {
  const long long K = 8LL * cin;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npad * K) return;
  const int n = (int)(i / K);
  const int k = (int)(i % K);  // kernel K order [ci/32][tap][ci%32] (cin is a multiple of 32)
  const int chunk = k / (8 * GBK), tap = (k / GBK) % 8, ci = chunk * GBK + k % GBK;
  Wt[i] = n < cout ? W[((long long)n * cin + ci) * 8 + tap] : 0.f;
}

__global__ void repack_conv1(const float* __restrict__ w1, float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;   // out index n*32 + tap*4 + ci
  if (i >= 320 * 32) return;
  const int n = i >> 5, k = i & 31, tap = k >> 2, ci = k & 3;
  out[i] = w1[n * 32 + ci * 8 + tap];
}

__global__ void repack_fc1(const float* __restrict__ W, int npad, float* __restrict__ Wp) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)npad * kFc1In) return;
  const int o = (int)(i / kFc1In);
  const int k = (int)(i % kFc1In);
  const int t = k / 640, c = k % 640;  // kernel order t*640+c <- reference flatten c*106+t
  Wp[i] = o < kFc1Out ? W[(long long)o * kFc1In + c * 106 + t] : 0.f;
}

__global__ void repack_fc2(const float* __restrict__ W, int npad, float* __restrict__ Wp) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)npad * kHidLd) return;
  const int o = (int)(i / kHidLd);
  const int k = (int)(i % kHidLd);
  Wp[i] = (o < kNFeat && k < kFc1Out) ? W[(long long)o * kFc1Out + k] : 0.f;
}

__global__ void pad_copy(const float* __restrict__ src, int n, int npad, float* __restrict__ dst) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < npad) dst[i] = i < n ? src[i] : 0.f;
}

// ---- f16x3 scaling --------------------------------------------------------------------
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// s_w[n] = 15 - e with max_k |W[n][k]| = m * 2^e (m in [0.5, 1)): the row's largest weight
// lands in [2^14, 2^15) after scaling.  All-zero (padding) rows get 0.
__global__ void row_scale_exp(const float* __restrict__ W, int K, int* __restrict__ sw) {
  __shared__ float red[4];
  const long long n = blockIdx.x;
  float m = 0.f;
  for (int k = threadIdx.x; k < K; k += blockDim.x) m = fmaxf(m, fabsf(W[n * K + k]));
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    int e = 0;
    (void)frexpf(m, &e);
    sw[n] = m > 0.f ? 15 - e : 0;
  }
}

// col_scale[n] = 2^-(s_in + s_w[n]): undoes both operand scales of a GEMM column exactly
__global__ void col_scales(const int* __restrict__ sw, int n, int s_in, float* __restrict__ cs) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) cs[i] = ldexpf(1.f, -(s_in + sw[i]));
}

// max over the valid rows (t_valid of every s_rows) and first C channels of a bf16x6-format
// activation buffer (non-negative: every boundary follows a ReLU), as float bits
__global__ void act_max(const float* __restrict__ A, long long groups, int s_rows, int t_valid, int ld, int C,
                        unsigned* __restrict__ out) {
  const long long rows = groups * t_valid;
  float m = 0.f;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < rows * C;
       i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / C;
    const int c = (int)(i - r * C);
    const long long row = (r / t_valid) * s_rows + r % t_valid;
    m = fmaxf(m, load_act<1>(A, row, ld, c));
  }
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) atomicMax(out, __float_as_uint(m));
}

__device__ __forceinline__ unsigned mix32(unsigned x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// Seeded calibration windows (A/G/C/T codes), a mix of what real genomes hold: half i.i.d.
// random windows, a quarter low-complexity tandem repeats (per 256-bp stretch one motif of
// period 1-6 repeated: homopolymer runs, (CA)n, (CAG)n, (GGGGCC)n-like), a quarter tandem copies
// of a block of 64-320 bp.  Repeats make every filter that matches the repeat fire at every
// position of a window, which random windows never do, so the f16x3 scales cover them too.
__global__ void calib_codes(uint8_t* __restrict__ codes, long long n, unsigned seed) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned w = (unsigned)(i / 2000), p = (unsigned)(i % 2000);
  const unsigned kind = mix32(w * 0x9e3779b9u ^ seed) & 3u;
  unsigned src = (unsigned)i;
  if (kind == 2) {                 // tandem repeat of a short motif, a new motif every 256 bp
    const unsigned h = mix32((w << 4 | (p >> 8)) * 0x85ebca6bu ^ seed);
    const unsigned period = 1 + h % 6;
    src = w * 2000u + (p >> 8) * 256u + (p % period);
  } else if (kind == 3) {          // tandem copies of one block
    const unsigned len = 64 + mix32(w ^ seed ^ 0xabcdu) % 257;
    src = w * 2000u + p % len;
  }
  codes[i] = (uint8_t)(mix32(src * 2654435761u ^ seed) & 3u);
}

}  // namespace expecto

using namespace expecto;


// ---- conv1 + ReLU + conv2 as a k-mer table (f16x3 and bf16x6, base-code inputs) ----------
// Conv1 (k = 8) sees 8 bases, so relu(conv1) at position p is a function of the 8-mer at p, and
// conv2 (k = 8) at p is  sum_{j<8} W2_j relu(conv1(p + j)) = sum_{i<4} T_i(9-mer at p + 2i)  with
//   T_i(x_0..x_8) = W2_{2i} relu(conv1(x_0..x_7)) + W2_{2i+1} relu(conv1(x_1..x_8))
// (Beluga.py:23-26 regrouped: a tap pair shares 9 bases).  Over the code alphabet A,G,C,T,N (N =
// the zero one-hot column, chromatin.py:155-160) the 4 pair tables T_i have 5^9 rows of 320 values
// each (10.0 GB fp32); the 2 quad tables Q_h (kmer_quad: taps 4h..4h+3 over 11-mers of A,G,C,T,
// 10.7 GB) halve the gathers again: 20.7 GB in all (kKmerFloats).  Built once per weight set in fp64 -- the conv1 sums, the 320-deep conv2
// products and the pair / quad sums -- and rounded to fp32 once.  The conv2 + pool1 layer of every
// f16x3 / bf16x6 forward from codes then is a gather (conv2_kmer_pool): a pooled row reads 8 table
// rows (4 conv2 rows x 2 tap quads, 10 KB) and adds them, in place of 4 x 819,200 multiply-adds x
// 3 f16x3 products on the MFMAs.  The tables are MORE accurate than the MFMA path (one fp32
// rounding per entry and one to three fp32 adds per conv2 value, against 22-bit operands and a
// 2,560-long fp32 accumulation); every path (per
// window, segments, pairs, the alt-delta patches) computes a conv2 row by this one formula from
// its codes, so the paths stay bitwise equal to each other.
constexpr int kMer8 = 390625;           // 5^8
constexpr long long kMer9 = 1953125LL;  // 5^9
constexpr long long kMer11 = 4194304LL; // 4^11: the quad tables cover A, G, C, T only
constexpr size_t kKmerFloats = (4 * (size_t)kMer9 + 2 * (size_t)kMer11) * 320;   // pair + quad tables, 20.7 GB

// F[m8][c] = relu(conv1) of 8-mer m8 (digit k = code at tap k, base 5), fp64
__global__ __launch_bounds__(320) void kmer_conv1(const float* __restrict__ w1, const float* __restrict__ b1,
                                                  double* __restrict__ F) {
  const int m8 = blockIdx.x, co = threadIdx.x;
  double s = b1[co];
  int v = m8;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int d = v % 5;
    v /= 5;
    if (d < 4) s += (double)w1[co * 32 + d * 8 + k];   // reference layout [320][4][1][8]
  }
  F[(long long)m8 * 320 + co] = s > 0.0 ? s : 0.0;
}

// G[m8][co] = sum_ci W2[co][ci][tap] F[m8][ci] in fp64 (wt0: the repacked conv2 weights,
// [co][ci/32][tap][ci%32]); 64 x 64 tiles, 4 x 4 outputs per thread
__global__ __launch_bounds__(256) void kmer_conv2(const double* __restrict__ F, const float* __restrict__ wt0, int tap,
                                                  double* __restrict__ G) {
  __shared__ double fs[16][65], ws[16][65];
  const int m0 = blockIdx.x * 64, n0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  double acc[4][4] = {};
  for (int k0 = 0; k0 < 320; k0 += 16) {
    for (int e = threadIdx.x; e < 16 * 64; e += 256) {
      const int r = e >> 4, c = e & 15, ci = k0 + c;
      const int m = m0 + r;
      fs[c][r] = m < kMer8 ? F[(long long)m * 320 + ci] : 0.0;
      ws[c][r] = (double)wt0[(long long)(n0 + r) * 2560 + (ci >> 5) * 256 + tap * 32 + (ci & 31)];
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      double a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a[i] = fs[c][ty + 16 * i];
        b[i] = ws[c][tx + 16 * i];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fma(a[i], b[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + ty + 16 * i;
    if (m >= kMer8) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) G[(long long)m * 320 + n0 + tx + 16 * j] = acc[i][j];
  }
}

// T[m9][co] = fp32(Ga[first 8-mer of m9][co] + Gb[last 8-mer][co]); the digits of m9 are the
// codes x_0..x_8 (base 5, x_0 lowest), so the first 8-mer is m9 % 5^8 and the last m9 / 5
__global__ void kmer_pair(const double* __restrict__ Ga, const double* __restrict__ Gb, float* __restrict__ T) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= kMer9 * 320) return;
  const long long m9 = e / 320;
  const int co = (int)(e - m9 * 320);
  T[e] = (float)(Ga[(m9 % kMer8) * 320 + co] + Gb[(m9 / 5) * 320 + co]);
}

// Quad tables (round 4): Q_h(y_0..y_10) = sum_{t<4} W2_{4h+t} F(y_t..y_{t+7}), h = 0, 1 -- taps 0-3
// and 4-7 of conv2, so a conv2 row is Q_0(11-mer at p) + Q_1(11-mer at p + 4): 2 table rows
// instead of 4.  Over A, G, C, T only (4^11 rows each; 5^11 would be 62.5 GB a table): a
// conv2 half whose 11-mer holds an N takes the two pair tables instead.  The fp64 sum over the
// four taps (tap order) is rounded to fp32 once.  G: all 8 taps, [tap][5^8][320].
__global__ void kmer_quad(const double* __restrict__ G, int h, float* __restrict__ Q) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= kMer11 * 320) return;
  const long long m11 = e / 320;
  const int co = (int)(e - m11 * 320);
  int d[11];
#pragma unroll
  for (int k = 0; k < 11; ++k) d[k] = (int)((m11 >> (2 * k)) & 3);
  double sum = 0.0;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    int i5 = 0;
#pragma unroll
    for (int k = 7; k >= 0; --k) i5 = i5 * 5 + d[t + k];
    sum += G[((long long)(4 * h + t) * kMer8 + i5) * 320 + co];
  }
  Q[e] = (float)sum;
}

// conv2 + bias + ReLU + maxpool4 of `rows` pooled rows per window from base codes (window w =
// code row row0 + w, strand mode as beluga_conv1_h3, code 4 past len), gathered from the k-mer
// table; output: the f16x3 planes of the pooled rows (scaled by osc = 2^sx[1], plain split, as
// the MFMA conv2's epilogue stores them; bf16x6: the exact 3-way bf16 split), row w * s_out + g.  640 threads = 8 pooled rows x 80
// channel quads; a conv2 row is Q_0 + Q_1 (2 16-B loads per quad, each from one 1,280-B table
// row), a half whose 11-mer holds an N (T_0 + T_1) or (T_2 + T_3).
constexpr int KP_ROWS = 8;
__global__ __launch_bounds__(640) void conv2_kmer_pool(const uint8_t* __restrict__ codes, long long stride, int n_src,
                                                       int mode, long long row0, int len, int rows, int row_blocks,
                                                       int s_out, const float* __restrict__ T,
                                                       const float* __restrict__ b2, float osc, int quad, int fmt,
                                                       float* __restrict__ out, int* __restrict__ ovf) {
  __shared__ unsigned char cl[4 * KP_ROWS + 16];
  __shared__ int ix[4 * KP_ROWS + 8];    // 9-mer (base 5) at offset o
  __shared__ int iq[4 * KP_ROWS + 8];    // 11-mer (base 4) at offset o, -1 if it holds an N
  const long long win = blockIdx.x / row_blocks;
  const int g0 = (int)(blockIdx.x - win * row_blocks) * KP_ROWS;
  const int tid = threadIdx.x;
  long long src = row0 + win;
  bool rc = mode == EXPECTO_STRAND_RC;
  if (mode == EXPECTO_STRAND_BOTH && src >= n_src) {
    src -= n_src;
    rc = true;
  }
  const int p0 = 4 * g0;
  if (tid < 4 * KP_ROWS + 15) {   // bases p0 .. p0 + 4*KP_ROWS + 14: the block's 9-mers at p0 + o, o < 4*KP_ROWS + 6
    const int pos = p0 + tid;
    unsigned c = 4;
    if (pos < len) {
      c = codes[src * stride + (rc ? len - 1 - pos : pos)];
      c = c < 4 ? (rc ? 3 - c : c) : 4;   // any code >= 4 is the zero column (as conv1 reads it): rows stay in the table
    }
    cl[tid] = (unsigned char)c;
  }
  __syncthreads();
  if (tid < 4 * KP_ROWS + 6) {
    int v = 0;
#pragma unroll
    for (int k = 8; k >= 0; --k) v = v * 5 + cl[tid + k];
    ix[tid] = v;
  } else if (tid >= 64 && tid < 64 + 4 * KP_ROWS + 4) {
    const int o = tid - 64;
    int v = 0;
    bool n = false;
#pragma unroll
    for (int k = 10; k >= 0; --k) {
      n |= cl[o + k] > 3;
      v = v * 4 + (cl[o + k] & 3);
    }
    iq[o] = n || !quad ? -1 : v;
  }
  __syncthreads();
  const int lr = tid / 80, q = tid - lr * 80, g = g0 + lr;
  if (g >= rows) return;
  const float* Q = T + 4 * kMer9 * 320;
  auto row = [&](const float* base, long long r) { return *reinterpret_cast<const floatx4*>(base + r * 320 + 4 * q); };
  floatx4 hv2[4][2];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int o = 4 * lr + r + 4 * h, k = iq[o];
      if (k >= 0)
        hv2[r][h] = row(Q + h * kMer11 * 320, k);
      else
        hv2[r][h] = row(T + 2 * h * kMer9 * 320, ix[o]) + row(T + (2 * h + 1) * kMer9 * 320, ix[o + 2]);
    }
  const floatx4 bb = *reinterpret_cast<const floatx4*>(b2 + 4 * q);
  floatx4 m;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const floatx4 s = hv2[r][0] + hv2[r][1];
#pragma unroll
    for (int c = 0; c < 4; ++c) m[c] = r == 0 ? s[c] : fmaxf(m[c], s[c]);
  }
  floatx4 v;
  float vmax = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    v[c] = fmaxf(fmaf(m[c], osc, bb[c] * osc), 0.f);   // maxpool(relu(x + b)) = relu(max(x) + b), scaled
    vmax = fmaxf(vmax, v[c]);
  }
  if (fmt == 1) {   // bf16x6 planes [row][C/32][3][32] (osc = 1): the exact 3-way split, as store_act<1>
    bf16x4 x0, x1, x2;
    split3(v, x0, x1, x2);
    char* d = reinterpret_cast<char*>(out) + ((win * s_out + g) * 10 + (q >> 3)) * 192 + (q & 7) * 8;
    *reinterpret_cast<bf16x4*>(d) = x0;
    *reinterpret_cast<bf16x4*>(d + 64) = x1;
    *reinterpret_cast<bf16x4*>(d + 128) = x2;
    return;
  }
  const halfx4 hv = __builtin_convertvector(v, halfx4);
  const halfx4 lv = __builtin_convertvector(v - __builtin_convertvector(hv, floatx4), halfx4);
  char* d = reinterpret_cast<char*>(out) + ((win * s_out + g) * 10 + (q >> 3)) * 128 + (q & 7) * 8;
  *reinterpret_cast<halfx4*>(d) = hv;
  *reinterpret_cast<halfx4*>(d + 64) = lv;
  if (!(vmax < 65504.f)) *ovf = 1;   // out of fp16 range: the call is recomputed (bf16x6)
}

// Beluga.forward's input (x[n][4][len] fp32, Beluga.py:50-51) as base codes: a column holding
// exactly one 1.0f and three +0.0f is that channel's code (A, G, C, T = channels 0..3 as encodeSeqs
// writes them, chromatin.py:155-160), an all-zero column is code 4 (N).  Any other column (another
// value, -0.0f, NaN, two ones) sets *bad: the call then keeps conv1 / conv2 on the MFMAs.  codes
// may be null (check only).  4 positions per thread, a 16-B load per channel (x 16-B aligned and
// len % 4 == 0, checked by the caller); HBM-bound, 32 KB read per window.
__global__ __launch_bounds__(256) void onehot_codes(const float* __restrict__ x, long long n, int len,
                                                    uint8_t* __restrict__ codes, int* __restrict__ bad) {
  const int len4 = len >> 2;
  const long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n * len4) return;
  const long long w = q / len4;
  const int p = (int)(q - w * len4) * 4;
  const float* xr = x + w * 4LL * len + p;
  unsigned b[4][4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const floatx4 v = *reinterpret_cast<const floatx4*>(xr + (long long)c * len);
#pragma unroll
    for (int e = 0; e < 4; ++e) b[c][e] = __float_as_uint(v[e]);
  }
  bool ok = true;
  unsigned packed = 0;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    unsigned code = 4, ones = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (b[c][e] == 0x3f800000u) {
        ++ones;
        code = c;
      } else if (b[c][e] != 0u) {
        ok = false;
      }
    }
    ok &= ones <= 1;
    packed |= code << (8 * e);
  }
  if (!ok) *bad = 1;
  if (codes) *reinterpret_cast<unsigned*>(codes + w * len + p) = packed;
}

// ---- handle -----------------------------------------------------------------------------
namespace {
constexpr int kNumLayers = 9;
struct ConvGeo {
  int cin, cout, s_in, t_valid, s_out, pool;
};
// conv2..conv6 (index 0..4) -- positions from SURVEY.md section 0 item 3.  Row strides per
// window are the valid rows, rounded up to a multiple of 4 where a pool epilogue follows
// (so a pool group never straddles two windows): 1993->1996, 489->492.
constexpr int kS1 = 1996;  // conv1 output rows per window (1993 valid)
constexpr ConvGeo kConv[5] = {
    {320, 320, kS1, 496, 496, 1},  // conv2: 1986 valid -> pool 496
    {320, 480, 496, 489, 492, 0},  // conv3
    {480, 480, 492, 120, 120, 1},  // conv4: 482 valid -> pool 120
    {480, 640, 120, 113, 113, 0},  // conv5
    {640, 640, 113, 106, 106, 0},  // conv6 -> FC1 reads 106*640 = 67840 contiguous floats
};
// FC1 split-K: a fixed number of slabs per handle (default 8 of 8480; a divisor of
// 67840/32 = 2120 K blocks), whatever the batch, so an FC1 output never depends on how many
// windows shared the launch.
constexpr int kFc2SplitsDefault = 7;   // FC2 K = 63 blocks of 32 -> 7 slabs of 9: a 2000-row FC2 fills
                                        // 728 workgroups instead of 104 (fixed: sums never depend on M)
constexpr int kFcSplitsDefault = 8;    // round 2 sweep (tools/knob_sweep.py, interleaved): 8 vs 20 slabs
                                       // +0.6-0.9 % on the 200-window workload, +0.3-1.2 % on configs[1]
                                       // (4: -0.6 / -3.7 %), with 2.5x less split-K partial traffic
}  // namespace

struct expecto_beluga {
  int device = 0;
  int max_batch = 0;
  float* w1 = nullptr;
  float* b1 = nullptr;
  float* wt[5] = {};
  float* bt[5] = {};
  float* fc1w = nullptr;
  float* fc1b = nullptr;
  float* fc2w = nullptr;
  float* fc2b = nullptr;
  float* wp[5] = {};             // bf16x6: weight planes of conv2..6, FC1, FC2 (split_planes)
  float* fc1p = nullptr;
  float* fc2p = nullptr;
  // f16x3 (built on the first switch to it): fp16 weight planes of the 7 GEMM layers (conv2..6,
  // FC1, FC2), their per-channel scale exponents, per-column unscale factors, the calibrated
  // activation scale exponents sx[g] of GEMM layer g's input (sx[0] = conv1 output), and the
  // device overflow flag.
  float* wh[7] = {};
  int* swd[7] = {};
  float* w1h = nullptr;          // conv1 on MFMA: fp16 planes [320][hi 32 | lo 32] (k = tap*4 + ci),
  float* cs1 = nullptr;          //   per-row unscale 2^-s_w[n] (one-hot input: no input scale)
  float* cs[7] = {};
  int sx[7] = {};
  int f16_target = 10;
  bool f16_ready = false;
  int* ovf = nullptr;
  bool ovf_deferred = false;     // leave the flag for expecto_beluga_overflow_pending (no sync per call)
  float* calib = nullptr;        // calibration windows' codes, outputs and maxima
  long long fallbacks = 0;
  // Host tables of a segment call go through pinned staging (two slots, each reused once the
  // event after its copies has fired), so the call returns without a host sync.
  void* stage_buf[2] = {};
  size_t stage_cap[2] = {};
  hipEvent_t stage_ev[2] = {};
  int stage_next = 0;
  double* macs_d = nullptr;      // executed-MAC counters summed on the device (alt FC1 slab share)
  float* P = nullptr;
  float* Q = nullptr;
  float* part = nullptr;
  float* part2 = nullptr;        // FC2 split-K partials (fc2_splits slabs; FC1's stay in `part`)
  float* h1 = nullptr;          // FC1 output rows: fc2_rows (+ max_batch alt rows) of the segment path
  long long* a_rows = nullptr;  // FC1 row table (segment path), max_batch entries
  long long* c_rows = nullptr;  // FC2 output-row table (segment path), fc2_rows + max_batch entries
  int fc2_rows = 0;             // segment path, FC2 unsplit: h1 rows gathered per FC2 launch
  int* win_seg_d = nullptr;     // window tables of the current segment call
  int* alt_w_d = nullptr;       //   segment pairs: windows holding the SNV / the others
  int* copy_w_d = nullptr;
  int* seg_var_d = nullptr;     //   segment pairs: SNV index per segment
  int seg_var_cap = 0;
  int* win_off_d = nullptr;
  int* win_row_d = nullptr;
  int* fc_perm_d = nullptr;      // segment pairs: FC row order per strand (2 x win_cap)
  hipStream_t st2 = nullptr;     // pair path: alt-delta launches overlap the ref launches
  hipEvent_t pev[16] = {};       //   (ordering events, no timing)
  bool overlap = true;           //   EXPECTO_OVERLAP=0: one stream (same bits either way)
  float* DA = nullptr;           // alt-delta buffers (pair path), lazily allocated:
  float* D0 = nullptr;           //   DA = assembled input patch, D0/D1 = alternating W_l-row runs
  float* D1 = nullptr;
  uint8_t* delta_codes = nullptr;
  int* seg_tab = nullptr;        //   per-segment delta rows (segment pairs)
  float* slab_mask = nullptr;    //   alt FC1 split-K slab mask per M tile (pair path)
  int win_cap = 0;
  size_t bytes = 0;
  std::vector<void*> allocs;
  int precision = EXPECTO_PRECISION_BF16X6;
  int fc_splits = kFcSplitsDefault;   // FC1 split-K slabs: a divisor of 2120 K blocks, <= 32
  int fc2_splits = kFc2SplitsDefault; // FC2 split-K slabs: a divisor of 63 K blocks
  double fc1_m_order_mb = 80.0;       // FC1 dispatch: M tiles fastest while one split's A is <= this
  int fc1_order = 3;                  // FC1 dispatch order (EXPECTO_FC1_ORDER): 3 grouped M tiles (default),
                                      // 0 M-fastest / N-fastest by A-slab size, 2 slab-outermost
  int fc1_m_group = 8;                // order 3: M tiles per group (EXPECTO_FC1_M_GROUP)
  bool fc_wide = true;                // f16x3 FC split-K GEMMs on 336-column tiles (EXPECTO_FC_WIDE; same bits)
  int conv_tile = 0;                  // f16x3 conv M tile: 0 = auto (conv_tile_rows), 256 or 384
  bool conv_ea = true;                // f16x3 conv consumers' early next-stage reads (EXPECTO_CONV_EA)
  bool fc_skinny = true;              // FC1 / FC2 of <= 32 rows on 32 x 32 tiles (EXPECTO_FC_SKINNY; same bits)
  int fc1_narrow = -1;                // grouped FC1 tile width: -1 auto (fc1_narrow), 0 336, 1 112 columns
  int conv_narrow = -1;               // conv5 / conv6 tile width: -1 auto (conv_narrow), 0 160, 1 64 columns
  bool narrow_scope = false;          // inside forward_chunk: auto narrow tiles allowed (nothing runs beside)
  int seg_chunk_windows = 0;          // segment path: windows per chunk cap (0 = none; tuning knob)
  int cus = 0;                        // compute units of the device (workgroups per round)
  bool pool_one_pass = true;          // segment path: pool2 of all phases in one pass (same bits)
  bool pool_fused = true;             // segment path, phases {0, 2}: pool2 in conv4's epilogue (EXPECTO_POOL_FUSED; same bits)
  float* seam = nullptr;              //   its tile-seam rows (4 per 256-row tile) and seg_delta_pool's ref rows
  float* edge = nullptr;
  size_t seam_cap = 0, edge_cap = 0;
  bool fuse_conv1 = true;             // f16x3 codes input: conv1 inside the conv2 launch (EXPECTO_FUSE_CONV1; same bits)
  bool kmer_on = true;                // f16x3 codes input: conv1 + conv2 + pool1 from the k-mer table (EXPECTO_CONV2_TABLE)
  float* kmer = nullptr;              //   the table (shared by handles with the same conv1 / conv2 weights)
  uint64_t kmer_key = 0;
  bool kmer_quad = true;              //   conv2 rows from the quad tables (EXPECTO_KMER_QUAD=0: pair tables only)
  int kmer_state = 1;                 //   0 held, 1 off (EXPECTO_CONV2_TABLE=0), 2 no room (conv2_table_active)
  bool fk_on = true;                  // f16x3 FC1 as a block-Karatsuba convolution (EXPECTO_FC1_KARATSUBA)
  int fk_role = 4;                    //   role of per-window forwards (EXPECTO_FC1_ROLE; 4 = direct FC1, the default; 0..3 Karatsuba)
  float* fkw = nullptr;               //   the 9 products' + tail weight planes [npad][kFkKbTotal][2][32] fp16
  int* fk_sw = nullptr;               //   their per-row scale exponents
  float* fk_cs = nullptr;             //   column unscale 2^-(sx[5] + fk_sw[n])
  float* fk_seq[3] = {};              //   row sequences D1, D2, DD (x's row layout), fk_seq_rows rows each
  long long fk_seq_rows = 0;
  long long* fk_grows = nullptr;      //   group starts (per product), window starts, partial rows, alt masks
  long long* fk_wrows = nullptr;
  int* fk_prow = nullptr;
  unsigned* fk_mask = nullptr;
  int fk_slice = 24576;               //   windows per Karatsuba FC1 launch on the segment path (EXPECTO_FC1K_SLICE):
  float* fk_part = nullptr;           //   its partial rows, FC1 output rows, window / output rows, block residues
  float* fk_h1 = nullptr;
  long long* fk_arows = nullptr;
  long long* fk_crows = nullptr;
  int* fk_gres = nullptr;
  long long fk_gres_cap = 0;
  float* fk_aseq[3] = {};             //   segment pairs' in-place alt FC1: the alt blocks' sequences, row groups
  long long fk_aseq_rows = 0;
  int* fk_rgrp = nullptr;             //   of the product rows, group / window (block, row), alt windows'
  int* fk_ginfo = nullptr;            //   partial rows and order, masks
  int* fk_winfo = nullptr;
  int* fk_aprow = nullptr;
  int* fk_aperm = nullptr;
  unsigned* fk_smask = nullptr;
  bool onehot_as_codes = true;        // forward_onehot: exact one-hot input through the k-mer gather (EXPECTO_ONEHOT_CODES)
  uint8_t* oh_codes = nullptr;        //   its codes, max_batch x 2000 (allocated on first use)
  int* oh_bad = nullptr;              //   its check flag
  bool oh_hint_bad = false;           //   the last input was not one-hot: check first instead of a speculative run
  int* hflags = nullptr;              // pinned, device-mapped host words the per-call checks read their flags into
  int* hflags_d = nullptr;            //   their device address (take_flags writes them: no blit kernels per call)
  bool profiling = false;
  std::vector<hipEvent_t> ev_pool;
  std::vector<std::pair<int, int>> pending;  // (layer, event index of start)
  size_t ev_next = 0;
  // timing slots 0..8: the layers of every forward; 9..17: the same layers' alt-delta launches
  // (pair / segment-pair paths), kept apart so a slot's launches are those of one kernel shape
  int timer_base = 0;            // kNumLayers while an alt-delta run is being launched
  double ms[2 * kNumLayers] = {};
  long long calls[2 * kNumLayers] = {};
  double macs[2 * kNumLayers] = {};  // executed multiply-adds per slot while profiling (host-side count)
  // the conv GEMM launches alone (no pool2 pass in the slot), per (layer slot, rows): bench.py's
  // roofline takes the group with the most rows, i.e. the full-size launches
  struct LaunchRec {
    int layer;
    long long rows;
    int idx;
    double macs;
  };
  std::vector<LaunchRec> pending_launch;
  std::map<std::pair<int, long long>, std::array<double, 3>> launch_stats;   // ms, calls, macs
};

namespace {
int dalloc(expecto_beluga* h, float** p, size_t nfloat) {
  void* ptr = nullptr;
  hipError_t e = hipMalloc(&ptr, nfloat * sizeof(float));
  if (e != hipSuccess) {
    set_error(std::string("hipMalloc: ") + hipGetErrorString(e));
    return EXPECTO_ENOMEM;
  }
  // zero-filled: rows a kernel reads past a layer's valid rows (padded strides, the last window's
  // Toeplitz tail) then hold finite values before any layer wrote them
  e = hipMemset(ptr, 0, nfloat * sizeof(float));
  if (e != hipSuccess) {
    (void)hipFree(ptr);
    set_error(std::string("hipMemset: ") + hipGetErrorString(e));
    return EXPECTO_EHIP;
  }
  h->allocs.push_back(ptr);
  h->bytes += nfloat * sizeof(float);
  *p = static_cast<float*>(ptr);
  return EXPECTO_OK;
}

int npad_of(int n) { return (n + GBN - 1) / GBN * GBN; }

// Process-wide k-mer tables: handles of one device with the same conv1 / conv2 weights share one
// (tests and benches create many handles of one seeded model); refcounted, freed with the last.
struct KmerEntry {
  int device;
  uint64_t key;
  std::vector<float> w;   // the conv1 / conv2 weights the tables were built from (exact match, not just the hash)
  float* T;
  std::vector<const expecto_beluga*> holders;   // the first one reports the bytes (expecto_beluga_device_bytes)
};
std::mutex g_kmer_mu;
std::vector<KmerEntry> g_kmer;

uint64_t fnv1a(const void* p, size_t n, uint64_t hsh = 1469598103934665603ULL) {
  const unsigned char* b = static_cast<const unsigned char*>(p);
  for (size_t i = 0; i < n; ++i) hsh = (hsh ^ b[i]) * 1099511628211ULL;
  return hsh;
}

// Build (or share) the handle's k-mer table from its conv1 weights (w1, b1) and repacked conv2
// weights.  If its 20.7 GB (plus 9 GB of fp64 scratch while building) do not fit, or exceed
// EXPECTO_KMER_MAX_BYTES, the handle runs conv2 on the MFMAs instead (kmer stays null,
// kmer_state 2, one line on stderr; expecto_beluga_conv2_table_active reports it).
int kmer_no_room(expecto_beluga* h, const char* why) {
  h->kmer_state = 2;
  fprintf(stderr, "expecto_hip: no k-mer tables on device %d (%s): conv2 runs on the MFMAs (about -25%% throughput)\n",
          h->device, why);
  return EXPECTO_OK;
}

int kmer_acquire(expecto_beluga* h, const float* const* params, hipStream_t st) {
  const size_t tb = kKmerFloats * sizeof(float), fb = (size_t)kMer8 * 320 * sizeof(double);
  if (const char* e = getenv("EXPECTO_KMER_MAX_BYTES"))
    if ((double)tb > atof(e)) return kmer_no_room(h, "EXPECTO_KMER_MAX_BYTES");
  std::vector<float> hw(320 * 32 + 320 + 320 * 320 * 8);
  EXPECTO_HIP_CHECK(hipMemcpyAsync(hw.data(), params[0], 320 * 32 * sizeof(float), hipMemcpyDeviceToHost, st));
  EXPECTO_HIP_CHECK(hipMemcpyAsync(hw.data() + 320 * 32, params[1], 320 * sizeof(float), hipMemcpyDeviceToHost, st));
  EXPECTO_HIP_CHECK(hipMemcpyAsync(hw.data() + 320 * 33, params[2], 320 * 320 * 8 * sizeof(float),
                                   hipMemcpyDeviceToHost, st));
  EXPECTO_HIP_CHECK(hipStreamSynchronize(st));
  const uint64_t key = fnv1a(hw.data(), hw.size() * sizeof(float));
  std::lock_guard<std::mutex> lock(g_kmer_mu);
  for (KmerEntry& e : g_kmer)
    if (e.device == h->device && e.key == key && e.w == hw) {
      e.holders.push_back(h);
      h->kmer = e.T;
      h->kmer_key = key;
      h->kmer_state = 0;
      return EXPECTO_OK;
    }
  void *t = nullptr, *f = nullptr, *gg = nullptr;
  if (hipMalloc(&t, tb) != hipSuccess || hipMalloc(&f, fb) != hipSuccess || hipMalloc(&gg, 8 * fb) != hipSuccess) {
    (void)hipGetLastError();
    for (void* x : {t, f, gg})
      if (x) (void)hipFree(x);
    return kmer_no_room(h, "device allocation failed");   // no table: conv2 on the MFMAs
  }
  float* T = static_cast<float*>(t);
  double* F = static_cast<double*>(f);
  double* G = static_cast<double*>(gg);
  kmer_conv1<<<dim3(kMer8), dim3(320), 0, st>>>(h->w1, h->b1, F);
  int rc = check_launch("kmer_conv1");
  for (int j = 0; j < 8; ++j)   // G: the 8 taps' products, [tap][5^8][320] fp64
    kmer_conv2<<<dim3((kMer8 + 63) / 64, 5), dim3(256), 0, st>>>(F, h->wt[0], j, G + (size_t)j * kMer8 * 320);
  for (int i = 0; i < 4; ++i)
    kmer_pair<<<dim3((unsigned)((kMer9 * 320 + 255) / 256)), dim3(256), 0, st>>>(
        G + (size_t)(2 * i) * kMer8 * 320, G + (size_t)(2 * i + 1) * kMer8 * 320, T + (size_t)i * kMer9 * 320);
  for (int hq = 0; hq < 2; ++hq)
    kmer_quad<<<dim3((unsigned)((kMer11 * 320 + 255) / 256)), dim3(256), 0, st>>>(
        G, hq, T + (4 * (size_t)kMer9 + hq * (size_t)kMer11) * 320);
  rc = rc ? rc : check_launch("kmer table");
  if (!rc && hipStreamSynchronize(st) != hipSuccess) rc = check_launch("kmer table sync");
  (void)hipFree(f);
  (void)hipFree(gg);
  if (rc) {
    (void)hipFree(t);
    return rc;
  }
  g_kmer.push_back({h->device, key, std::move(hw), T, {h}});
  h->kmer = T;
  h->kmer_key = key;
  h->kmer_state = 0;
  return EXPECTO_OK;
}

void kmer_release(expecto_beluga* h) {
  if (!h->kmer) return;
  std::lock_guard<std::mutex> lock(g_kmer_mu);
  for (size_t i = 0; i < g_kmer.size(); ++i)
    if (g_kmer[i].T == h->kmer) {
      auto& hs = g_kmer[i].holders;
      const auto it = std::find(hs.begin(), hs.end(), h);
      assert(it != hs.end() && "k-mer table held by an unregistered handle");
      if (it != hs.end()) hs.erase(it);   // (never erase end(): a handle not in the list is left alone)
      if (hs.empty()) {
        (void)hipFree(g_kmer[i].T);
        g_kmer.erase(g_kmer.begin() + (long)i);
      }
      break;
    }
  h->kmer = nullptr;
}

// Bytes of the k-mer tables h reports: all of them if h is their first live holder, else 0, so
// device_bytes summed over the handles sharing one table counts it once.
size_t kmer_reported_bytes(const expecto_beluga* h) {
  if (!h->kmer) return 0;
  std::lock_guard<std::mutex> lock(g_kmer_mu);
  for (const KmerEntry& e : g_kmer)
    if (e.T == h->kmer) return e.holders.front() == h ? kKmerFloats * sizeof(float) : 0;
  return 0;
}


// Host -> device copies of one call's tables through a pinned staging slot.  The slot was last
// filled two calls ago; its event fires once those copies ran (they precede that call's kernels
// on the stream), so the wait is normally already satisfied.
struct HostCopy {
  void* dst;
  const void* src;
  size_t bytes;
};
int stage_copies(expecto_beluga* h, const std::vector<HostCopy>& cp, hipStream_t st) {
  size_t total = 0;
  for (const HostCopy& c : cp) total += (c.bytes + 15) / 16 * 16;
  if (total == 0) return EXPECTO_OK;
  const int s = h->stage_next;
  h->stage_next ^= 1;
  if (h->stage_ev[s])
    EXPECTO_HIP_CHECK(hipEventSynchronize(h->stage_ev[s]));
  else
    EXPECTO_HIP_CHECK(hipEventCreateWithFlags(&h->stage_ev[s], hipEventDisableTiming));
  if (h->stage_cap[s] < total) {
    if (h->stage_buf[s]) EXPECTO_HIP_CHECK(hipHostFree(h->stage_buf[s]));
    h->stage_buf[s] = nullptr;
    h->stage_cap[s] = 0;
    const size_t cap = std::max<size_t>(total + total / 4, 1 << 16);
    EXPECTO_HIP_CHECK(hipHostMalloc(&h->stage_buf[s], cap, hipHostMallocDefault));
    h->stage_cap[s] = cap;
  }
  char* p = static_cast<char*>(h->stage_buf[s]);
  for (const HostCopy& c : cp) {
    if (c.bytes == 0) continue;
    std::memcpy(p, c.src, c.bytes);
    EXPECTO_HIP_CHECK(hipMemcpyAsync(c.dst, p, c.bytes, hipMemcpyHostToDevice, st));
    p += (c.bytes + 15) / 16 * 16;
  }
  EXPECTO_HIP_CHECK(hipEventRecord(h->stage_ev[s], st));
  return EXPECTO_OK;
}

// floats to allocate for `elements` activation elements in either format (6 B per bf16x6 element)
size_t act_alloc(size_t elements) { return elements + (elements + 1) / 2; }

// bf16 planes of a repacked fp32 B [rows][K] for the bf16x6 GEMM
int make_planes(expecto_beluga* h, const float* W, long long rows, long long K, float** out, hipStream_t st) {
  int rc;
  if ((rc = dalloc(h, out, act_alloc((size_t)(rows * K))))) return rc;
  const long long n4 = rows * K / 4;
  split_planes<<<dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st>>>(W, rows, (int)K,
                                                                           reinterpret_cast<__bf16*>(*out));
  return check_launch("split_planes");
}

// Activation buffers are sized in ELEMENTS (p_floats/q_floats) and allocated with 1.5 floats
// per element, so they hold either fp32 rows or bf16 planes (6 B per element).
size_t p_floats(int nb) { return (size_t)nb * kS1 * 320 + 16 * 640; }
size_t q_floats(int nb) { return (size_t)nb * 496 * 320 + 16 * 640; }

int resolve_events(expecto_beluga* h) {
  for (auto& pr : h->pending) {
    EXPECTO_HIP_CHECK(hipEventSynchronize(h->ev_pool[pr.second + 1]));
    float ms = 0.f;
    EXPECTO_HIP_CHECK(hipEventElapsedTime(&ms, h->ev_pool[pr.second], h->ev_pool[pr.second + 1]));
    h->ms[pr.first] += ms;
    h->calls[pr.first] += 1;
  }
  h->pending.clear();
  for (auto& r : h->pending_launch) {
    EXPECTO_HIP_CHECK(hipEventSynchronize(h->ev_pool[r.idx + 1]));
    float ms = 0.f;
    EXPECTO_HIP_CHECK(hipEventElapsedTime(&ms, h->ev_pool[r.idx], h->ev_pool[r.idx + 1]));
    auto& a = h->launch_stats[{r.layer, r.rows}];
    a[0] += ms;
    a[1] += 1;
    a[2] += r.macs;
  }
  h->pending_launch.clear();
  h->ev_next = 0;
  return EXPECTO_OK;
}

// Times ONE GEMM launch (its own event pair, beside the layer slot's) for the per-launch log.
struct LaunchTimer {
  expecto_beluga* h;
  int idx = -1;
  hipStream_t st;
  expecto_beluga::LaunchRec rec;
  LaunchTimer(expecto_beluga* hh, int layer, long long rows, double macs, hipStream_t s) : h(hh), st(s) {
    if (!h->profiling) return;
    if (h->ev_next + 2 > h->ev_pool.size()) resolve_events(h);
    idx = (int)h->ev_next;
    h->ev_next += 2;
    rec = {h->timer_base + layer, rows, idx, macs};
    (void)hipEventRecord(h->ev_pool[idx], st);
  }
  ~LaunchTimer() {
    if (idx < 0) return;
    (void)hipEventRecord(h->ev_pool[idx + 1], st);
    h->pending_launch.push_back(rec);
  }
};

struct LayerTimer {
  expecto_beluga* h;
  int layer;
  int idx = -1;
  hipStream_t st;
  LayerTimer(expecto_beluga* hh, int l, hipStream_t s) : h(hh), layer(hh->timer_base + l), st(s) {
    if (!h->profiling) return;
    if (h->ev_next + 2 > h->ev_pool.size()) resolve_events(h);
    idx = (int)h->ev_next;
    h->ev_next += 2;
    (void)hipEventRecord(h->ev_pool[idx], st);
  }
  ~LayerTimer() {
    if (idx < 0) return;
    (void)hipEventRecord(h->ev_pool[idx + 1], st);
    h->pending.push_back({layer, idx});
  }
};

// Launches inside this scope are timed and counted in the alt-delta slots (layer + kNumLayers).
struct DeltaScope {
  expecto_beluga* h;
  explicit DeltaScope(expecto_beluga* hh) : h(hh) { h->timer_base = kNumLayers; }
  ~DeltaScope() { h->timer_base = 0; }
};

// Arithmetic of the MFMA GEMMs: exact fp32 (v_mfma_f32_32x32x2_f32), the fp32-faithful 3-way
// bf16 split (bf16x6) or the scaled 2-way fp16 split (f16x3), gemm_kernel.h.
thread_local int g_precision = EXPECTO_PRECISION_BF16X6;
// f16x3 conv consumers read the next stage's operands inside the stage's last unit (gemm_kernel.h
// gemm_conv_h3p_body EA, TM bit 64; EXPECTO_CONV_EA=0 restores the reads after the last MFMA; same
// bits either way), set from the handle with g_precision
thread_local bool g_conv_ea = true;

// activation storage format (gemm_kernel.h): 1 bf16 planes (bf16x6), 2 scaled fp16 planes
// (f16x3), 0 fp32 rows; bytes per element 6 / 4 / 4
int act_fmt() {
  return g_precision == EXPECTO_PRECISION_BF16X6 ? 1 : g_precision == EXPECTO_PRECISION_F16X3 ? 2 : 0;
}
int act_bytes() { return act_fmt() == 1 ? 6 : 4; }
bool planes_gemm() { return g_precision != EXPECTO_PRECISION_FP32; }
long long gemm_bm() { return planes_gemm() ? X6P_BM : GBM; }
float exp2i(int e) { return std::ldexp(1.0f, e); }

// M tile rows of an f16x3 conv launch.  The 384-row kernel (beluga_conv_h3r: 4 waves of 96 x 160,
// each issuing its own LDS-DMA pieces one per MFMA unit) and the 256-row producer / consumer
// kernel (beluga_conv_h3p<.., 256, 4>: 4-deep B ring, next-stage fragments read before the
// barrier) give bitwise-equal results, so the choice is free per launch
// (tests/test_gpu_forward.py::test_conv_tile_choice_is_bitwise).  tools/gemm_bench (1000 windows,
// one box, fp32-equivalent TF/s, round 2): conv2 h3r 565 vs h3p 553, conv3 h3p 509 vs h3r 487,
// conv5 h3r 504 vs h3p 482, conv6 h3p 524 vs h3r 498 (conv4, pooled: 537 vs 533): 384-row tiles
// for conv2 and conv5.  One workgroup fills a CU, so a launch is priced by its rounds of 256
// workgroups (the alt-delta runs of the pair path, 30-60 k rows, take whichever tile needs the
// fewer row-rounds).  l: 0 = conv2 .. 4 = conv6.
int conv_tile_rows(const expecto_beluga* h, int l, bool pool, long long M, int n_tiles) {
  if (g_precision != EXPECTO_PRECISION_F16X3) return (int)gemm_bm();
  if (h->conv_tile) return h->conv_tile;
  // round 3 (tools/gemm_bench 2000 windows, two boxes): the producer / consumer 256-row kernel at
  // or above h3r on every layer (conv2 546 / 560 vs 535 / 558, conv5 503 / 512 vs 485 / 507), and
  // the 200-window pipeline +0.3-0.5 % with EXPECTO_CONV_TILE=256 (tools/knob_sweep.py, three
  // alternating rounds): 384-row tiles only where they need clearly fewer rounds of 256
  // workgroups (the small alt-delta launches of the pair path)
  const int cus = h->cus > 0 ? h->cus : 256;
  auto cost = [&](int bm, double per_row) {
    const long long blocks = (M + bm - 1) / bm * n_tiles;
    return (double)((blocks + cus - 1) / cus) * bm * per_row;
  };
  return cost(384, 1.0) * 1.1 <= cost(256, 1.0) ? 384 : 256;
}

// 64-column tiles for conv5 / conv6 (640 outputs: 10 N tiles instead of 4; gemm_kernel.h
// gemm_conv_h3p_body NB 4, same bits) for launches whose 160-column form leaves most of the chip
// idle -- the per-window forwards of small batches (batch 32: 60 workgroups on 256 CUs).  EXPECTO_CONV_NARROW=0 / 1 forces it (same bits either way).
// Round 6: conv3 / conv4 (480 outputs) of such batches on 128-column tiles (4 N tiles instead of 3;
// the weight planes carry 32 zero rows): batch 32 is 62 M tiles, 186 workgroups on 256 CUs at 160
// columns, 248 at 128 -- one round either way, 0.8 of the work per workgroup.
int conv_narrow_cols(int l) { return l == 1 || l == 2 ? 128 : 64; }
bool conv_narrow(const expecto_beluga* h, int l, long long M, int bm, int n_tiles) {
  if (g_precision != EXPECTO_PRECISION_F16X3 || l < 1 || l > 4) return false;
  if (h->conv_narrow >= 0) return h->conv_narrow != 0;
  if (!h->narrow_scope) return false;
  // only when the narrow launch is one round of workgroups (per column the 64-column tile runs at
  // ~0.8 of the 160-column one: batch 32, conv5 + conv6 281 -> 138 us for 0.4 of the work per
  // workgroup), and only for the per-window forwards (narrow_scope): the segment path's small
  // alt-delta conv5 / conv6 launches run beside the trunk on the second stream, where more
  // workgroups for the same work cost the trunk (conv6 11.1 -> 11.6 ms per headline step, same box)
  const long long cus = h->cus > 0 ? h->cus : 256;
  const int nc = conv_narrow_cols(l);
  const long long narrow = (M + 255) / 256 * ((kConv[l].cout + nc - 1) / nc), wide = (M + bm - 1) / bm * n_tiles;
  return narrow <= cus && wide < cus;
}

template <int LAYER, int EPI>
int launch_gemm(const GemmArgs& a, int splits, hipStream_t st, int bm = 0) {
  if (bm == 0) bm = (int)gemm_bm();
  const long long nblk = a.m_tiles * a.n_tiles * splits;
  EXPECTO_REQUIRE(nblk > 0 && nblk < (1LL << 31), "gemm grid out of range");
  EXPECTO_REQUIRE(a.kper % GBK == 0 && a.kper > 0, "gemm K not a multiple of 32");
  EXPECTO_REQUIRE(a.lda % 4 == 0 && a.ldb % 4 == 0, "gemm leading dims must be multiples of 4");
  EXPECTO_REQUIRE(a.taps == 1 || (a.taps == 8 && a.lda % GBK == 0), "conv GEMM needs Cin % 32 == 0");
  EXPECTO_REQUIRE(a.m_tiles * bm >= a.M, "gemm M tiles do not cover M");
  EXPECTO_REQUIRE(bm == gemm_bm() || (bm == 384 && a.taps == 8 && g_precision == EXPECTO_PRECISION_F16X3),
                  "384-row tiles: f16x3 conv kernel only");
  if (g_precision == EXPECTO_PRECISION_BF16X6) {
    EXPECTO_REQUIRE(a.Bp != nullptr && a.lda % GBK == 0 && a.ldb % GBK == 0, "bf16x6 GEMM needs planes, K % 32");
    beluga_gemm_x6q<LAYER, EPI><<<dim3((unsigned)nblk), dim3(256), 0, st>>>(a);
  } else if (g_precision == EXPECTO_PRECISION_F16X3) {
    EXPECTO_REQUIRE(a.Bp != nullptr && a.lda % GBK == 0 && a.ldb % GBK == 0, "f16x3 GEMM needs planes, K % 32");
    EXPECTO_REQUIRE(EPI == EPI_PARTIAL || a.col_scale != nullptr, "f16x3 GEMM needs column scales");
    if (a.taps == 8) {   // conv: chunk-slab kernel (one Toeplitz A slab per 32-channel chunk)
      EXPECTO_REQUIRE(splits == 1 && a.kper == a.ldb && a.ldb == 8 * a.lda && !a.m_fastest && !a.a_rows,
                      "f16x3 conv GEMM: full K, no split, no row gather");
      // all bitwise equal (same products and k order per output); per-layer choice from
      // tools/gemm_bench: 256-row tiles on the producer/consumer kernel (MFMA waves never issue
      // LDS-DMA), 384-row tiles (conv2) on the 4-wave 96-row kernel
      if (a.c1_codes) {   // conv2 with conv1 fused into the producers (A slabs from base codes)
        if constexpr (LAYER == 2 && EPI == EPI_RELU_POOL4) {
          EXPECTO_REQUIRE(bm == 256 && a.c1_w && a.c1_cs && a.c1_b, "fused conv1: 256-row tiles, conv1 planes");
          if (g_conv_ea)
            beluga_conv_h3p<LAYER, EPI, 256 | 64 | H3P_FUSE_CONV1, 4><<<dim3((unsigned)nblk), dim3(512), 0, st>>>(a);
          else
            beluga_conv_h3p<LAYER, EPI, 256 | H3P_FUSE_CONV1, 4><<<dim3((unsigned)nblk), dim3(512), 0, st>>>(a);
        } else {
          EXPECTO_REQUIRE(false, "fused conv1: conv2 + pool1 only");
        }
      } else if (a.n_tile_cols == 64) {   // 64-column tiles (conv_narrow: conv5 / conv6 of small batches)
        if constexpr ((LAYER == 5 || LAYER == 6) && EPI == EPI_RELU) {
          EXPECTO_REQUIRE(bm == 256 && a.n_tiles * 64 >= a.n_store, "64-column conv tiles: 256 rows");
          beluga_conv_h3p_narrow<LAYER, EPI, 4><<<dim3((unsigned)nblk), dim3(512), 0, st>>>(a);
        } else {
          EXPECTO_REQUIRE(false, "64-column conv tiles: conv5 / conv6 only");
        }
      } else if (a.n_tile_cols == 128) {   // 128-column tiles (conv_narrow: conv3 / conv4 of small batches)
        if constexpr (LAYER == 3 || LAYER == 4) {
          EXPECTO_REQUIRE(bm == 256 && a.n_tiles == 4 && a.n_store == 480, "128-column conv tiles: conv3 / conv4");
          beluga_conv_h3p_narrow<LAYER, EPI, 8><<<dim3((unsigned)nblk), dim3(512), 0, st>>>(a);
        } else {
          EXPECTO_REQUIRE(false, "128-column conv tiles: conv3 / conv4 only");
        }
      } else if (bm == 384)
        beluga_conv_h3r<LAYER, EPI><<<dim3((unsigned)nblk), dim3(256), 0, st>>>(a);
      else if (g_conv_ea)   // 4-deep B ring, next-stage fragments read inside the stage's last unit (TM 256 | 64)
        beluga_conv_h3p<LAYER, EPI, 256 | 64, 4><<<dim3((unsigned)nblk), dim3(512), 0, st>>>(a);
      else   // 4-deep B ring, next-stage fragments read before the stage barrier (TM 256)
        beluga_conv_h3p<LAYER, EPI, 256, 4><<<dim3((unsigned)nblk), dim3(512), 0, st>>>(a);
    } else if constexpr (EPI == EPI_PARTIAL) {
      // FC split-K partials: 336-column tiles on 8 MFMA waves when the caller tiled N that way
      // (n_tile_cols, set from fc_wide_tiles), else 160-column producer / consumer tiles (same
      // bits either way)
      EXPECTO_REQUIRE(a.n_tile_cols == 0 || a.n_tile_cols == FCW_BN || a.n_tile_cols == 112 ||
                          a.n_tile_cols == 16 * FCS_NB,
                      "FC tile width: 0 (160), 336, 112 or 32 columns");
      EXPECTO_REQUIRE((long long)a.n_tiles * (a.n_tile_cols ? a.n_tile_cols : GBN) >= a.n_store,
                      "FC N tiles do not cover the stored columns");
      if (a.n_tile_cols == FCW_BN)
        beluga_fc_h3w<LAYER, EPI><<<dim3((unsigned)nblk), dim3(512), 0, st>>>(a);
      else if (a.n_tile_cols == 112)
        beluga_fc_h3w_narrow<LAYER, EPI><<<dim3((unsigned)nblk), dim3(512), 0, st>>>(a);
      else if (a.n_tile_cols == 16 * FCS_NB) {   // <= 32 rows: 32 x 32 tiles, 9-stage ring (fc_skinny)
        EXPECTO_REQUIRE(a.m_tiles == 1 && a.M <= 32 && !a.ks_mask, "skinny FC tiles: one tile of <= 32 rows");
        beluga_fc_h3s<LAYER, EPI><<<dim3((unsigned)nblk), dim3(64 * 2 * FCS_NB), 0, st>>>(a);
      }
      else
        beluga_fc_h3p<LAYER, EPI><<<dim3((unsigned)nblk), dim3(512), 0, st>>>(a);
    } else {   // FC layers: producer / consumer waves, both operands through an LDS ring (same bits)
      beluga_fc_h3p<LAYER, EPI><<<dim3((unsigned)nblk), dim3(512), 0, st>>>(a);
    }
  } else
    beluga_gemm<LAYER, EPI, kWM, kMinBlocks, GBK, kPipe><<<dim3((unsigned)nblk), dim3(64 * kWM), 0, st>>>(a);
  return check_launch("beluga_gemm");
}

int run_conv1(expecto_beluga* h, const float* x, const uint8_t* codes, long long code_stride, int n_src, int mode,
              long long row0, int nb, int len, int out_rows, hipStream_t st, float* dst = nullptr) {
  LayerTimer lt(h, 0, st);
  if (h->profiling) h->macs[h->timer_base + 0] += (double)nb * (len - 7) * 320 * 32;
  if (g_precision == EXPECTO_PRECISION_F16X3 && h->w1h) {
    dim3 grid((len - 7 + C1H_ROWS - 1) / C1H_ROWS, nb);
    beluga_conv1_h3<<<grid, dim3(320), 0, st>>>(x, codes, code_stride, n_src, mode, row0,
                                                reinterpret_cast<const _Float16*>(h->w1h), h->cs1, h->b1,
                                                dst ? dst : h->P, out_rows, len, exp2i(h->sx[0]), h->ovf);
    return check_launch("beluga_conv1_h3");
  }
  dim3 grid((len - 7 + C1_T - 1) / C1_T, nb);
  beluga_conv1<<<grid, dim3(320), 0, st>>>(x, codes, code_stride, n_src, mode, row0, h->w1, h->b1,
                                           dst ? dst : h->P, out_rows, len, act_fmt(), exp2i(h->sx[0]), h->ovf);
  return check_launch("beluga_conv1");
}

// Base codes of a conv1 input, as run_conv1 takes them (window w = code row row0 + w; mode
// EXPECTO_STRAND_*, rows >= n_src of a BOTH call are the rc of row - n_src; len bases).
struct C1Src {
  const uint8_t* codes;
  long long stride;
  int n_src, mode;
  long long row0;
  int len;
};

// conv1 fused into conv2 (f16x3, codes input): no conv1 launch, no conv1 planes in HBM; the conv2
// producers compute the A slabs from the codes (gemm_kernel.h conv12_producer; same bits).
// EXPECTO_FUSE_CONV1=0 keeps the separate beluga_conv1_h3 launch.
bool fuse_conv1(const expecto_beluga* h, const float* x) {
  return h->fuse_conv1 && !x && g_precision == EXPECTO_PRECISION_F16X3 && h->w1h;
}

// conv1 + conv2 + pool1 from the k-mer table (f16x3 and bf16x6, codes input; EXPECTO_CONV2_TABLE=0 runs them
// on the MFMAs): `rows` pooled rows per window into dst rows w * s_out + g
bool use_kmer(const expecto_beluga* h, const float* x) {
  return h->kmer && !x && (g_precision == EXPECTO_PRECISION_F16X3 || g_precision == EXPECTO_PRECISION_BF16X6);
}

int run_conv2_kmer(expecto_beluga* h, const C1Src& f, long long n_win, int rows, int s_out, float* dst, hipStream_t st) {
  LayerTimer lt(h, 1, st);
  const int rb = (rows + KP_ROWS - 1) / KP_ROWS;
  const long long nblk = n_win * rb;
  EXPECTO_REQUIRE(nblk > 0 && nblk < (1LL << 31) && f.len >= 18, "conv2 k-mer grid / window length");
  conv2_kmer_pool<<<dim3((unsigned)nblk), dim3(640), 0, st>>>(f.codes, f.stride, f.n_src, f.mode, f.row0, f.len, rows,
                                                              rb, s_out, h->kmer, h->bt[0],
                                                              act_fmt() == 2 ? exp2i(h->sx[1]) : 1.f,
                                                              h->kmer_quad ? 1 : 0, act_fmt(), dst, h->ovf);
  return check_launch("conv2_kmer_pool");
}

// conv layer l (0 = conv2 .. 4 = conv6) over `groups` row groups of s_in rows each.  f1 (conv2
// only): compute conv1 from these codes inside the conv2 launch instead of reading src.
int run_conv(expecto_beluga* h, int l, const float* src, float* dst, long long groups, int s_in, int t_valid,
             int s_out, bool pool, hipStream_t st, const C1Src* f1 = nullptr) {
  const ConvGeo& g = kConv[l];
  GemmArgs a{};
  a.A = src;
  a.lda = g.cin;
  a.M = groups * s_in;
  a.B = h->wt[l];
  a.Bp = g_precision == EXPECTO_PRECISION_F16X3 ? h->wh[l] : h->wp[l];
  a.col_scale = g_precision == EXPECTO_PRECISION_F16X3 ? h->cs[l] : nullptr;
  a.out_scale = exp2i(h->sx[l + 1]);
  a.ovf = h->ovf;
  a.ldb = 8LL * g.cin;
  a.kper = 8 * g.cin;
  a.taps = 8;
  a.n_tiles = npad_of(g.cout) / GBN;
  int bm = f1 ? 256 : conv_tile_rows(h, l, pool, a.M, (int)a.n_tiles);
  if (!f1 && (!pool || l == 2) && conv_narrow(h, l, a.M, bm, (int)a.n_tiles)) {
    bm = 256;
    a.n_tile_cols = conv_narrow_cols(l);
    a.n_tiles = (g.cout + a.n_tile_cols - 1) / a.n_tile_cols;
  }
  a.m_tiles = (a.M + bm - 1) / bm;
  a.m_fastest = 0;
  a.bias = h->bt[l];
  a.C = dst;
  a.ldc = g.cout;
  a.n_store = g.cout;
  a.s_in = s_in;
  a.t_valid = t_valid;
  a.s_out = s_out;
  if (f1) {
    EXPECTO_REQUIRE(l == 0 && pool && g_precision == EXPECTO_PRECISION_F16X3 && h->w1h && f1->len >= 8,
                    "fused conv1: f16x3 conv2 + pool1 from codes");
    a.A = nullptr;
    a.c1_codes = f1->codes;
    a.c1_stride = f1->stride;
    a.c1_row0 = f1->row0;
    a.c1_n_src = f1->n_src;
    a.c1_mode = f1->mode;
    a.c1_len = f1->len;
    a.c1_n_win = (int)groups;
    a.c1_w = reinterpret_cast<const _Float16*>(h->w1h);
    a.c1_cs = h->cs1;
    a.c1_b = h->b1;
    a.c1_osc = exp2i(h->sx[0]);
    // conv1's algorithmic MACs stay in conv1's slot (its time is inside this launch)
    if (h->profiling) h->macs[h->timer_base + 0] += (double)groups * (f1->len - 7) * 320 * 32;
  }
  LayerTimer lt(h, l + 1, st);
  if (h->profiling) h->macs[h->timer_base + l + 1] += (double)a.M * g.cout * a.kper;
  LaunchTimer lrec(h, l + 1, a.M, (double)a.M * g.cout * a.kper, st);
  if (pool) {
    EXPECTO_REQUIRE(s_in % 4 == 0, "pool epilogue needs 4-aligned row groups");
    return l == 0 ? launch_gemm<2, EPI_RELU_POOL4>(a, 1, st, bm) : launch_gemm<4, EPI_RELU_POOL4>(a, 1, st, bm);
  }
  switch (l) {
    case 1: return launch_gemm<3, EPI_RELU>(a, 1, st, bm);
    case 2: return launch_gemm<4, EPI_RELU>(a, 1, st, bm);
    case 3: return launch_gemm<5, EPI_RELU>(a, 1, st, bm);
    default: return launch_gemm<6, EPI_RELU>(a, 1, st, bm);
  }
}

// Segment path, f16x3, pool2 phases {0, 2} (the 200-bp shift sweeps): conv4 with its pool2 in the
// epilogue (gemm_kernel.h epilogue_pool_ph02) straight into the phase blocks at `dst` (n_ph = 2, s5
// pooled rows each), then pool2_tile_seams for the phase-2 rows across tile boundaries.  The same
// bits as conv4 unpooled + pool4_phases_h2m; the unpooled rows themselves are written only where
// something reads them: the tile seams (h->seam) and, for segment pairs (tab), seg_delta_pool's ref
// rows (h->edge, kSegEdge per segment).  EXPECTO_POOL_FUSED=0 keeps the separate pool pass.
bool conv4_pool_fused(const expecto_beluga* h, long long M, int n_ph, const int* ph) {
  if (!h->pool_fused || act_fmt() != 2 || !h->pool_one_pass || n_ph != 2 || ph[0] != 0 || ph[1] != 2) return false;
  const int bm = conv_tile_rows(h, 2, false, M, npad_of(480) / GBN);
  return bm == 256 && !conv_narrow(h, 2, M, bm, npad_of(480) / GBN);
}
int run_conv4_pool_fused(expecto_beluga* h, const float* src, float* dst, long long groups, int s_in, int t4, int s5,
                         const int* tab, hipStream_t st) {
  const ConvGeo& g = kConv[2];
  GemmArgs a{};
  a.A = src;
  a.lda = g.cin;
  a.M = groups * s_in;
  a.B = h->wt[2];
  a.Bp = h->wh[2];
  a.col_scale = h->cs[2];
  a.out_scale = exp2i(h->sx[3]);
  a.ovf = h->ovf;
  a.ldb = 8LL * g.cin;
  a.kper = 8 * g.cin;
  a.taps = 8;
  a.n_tiles = npad_of(g.cout) / GBN;
  a.m_tiles = (a.M + 255) / 256;
  a.bias = h->bt[2];
  a.C = dst;
  a.ldc = g.cout;
  a.n_store = g.cout;
  a.s_in = s_in;
  a.t_valid = t4;
  a.s_out = s5;
  EXPECTO_REQUIRE(g_precision == EXPECTO_PRECISION_F16X3 && s_in % 4 == 0 && t4 <= s_in && a.n_tiles == 3,
                  "fused conv4 + pool2: f16x3 segment blocks at a 4-aligned row stride");
  const size_t seam_rows = (size_t)a.m_tiles * 4, edge_rows = tab ? (size_t)groups * kSegEdge : 0;
  auto grow = [&](float*& b, size_t& cap, size_t rows) -> int {   // (grown once per handle and size)
    if (rows <= cap) return EXPECTO_OK;
    if (b) EXPECTO_HIP_CHECK(hipFree(b));
    b = nullptr;
    h->bytes -= cap * 480 * 4;
    cap = 0;
    EXPECTO_HIP_CHECK(hipMalloc(&b, rows * 480 * 4));
    EXPECTO_HIP_CHECK(hipMemset(b, 0, rows * 480 * 4));
    cap = rows;
    h->bytes += rows * 480 * 4;
    return EXPECTO_OK;
  };
  int rc;
  if ((rc = grow(h->seam, h->seam_cap, seam_rows)) || (rc = grow(h->edge, h->edge_cap, edge_rows))) return rc;
  a.c_seam = h->seam;
  a.c_edge = h->edge;
  a.unp_tab = tab;
  a.unp_ld = kSegTab;
  a.unp_dw = kDW[4];
  const long long nblk = a.m_tiles * a.n_tiles;
  EXPECTO_REQUIRE(nblk > 0 && nblk < (1LL << 31), "gemm grid out of range");
  {
    LayerTimer lt(h, 3, st);
    if (h->profiling) h->macs[h->timer_base + 3] += (double)a.M * g.cout * a.kper;
    LaunchTimer lrec(h, 3, a.M, (double)a.M * g.cout * a.kper, st);
    if (g_conv_ea)
      beluga_conv_h3p<4, EPI_POOL_PH02, 256 | 64, 4><<<dim3((unsigned)nblk), dim3(512), 0, st>>>(a);
    else
      beluga_conv_h3p<4, EPI_POOL_PH02, 256, 4><<<dim3((unsigned)nblk), dim3(512), 0, st>>>(a);
    if ((rc = check_launch("beluga_conv_h3p pool2"))) return rc;
  }
  LayerTimer lt(h, 3, st);   // pool2 is timed with conv4
  if (a.m_tiles > 1)
    pool2_tile_seams<<<dim3((unsigned)(a.m_tiles - 1)), dim3(64), 0, st>>>(h->seam, a.M, s_in, t4, s5, dst);
  return check_launch("pool2_tile_seams");
}

// FC1 (split-K) + reduce + FC2/sigmoid for nb windows whose conv6 rows are at act
// (+ a_rows[m] when given, else m*67840).
// part_rows: row count of the split-K partial slabs (default nb): an alt FC1 that recomputes
// only some slabs of the first nb rows of an earlier ref FC1 over part_rows rows reuses its
// partials for the others.
// h1 rows (FC1 output, FC2 input) start `rows` rows into the h1 buffer
float* h1_rows(expecto_beluga* h, long long rows) { return h->h1 + rows * kHidLd * act_bytes() / 4; }

// FC split-K GEMMs on 336-column tiles (beluga_fc_h3w): f16x3 only (the other arithmetics keep
// their 160-column kernels).  tools/gemm_bench fc1 (8,192 segment-like rows, 8 slabs, one box,
// fp32-eq TF/s): 485 vs 449.5 (160-column tiles, N fastest) / 464.6 (grouped M tiles); bitwise
// equal.  Their N order is the XCD-remapped N-fastest one (m_fastest 0): 6 N tiles of one M
// tile share its A rows, ~5.3 M tiles per XCD share a weight tile.
bool fc_wide_tiles(const expecto_beluga* h) { return h->fc_wide && g_precision == EXPECTO_PRECISION_F16X3; }

bool fc1_narrow(const expecto_beluga* h, long long mtt);
bool fc_skinny(const expecto_beluga* h, long long rows);

// FC1 (split-K slabs into `part`) + fc1_reduce (bias, ReLU, activation planes) into h1.
int run_fc1(expecto_beluga* h, const float* act, const long long* a_rows, int nb, float* h1, hipStream_t st,
            const unsigned* ks_mask = nullptr, double slab_frac = 1.0, long long part_rows = 0) {
  if (part_rows <= 0) part_rows = nb;
  int rc;
  const long long m_tiles = (nb + gemm_bm() - 1) / gemm_bm();
  const bool wide = fc_wide_tiles(h);
  const int n_tiles1 = wide ? (kHidLd + FCW_BN - 1) / FCW_BN : npad_of(kFc1Out) / GBN;
  const int splits = h->fc_splits;
  {
    GemmArgs a{};
    a.A = act;
    a.a_rows = a_rows;
    a.lda = (long long)kFc1In;
    a.M = nb;
    a.B = h->fc1w;
    a.Bp = g_precision == EXPECTO_PRECISION_F16X3 ? h->wh[5] : h->fc1p;
    a.ldb = kFc1In;
    a.kper = kFc1In / splits;
    a.taps = 1;
    a.n_tiles = n_tiles1;
    a.m_tiles = m_tiles;
    // dispatch order: M tiles fastest while one split-K slab of A (all rows) is small (<= 80 MB:
    // 2,000-row configs[1] calls, 69 MB), so every XCD sweeps the same K slab (B slab read once);
    // for larger M N tiles fastest, so the 13 N tiles of an A tile run together (tools/gemm_bench
    // fc1: +8 % at 4,000 rows, +5 % at 19,200 rows; round 2: the 2,816-row last FC slice of the
    // 200-window workload, 95 MB per slab, read 6.6 TB/s of L2 misses in M order, and 80 instead
    // of 128 MB gained 0.6-0.7 % on that workload in two interleaved sweeps)
    a.m_fastest = (double)m_tiles * gemm_bm() * (kFc1In / splits) * 4.0 <= h->fc1_m_order_mb * (1 << 20) ? 1 : 0;
    a.linear_order = a.m_fastest;   // N tiles fastest: XCD-aware remap (consecutive tiles share an XCD)
    if (h->fc1_order == 2 && !a.m_fastest && m_tiles % 8 == 0 && planes_gemm() && g_precision == EXPECTO_PRECISION_F16X3)
      a.m_fastest = 2;              // slab-outermost, XCD-owned M tiles (gemm_fc_h3p_body)
    // round 3 default: grouped order (gemm_fc_h3p_body m_fastest 3; XCD remap, so an XCD's ~32
    // concurrent workgroups cover m_group M tiles x ~32/m_group N tiles of one split-K slab):
    // tools/gemm_bench fc1 (segment-like a_rows, 8 slabs), one box, fp32-eq TF/s: 8,192 rows
    // 460 vs 433 (N fastest) / 441 (M fastest), 2,816 rows 434 vs 411 / 397; same bits
    if (h->fc1_order == 3 && g_precision == EXPECTO_PRECISION_F16X3) {
      a.m_fastest = 3;
      a.m_group = h->fc1_m_group;
      a.linear_order = 0;
    }
    if (wide) {   // 336-column tiles: N fastest per XCD (orders measured equal within 1 %)
      a.m_fastest = 0;
      a.linear_order = 0;
      a.n_tile_cols = FCW_BN;
      if (!ks_mask && fc_skinny(h, nb)) {   // <= 32 rows: 48 columns, deep ring
        a.n_tile_cols = 16 * FCS_NB;
        a.n_tiles = kHidLd / a.n_tile_cols;
      } else if (!ks_mask && fc1_narrow(h, m_tiles * splits)) {   // small per-window batches: 112 columns
        a.n_tile_cols = 112;
        a.n_tiles = kHidLd / 112;
      }
    }
    a.C = h->part;
    a.ldc = kHidLd;
    a.n_store = kHidLd;
    a.split_stride = part_rows * kHidLd;
    a.ks_mask = ks_mask;
    EXPECTO_REQUIRE(!ks_mask || planes_gemm(), "slab mask needs the planes GEMM");
    LayerTimer lt(h, 6, st);
    if (h->profiling) h->macs[h->timer_base + 6] += (double)nb * kFc1Out * kFc1In * slab_frac;
    if ((rc = launch_gemm<7, EPI_PARTIAL>(a, splits, st))) return rc;
  }
  {
    LayerTimer lt(h, 7, st);
    const long long count = (long long)nb * kHidLd;
    const bool f16 = g_precision == EXPECTO_PRECISION_F16X3;
    if (act_fmt() == 2)
      fc1_reduce_h2<<<dim3((unsigned)((count / 4 + 255) / 256)), dim3(256), 0, st>>>(
          h->part, splits, part_rows * kHidLd, count / 4, h->fc1b, h1, h->cs[5], exp2i(h->sx[6]), h->ovf);
    else
      fc1_reduce<<<dim3((unsigned)((count + 255) / 256)), dim3(256), 0, st>>>(
          h->part, splits, part_rows * kHidLd, count, h->fc1b, h1, act_fmt(), f16 ? h->cs[5] : nullptr, exp2i(h->sx[6]), h->ovf);
    if ((rc = check_launch("fc1_reduce"))) return rc;
  }
  return EXPECTO_OK;
}

// FC2 + sigmoid over nb h1 rows; output row m goes to y row c_rows[m] (or m).
int run_fc2(expecto_beluga* h, const float* h1, int nb, float* y, hipStream_t st, const long long* c_rows) {
  int rc;
  const long long m_tiles = (nb + gemm_bm() - 1) / gemm_bm();
  {
    GemmArgs a{};
    a.A = h1;
    a.lda = kHidLd;
    a.M = nb;
    a.B = h->fc2w;
    a.Bp = g_precision == EXPECTO_PRECISION_F16X3 ? h->wh[6] : h->fc2p;
    a.col_scale = g_precision == EXPECTO_PRECISION_F16X3 ? h->cs[6] : nullptr;
    a.ldb = kHidLd;
    a.kper = kHidLd / h->fc2_splits;
    a.taps = 1;
    const bool wide = fc_wide_tiles(h) && h->fc2_splits > 1;
    a.n_tiles = wide ? (kNFeat + FCW_BN - 1) / FCW_BN : npad_of(kNFeat) / GBN;
    a.m_tiles = m_tiles;
    // M tiles fastest while the A slab is small; N tiles fastest (XCD-aware remap: an XCD runs
    // the 13 N tiles of its A tiles back to back) for the large unsplit launches of the segment
    // path, whose h1 rows (up to fc2_rows x 8 KB) would otherwise be streamed once per N tile
    a.m_fastest = (double)m_tiles * gemm_bm() * (kHidLd / h->fc2_splits) * 4.0 <= h->fc1_m_order_mb * (1 << 20) ? 1 : 0;
    if (wide) {
      a.m_fastest = 0;
      a.n_tile_cols = FCW_BN;
      if (fc_skinny(h, nb)) {   // <= 32 rows: 48 columns, deep ring
        a.n_tile_cols = 16 * FCS_NB;
        a.n_tiles = (kNFeat + a.n_tile_cols - 1) / a.n_tile_cols;
      } else if (fc1_narrow(h, m_tiles * h->fc2_splits)) {   // small per-window batches: 112 columns
        a.n_tile_cols = 112;
        a.n_tiles = (kNFeat + 111) / 112;
      }
    }
    a.C = h->part2;
    a.ldc = kHidLd;
    a.n_store = kNFeat;
    a.split_stride = (long long)nb * kHidLd;
    LayerTimer lt(h, 8, st);
    if (h->profiling) h->macs[h->timer_base + 8] += (double)nb * kNFeat * kFc1Out;
    if (h->fc2_splits == 1) {
      // no split: bias + sigmoid in the GEMM epilogue, rows scattered through c_rows (the
      // same per-element unscale, bias and expf as fc2_reduce over one slab: same bits)
      a.C = y;
      a.ldc = kNFeat;
      a.c_rows = c_rows;
      a.bias = h->fc2b;
      a.s_in = a.t_valid = a.s_out = 1;
      return launch_gemm<8, EPI_SIGMOID>(a, 1, st);
    }
    if ((rc = launch_gemm<8, EPI_PARTIAL>(a, h->fc2_splits, st))) return rc;
    if ((reinterpret_cast<uintptr_t>(y) & 7) == 0)
      fc2_reduce<<<dim3((unsigned)((kNFeat / 2 + 255) / 256), (unsigned)std::max<long long>(1, std::min<long long>(nb, 65535))), dim3(256), 0,
                   st>>>(h->part2, h->fc2_splits, (long long)nb * kHidLd, nb, h->fc2b, a.col_scale, c_rows, y);
    else
      fc2_reduce1<<<dim3((unsigned)(((long long)nb * kNFeat + 255) / 256)), dim3(256), 0, st>>>(
          h->part2, h->fc2_splits, (long long)nb * kHidLd, nb, h->fc2b, a.col_scale, c_rows, y);
    if ((rc = check_launch("fc2_reduce"))) return rc;
  }
  return EXPECTO_OK;
}

int run_fc(expecto_beluga* h, const float* act, const long long* a_rows, int nb, float* y, hipStream_t st,
           const long long* c_rows = nullptr, const unsigned* ks_mask = nullptr, double slab_frac = 1.0,
           long long part_rows = 0) {
  int rc;
  if ((rc = run_fc1(h, act, a_rows, nb, h->h1, st, ks_mask, slab_frac, part_rows))) return rc;
  return run_fc2(h, h->h1, nb, y, st, c_rows);
}

int count_desc_macs(expecto_beluga* h, const unsigned* mask, int tiles, double per_tile, hipStream_t st);

// ---- FC1 block Karatsuba (f16x3): host side (kernels and algebra: "FC1 as a block-Karatsuba
// convolution" above) ------------------------------------------------------------------------
// (its grouped launch always runs the 336-column tile); per-window forwards: role 4 = the direct FC1
bool fk_use(const expecto_beluga* h) {
  return h->fk_on && h->fkw && g_precision == EXPECTO_PRECISION_F16X3 && h->fk_role < 4;
}
bool fk_use_seg(const expecto_beluga* h) { return h->fk_on && h->fkw && g_precision == EXPECTO_PRECISION_F16X3; }

// Table buffers, allocated with the first Karatsuba FC1: group starts (9 lists of <= max_batch),
// window starts, kFkParts partial rows per window, kFkParts x tiles alt-mask words.
int fk_cap(const expecto_beluga* h) { return std::max(h->max_batch, h->fk_slice); }

int fk_tables(expecto_beluga* h) {
  if (h->fk_grows) return EXPECTO_OK;
  const size_t mb = h->max_batch, tiles = (mb + 255) / 256, cap = fk_cap(h);
  float *a = nullptr, *b = nullptr, *c = nullptr, *d = nullptr;
  int rc;
  if ((rc = dalloc(h, &a, 2 * 9 * cap)) || (rc = dalloc(h, &b, 2 * mb)) || (rc = dalloc(h, &c, kFkParts * cap)) ||
      (rc = dalloc(h, &d, kFkParts * tiles)))
    return rc;
  h->fk_grows = reinterpret_cast<long long*>(a);
  h->fk_wrows = reinterpret_cast<long long*>(b);
  h->fk_prow = reinterpret_cast<int*>(c);
  h->fk_mask = reinterpret_cast<unsigned*>(d);
  return EXPECTO_OK;
}

// Segment-path FC1 launches of up to fk_cap windows (one launch per strand for the 200-window
// workload's 19,200 windows: one round structure instead of three part-filled ones): partial rows,
// FC1 output rows, window starts and output rows, allocated with the first segment call.
int fk_seg_buffers(expecto_beluga* h) {
  if (h->fk_part) return EXPECTO_OK;
  const size_t cap = fk_cap(h);
  float *a = nullptr, *b = nullptr;
  int rc;
  if ((rc = dalloc(h, &h->fk_part, (size_t)kFkParts * cap * kHidLd)) || (rc = dalloc(h, &h->fk_h1, act_alloc(cap * kHidLd))) ||
      (rc = dalloc(h, &a, 2 * cap)) || (rc = dalloc(h, &b, 2 * cap)))
    return rc;
  h->fk_arows = reinterpret_cast<long long*>(a);
  h->fk_crows = reinterpret_cast<long long*>(b);
  float *c = nullptr, *d = nullptr, *e = nullptr, *f = nullptr, *q = nullptr, *m = nullptr;
  if ((rc = dalloc(h, &c, 9 * cap)) || (rc = dalloc(h, &d, 2 * cap)) || (rc = dalloc(h, &e, 2 * cap)) ||
      (rc = dalloc(h, &f, kFkParts * cap)) || (rc = dalloc(h, &q, cap)) || (rc = dalloc(h, &m, 19 * (cap / 256 + 1))))
    return rc;
  h->fk_rgrp = reinterpret_cast<int*>(c);
  h->fk_ginfo = reinterpret_cast<int*>(d);
  h->fk_winfo = reinterpret_cast<int*>(e);
  h->fk_aprow = reinterpret_cast<int*>(f);
  h->fk_aperm = reinterpret_cast<int*>(q);
  h->fk_smask = reinterpret_cast<unsigned*>(m);
  return EXPECTO_OK;
}

// The D1 / D2 / DD sequence buffers for `rows` conv6 rows (grown on demand; hipFree synchronises,
// so they are sized once for the largest call).
int fk_seq_alloc(expecto_beluga* h, long long rows, int set = 0) {
  float** b = set ? h->fk_aseq : h->fk_seq;
  long long& cap = set ? h->fk_aseq_rows : h->fk_seq_rows;
  if (rows <= cap && b[0]) return EXPECTO_OK;
  for (int i = 0; i < 3; ++i)
    if (b[i]) {
      EXPECTO_HIP_CHECK(hipFree(b[i]));
      b[i] = nullptr;
    }
  h->bytes -= (size_t)cap * 640 * 4 * 3;
  cap = 0;
  for (int i = 0; i < 3; ++i) {
    hipError_t e = hipMalloc(&b[i], (size_t)rows * 640 * 4 + 16 * 640 * 4);
    if (e != hipSuccess) {
      set_error(std::string("hipMalloc (FC1 sequences): ") + hipGetErrorString(e));
      return EXPECTO_ENOMEM;
    }
  }
  cap = rows;
  h->bytes += (size_t)rows * 640 * 4 * 3;
  return EXPECTO_OK;
}

// D1 / D2 / DD of `blocks` blocks of T conv6 rows at a stride of s rows (tab: alt blocks, see fk_seq_h2)
int fk_sequences(expecto_beluga* h, const float* x, long long blocks, int T, int s, const int* tab, int n_ph,
                 hipStream_t st, const int* gres = nullptr, int set = 0) {
  int rc;
  if ((rc = fk_seq_alloc(h, blocks * s, set))) return rc;
  float* const* out = set ? h->fk_aseq : h->fk_seq;
  LayerTimer lt(h, 7, st);   // the sequences are timed with the FC1 reduction (slot fc1_reduce)
  const long long nblk = blocks * 7;   // 7 workgroups of 4 residue walks per block
  EXPECTO_REQUIRE(nblk > 0 && nblk < (1LL << 31), "FC1 sequence grid");
  fk_seq_h2<<<dim3((unsigned)nblk), dim3(320), 0, st>>>(x, T, s, tab, n_ph, gres, out[0], out[1], out[2], h->ovf);
  return check_launch("fk_seq_h2");
}

// Which products a window set needs: product g's group rows are cnt[g] starts at g_rows + off[g].
struct FkProducts {
  const long long* g_rows;
  int off[9];
  int cnt[9];
  int lay[9];   // partial-row layout counts (0: cnt); an in-place alt launch runs cnt <= lay rows of the ref layout
};

// FC1 output rows of n windows from their kFkParts partial rows each (prow), fk_reduce_h2
int fk_reduce(expecto_beluga* h, const float* part, const int* prow, int n, float* h1, hipStream_t st) {
  LayerTimer lt(h, 7, st);
  const long long count4 = (long long)n * (kHidLd / 4);
  fk_reduce_h2<<<dim3((unsigned)((count4 + 255) / 256)), dim3(256), 0, st>>>(part, prow, count4, h->fc1b, h1, h->fk_cs,
                                                                           exp2i(h->sx[6]), h->ovf);
  return check_launch("fk_reduce_h2");
}

// Tile width of a full grouped FC1 launch over mtt M tiles (256 rows each): the 336-column tile
// (6 N tiles) unless 112-column tiles (18 N tiles, a third of the work each; gemm_kernel.h
// fc_h3w_tile NB 7, same bits) fit in one round of the chip's workgroups -- the per-window forwards
// of small batches (the reference's batch 32 / 200 calls: 9 M tiles, 54 workgroups on 256 CUs;
// FC1 525 -> ~185 us at batch 32).  EXPECTO_FC1_NARROW=0 / 1 forces the choice (same bits either way).
constexpr int kFcNarrowNb = 7;   // beluga_fc_h3w_narrow
static_assert(kHidLd % (16 * kFcNarrowNb) == 0 && kHidLd % FCW_BN == 0, "FC1 N tiles");
bool fc1_narrow(const expecto_beluga* h, long long mtt) {
  if (h->fc1_narrow >= 0) return h->fc1_narrow != 0;
  if (!h->narrow_scope) return false;
  // only when the narrow launch is one round of workgroups (batch 512, 2 narrow rounds against 1
  // wide: no gain measured)
  const long long cus = h->cus > 0 ? h->cus : 256;
  return mtt * (kHidLd / (16 * kFcNarrowNb)) <= cus;
}

// Batches of <= 32 rows (the reference's per-window batch): FC1 / FC2 on beluga_fc_h3s (32 x 32 tiles,
// a 9-stage ring; the same bits) where the narrow tiles would run: FC1 at batch 32 160 -> 125 us
// (32 x 48 tiles on a 7-stage ring: 145 us).  EXPECTO_FC_SKINNY=0 keeps the narrow tiles.
static_assert(kHidLd % (16 * FCS_NB) == 0 &&
                  (kNFeat + 16 * FCS_NB - 1) / (16 * FCS_NB) * 16 * FCS_NB <= (kNFeat + GBN - 1) / GBN * GBN,
              "skinny FC tiles");
bool fc_skinny(const expecto_beluga* h, long long rows) {
  return h->fc_skinny && rows <= 32 && (h->fc1_narrow >= 0 ? h->fc1_narrow != 0 : h->narrow_scope);
}

// One grouped launch of the Karatsuba FC1 over n windows: per product g with cnt[g] groups, its
// kFkSlabs K slabs, then the tail over the windows (w_rows: window starts), as split-K partial rows
// of `part` in that order (the layout prow was built for); then fk_reduce_h2 into h1.  x: conv6 rows
// (the product X@3 and the tail), seq: their D1 / D2 / DD.  mask (alt, in place): descriptor d runs
// only the M tiles with bit 0 of mask[d * tiles + tile] set.
int fk_fc1(expecto_beluga* h, const float* x, float* const* seq, const FkProducts& pr, const long long* w_rows, int n,
           const int* prow, float* h1, hipStream_t st, const unsigned* mask = nullptr, int tiles = 0,
           float* part = nullptr, long long part_cap = 0) {
  if (!part) {
    part = h->part;
    part_cap = (long long)std::max(h->fc_splits, kFkParts) * h->max_batch;
  }
  FcGroup G{};
  G.kb_total = kFkKbTotal;
  G.n_tiles = (kHidLd + FCW_BN - 1) / FCW_BN;
  G.n_store = kHidLd;
  G.ldc = kHidLd;
  const char* wb = reinterpret_cast<const char*>(h->fkw);
  long long row = 0;
  long long blk = 0;
  int mslot = 0;   // mask slot: descriptor order of the full layout (2 per product in use, then the tail)
  double macs = 0.0;
  auto add = [&](const float* A, const long long* ar, long long aoff, int kb0, int nk, int M, int lay) {
    FcDesc& d = G.d[G.n];
    d.A = A;
    d.a_rows = ar;
    d.a_off = aoff;
    d.Bp = wb + (long long)kb0 * 128;
    d.C = part + row * kHidLd;
    d.mask = mask ? mask + (size_t)mslot * tiles : nullptr;
    ++mslot;
    d.M = M;
    d.m_tiles = (M + X6P_BM - 1) / X6P_BM;
    d.nk = nk;
    d.blk0 = (int)blk;
    blk += (long long)d.m_tiles * G.n_tiles;
    row += lay;
    macs += (double)M * kFc1Out * nk * GBK;
    ++G.n;
  };
  for (int g = 0; g < 9; ++g) {
    const int lay = pr.lay[g] ? pr.lay[g] : pr.cnt[g];
    for (int s = 0; lay > 0 && s < kFkSlabs; ++s) {
      if (pr.cnt[g] > 0)
        add(kFkSeq[g] ? seq[kFkSeq[g] - 1] : x, pr.g_rows + pr.off[g], 25LL * kFkBlk[g] * 640 + (long long)s * kFkK / kFkSlabs,
            g * kFkKb + s * kFkKb / kFkSlabs, kFkKb / kFkSlabs, pr.cnt[g], lay);
      else {
        row += lay;   // (in-place alt launch: no alt group needs this product; keep the ref layout)
        ++mslot;
      }
    }
  }
  add(x, w_rows, 100LL * 640, 9 * kFkKb, kFkTailK / GBK, n, n);
  EXPECTO_REQUIRE(G.n <= FCK_MAX && blk < (1LL << 31), "Karatsuba FC1 descriptors");
  EXPECTO_REQUIRE(row <= part_cap, "Karatsuba FC1 partial rows");
  {
    LayerTimer lt(h, 6, st);
    if (h->profiling) {
      if (!mask) {
        h->macs[h->timer_base + 6] += macs;
      } else {   // executed share of the masked descriptors, counted on the device (no sync)
        for (int i = 0; i < G.n; ++i) {
          const FcDesc& d = G.d[i];
          int rc = count_desc_macs(h, d.mask, d.m_tiles, (double)d.M / d.m_tiles * kFc1Out * d.nk * GBK, st);
          if (rc) return rc;
        }
      }
    }
    G.rr = mask ? 0 : 1;   // full launches: M tiles dealt round robin to the 8 XCDs (gemm_kernel.h)
    const long long mtt = blk / G.n_tiles;
    const bool narrow = !mask && fc1_narrow(h, mtt);
    if (narrow) {   // 112-column tiles: same bits, 3x the workgroups
      G.n_tiles = kHidLd / (16 * kFcNarrowNb);
      for (int i = 0; i < G.n; ++i) G.d[i].blk0 = G.d[i].blk0 / (kHidLd / FCW_BN) * G.n_tiles;
    }
    const long long grid = G.rr ? (mtt + 7) / 8 * 8 * G.n_tiles : mtt * G.n_tiles;
    if (narrow)
      beluga_fc_h3k_narrow<<<dim3((unsigned)grid), dim3(512), 0, st>>>(G);
    else
      beluga_fc_h3k<0><<<dim3((unsigned)grid), dim3(512), 0, st>>>(G);
    int rc = check_launch("beluga_fc_h3k");
    if (rc) return rc;
  }
  return prow ? fk_reduce(h, part, prow, n, h1, st) : EXPECTO_OK;
}

// A window of the segment path for the Karatsuba FC1: its conv6 block (segment - s0, pool2 phase) and
// offset in conv6 rows (as seg_a_rows computes them); its role is its 25-row step mod 4 and its
// group the windows of its block with the same group start off6 - 25 role.
struct FkWin {
  int w, blk, off6;
};
int fk_role_of(int off6) { return (off6 / 25) & 3; }
FkWin fk_win(int w, const int* win_seg, const int* win_off, int s0, bool rc, int L, int n_ph, const int* ph_idx) {
  const int o = rc ? L - kLen - win_off[w] : win_off[w];
  const int q = o >> 2, p = q & 3;
  return {w, (win_seg[w] - s0) * n_ph + ph_idx[p], (q - p) >> 2};
}
bool fk_same_group(const FkWin& a, const FkWin& b) {
  return a.blk == b.blk && a.off6 - 25 * fk_role_of(a.off6) == b.off6 - 25 * fk_role_of(b.off6);
}

// Tables of windows ws[i0, i1) (whole groups, group order) for fk_fc1: per product the starts of
// the groups that need it (element offsets into the block rows, T6 rows per block) and each
// window's partial rows, in fk_fc1's descriptor order (products, slabs, then the tail).
void fk_slice_tables(const std::vector<FkWin>& ws, int i0, int i1, int T6, std::vector<long long>& grows,
                     FkProducts& pr, std::vector<int>& prow, std::vector<int>* rgrp = nullptr,
                     std::vector<int>* ginfo = nullptr) {
  const int n = i1 - i0;
  std::vector<int> gi(n);
  std::vector<long long> gst;
  std::vector<unsigned> need;
  for (int i = i0; i < i1; ++i) {
    const FkWin& w = ws[i];
    if (i == i0 || !fk_same_group(w, ws[i - 1])) {
      gst.push_back(((long long)w.blk * T6 + w.off6 - 25 * fk_role_of(w.off6)) * 640);
      need.push_back(0u);
    }
    gi[i - i0] = (int)gst.size() - 1;
    for (int j = 0; j < 4; ++j) need.back() |= 1u << kFkRole[fk_role_of(w.off6)][j];
    if (ginfo && gi[i - i0] * 2 == (int)ginfo->size()) {   // (block, start row) of a new group
      ginfo->push_back(w.blk);
      ginfo->push_back(w.off6 - 25 * fk_role_of(w.off6));
    }
  }
  const int ng = (int)gst.size();
  std::vector<int> ridx((size_t)9 * ng, -1);
  grows.clear();
  if (rgrp) rgrp->clear();
  for (int g = 0; g < 9; ++g) {
    pr.off[g] = (int)grows.size();
    int c = 0;
    for (int k = 0; k < ng; ++k)
      if ((need[k] >> g) & 1u) {
        ridx[(size_t)g * ng + k] = c++;
        grows.push_back(gst[k]);
        if (rgrp) rgrp->push_back(k);
      }
    pr.cnt[g] = c;
    pr.lay[g] = 0;
  }
  int base[9][kFkSlabs] = {};
  int row = 0;
  for (int g = 0; g < 9; ++g)
    for (int s = 0; pr.cnt[g] > 0 && s < kFkSlabs; ++s) {
      base[g][s] = row;
      row += pr.cnt[g];
    }
  prow.assign((size_t)n * kFkParts, 0);
  for (int i = 0; i < n; ++i) {
    const int role = fk_role_of(ws[i0 + i].off6);
    for (int j = 0; j < 4; ++j) {
      const int g = kFkRole[role][j];
      for (int s = 0; s < kFkSlabs; ++s) prow[(size_t)i * kFkParts + kFkSlabs * j + s] = base[g][s] + ridx[(size_t)g * ng + gi[i]];
    }
    prow[(size_t)i * kFkParts + kFkParts - 1] = row + i;
  }
}

// Karatsuba FC1 + FC2 of R windows whose conv6 rows are at act (106 rows per window), each alone in
// the handle's per-window role; mask (alt, in place over the same R rows' ref partials): per
// descriptor and M tile, see fk_window_mask.
int fk_windows(expecto_beluga* h, const float* act, int R, float* y, hipStream_t st, const long long* c_rows,
               const unsigned* mask = nullptr, int tiles = 0) {
  int rc;
  if ((rc = fk_tables(h)) || (rc = fk_sequences(h, act, R, 106, 106, nullptr, 1, st))) return rc;
  fk_window_tables<<<dim3((R + 255) / 256), dim3(256), 0, st>>>(R, 106, h->fk_role, h->fk_grows, h->fk_wrows, h->fk_prow);
  if ((rc = check_launch("fk_window_tables"))) return rc;
  FkProducts pr{h->fk_grows, {}, {}, {}};
  for (int j = 0; j < 4; ++j) pr.cnt[kFkRole[h->fk_role][j]] = R;
  if ((rc = fk_fc1(h, act, h->fk_seq, pr, h->fk_wrows, R, h->fk_prow, h->h1, st, mask, tiles))) return rc;
  return run_fc2(h, h->h1, R, y, st, c_rows);
}

// Profiling: the executed MACs of an alt FC1 that runs only the masked split-K slabs of its
// `tiles` M tiles (nb rows) go to the device counter of the fc1_delta slot.
int count_slab_macs(expecto_beluga* h, const unsigned* mask, int tiles, long long nb, hipStream_t st) {
  if (!h->macs_d) {
    float* f = nullptr;
    int rc = dalloc(h, &f, 4 * kNumLayers);
    if (rc) return rc;
    h->macs_d = reinterpret_cast<double*>(f);
    EXPECTO_HIP_CHECK(hipMemsetAsync(h->macs_d, 0, 2 * kNumLayers * sizeof(double), st));
  }
  const double per_bit = (double)nb * kFc1Out * kFc1In / ((double)tiles * h->fc_splits);
  slab_macs<<<dim3(1), dim3(64), 0, st>>>(mask, tiles, per_bit, h->macs_d + kNumLayers + 6);   // fc1_delta
  return check_launch("slab_macs");
}

// Profiling: executed MACs of one masked descriptor of the grouped Karatsuba FC1 (set M-tile bits x
// per_tile MACs) into the device counter of the current FC1 slot.
int count_desc_macs(expecto_beluga* h, const unsigned* mask, int tiles, double per_tile, hipStream_t st) {
  if (!h->macs_d) {
    float* f = nullptr;
    int rc = dalloc(h, &f, 4 * kNumLayers);
    if (rc) return rc;
    h->macs_d = reinterpret_cast<double*>(f);
    EXPECTO_HIP_CHECK(hipMemsetAsync(h->macs_d, 0, 2 * kNumLayers * sizeof(double), st));
  }
  slab_macs<<<dim3(1), dim3(64), 0, st>>>(mask, tiles, per_tile, h->macs_d + h->timer_base + 6);
  return check_launch("slab_macs");
}

// One chunk of nb independent windows; conv1 input from x (one-hot) or codes.
int forward_chunk(expecto_beluga* h, const float* x, const uint8_t* codes, long long code_stride, int n_src,
                  int mode, long long row0, int nb, float* y, hipStream_t st) {
  int rc;
  g_precision = h->precision;
  g_conv_ea = h->conv_ea;
  struct Scope {
    expecto_beluga* h;
    ~Scope() { h->narrow_scope = false; }
  } scope{h};
  h->narrow_scope = true;
  const bool kmer = use_kmer(h, x);
  const bool fuse = !kmer && fuse_conv1(h, x);
  const C1Src f1{codes, code_stride, n_src, mode, row0, kLen};
  if (!kmer && !fuse && (rc = run_conv1(h, x, codes, code_stride, n_src, mode, row0, nb, kLen, kS1, st))) return rc;
  float* src = h->P;
  float* dst = h->Q;
  for (int l = 0; l < 5; ++l) {
    const ConvGeo& g = kConv[l];
    if (l == 0 && kmer)
      rc = run_conv2_kmer(h, f1, nb, g.t_valid, g.s_out, dst, st);
    else
      rc = run_conv(h, l, src, dst, nb, g.s_in, g.t_valid, g.s_out, g.pool != 0, st, l == 0 && fuse ? &f1 : nullptr);
    if (rc) return rc;
    std::swap(src, dst);
  }
  if (fk_use(h)) return fk_windows(h, src, nb, y, st, nullptr);   // FC1 as the block Karatsuba, role fk_role
  return run_fc(h, src, nullptr, nb, y, st);  // src = act5 (buffer Q), 106 x 640 rows per window
}

// Alt-run buffers, sized for max_batch blocks (a window, or a (segment, phase) block):
// the largest input patch (27 x 640) and run (20 x 640), + Toeplitz over-read pad.
int ensure_delta(expecto_beluga* h) {
  if (h->DA) return EXPECTO_OK;
  const size_t pad = 16 * 640;
  const size_t da = (size_t)h->max_batch * kDA[6] * 640 + pad, dd = (size_t)h->max_batch * kDW[6] * 640 + pad;
  float *pc = nullptr, *tb = nullptr;
  int rc;
  if ((rc = dalloc(h, &h->DA, act_alloc(da))) || (rc = dalloc(h, &h->D0, act_alloc(dd))) ||
      (rc = dalloc(h, &h->D1, act_alloc(dd))) || (rc = dalloc(h, &pc, (size_t)h->max_batch * kC1PatStride / 4)) ||
      (rc = dalloc(h, &tb, (size_t)h->max_batch * kSegTab)) ||
      (rc = dalloc(h, &h->slab_mask, (size_t)h->max_batch / 64 + 64)))
    return rc;
  h->delta_codes = reinterpret_cast<uint8_t*>(pc);
  h->seg_tab = reinterpret_cast<int*>(tb);
  if (h->overlap) {
    EXPECTO_HIP_CHECK(hipStreamCreateWithFlags(&h->st2, hipStreamNonBlocking));
    for (hipEvent_t& e : h->pev) EXPECTO_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  return EXPECTO_OK;
}

// ---- segment path: windows that are slices of longer sequences share the trunk --------
// A segment of L codes (L % 4 == 0); a window at offset o (o % 4 == 0, o + 2000 <= L).
// conv1..conv4 run once over the segment; pool1 is fused into conv2 (phase 0 serves every
// window since o % 4 == 0); pool2 runs separately for each phase p = (o/4) % 4 present;
// conv5/conv6 run per (segment, phase) block; FC1 reads each window's 106 conv6 rows
// through a row table.  Every per-window output element is computed with the same operands
// and K order as the per-window path, so results are bit-identical to it.
struct SegGeo {
  int L, T1, S1, P1, T3, T4, S5, T5, T6;
  size_t p_rows_floats, q_rows_floats;  // per segment, given n_ph phases
};

SegGeo seg_geo(int L, int n_ph) {
  SegGeo g{};
  g.L = L;
  g.T1 = L - 7;
  g.S1 = (g.T1 + 3) / 4 * 4;
  g.P1 = (g.T1 - 7) / 4;
  g.T3 = g.P1 - 7;
  g.T4 = g.T3 - 7;
  g.S5 = g.T4 / 4;        // rows of the phase-0 pool2 block (the longest)
  g.T5 = g.S5 - 7;
  g.T6 = g.T5 - 7;
  const size_t p_conv1 = (size_t)g.S1 * 320, p_conv3 = (size_t)((g.T3 + 3) & ~3) * 480, p_pool2 = (size_t)n_ph * g.S5 * 480,
               p_conv6 = (size_t)n_ph * g.T6 * 640;
  const size_t q_pool1 = (size_t)g.P1 * 320, q_conv4 = (size_t)g.T4 * 480, q_conv5 = (size_t)n_ph * g.T5 * 640;
  g.p_rows_floats = std::max(std::max(p_conv1, p_conv3), std::max(p_pool2, p_conv6));
  g.q_rows_floats = std::max(q_pool1, std::max(q_conv4, q_conv5));
  return g;
}

// Segment pairs: the alt segment s is segment s with code alt_code[s] (DEVICE) at var_pos[s]
// (HOST); its windows (the same offsets) go to y_alt.  Windows that hold the SNV get their
// alt trunk through per-layer alt runs and their own FC; the others equal their ref window
// and their rows are copied.
struct SegPairs {
  const int* var_pos;
  const uint8_t* alt_code;
  float* y_alt;
  long long strand_stride;
};

int forward_segments(expecto_beluga* h, const uint8_t* codes, int n_seg, int L, long long code_stride, int mode,
                     const int* win_seg, const int* win_off, const int* win_row, int n_win, float* y,
                     hipStream_t st, const SegPairs* pr = nullptr) {
  EXPECTO_REQUIRE(L >= kLen && L % 4 == 0, "segment length must be >= 2000 and a multiple of 4");
  g_precision = h->precision;
  g_conv_ea = h->conv_ea;
  int rc;
  if (pr && (rc = ensure_delta(h))) return rc;
  // phases present (fwd and, for BOTH, the mirrored rc offsets)
  int present[4] = {0, 0, 0, 0};
  for (int w = 0; w < n_win; ++w) {
    EXPECTO_REQUIRE(win_seg[w] >= 0 && win_seg[w] < n_seg, "window segment out of range");
    EXPECTO_REQUIRE(w == 0 || win_seg[w] >= win_seg[w - 1], "windows must be sorted by segment");
    const int o = win_off[w];
    EXPECTO_REQUIRE(o >= 0 && o % 4 == 0 && o + kLen <= L, "window offset must be 4-aligned inside the segment");
    // phases in the computed strands' coordinates (seg_a_rows: rc windows start at L - 2000 - o)
    if (mode != EXPECTO_STRAND_RC) present[(o >> 2) & 3] = 1;
    if (mode != EXPECTO_STRAND_FWD) present[((L - kLen - o) >> 2) & 3] = 1;
  }
  int n_ph = 0, ph[4] = {0, 0, 0, 0}, ph_idx[4] = {0, 0, 0, 0};
  for (int p = 0; p < 4; ++p)
    if (present[p]) {
      ph_idx[p] = n_ph;
      ph[n_ph++] = p;
    }
  const SegGeo g = seg_geo(L, std::max(n_ph, 1));
  const size_t p_cap = p_floats(h->max_batch) - 16 * 640, q_cap = q_floats(h->max_batch) - 16 * 640;
  const int seg_cap = (int)std::min<size_t>(p_cap / g.p_rows_floats, q_cap / g.q_rows_floats);
  EXPECTO_REQUIRE(seg_cap >= 1, "segment too long for this handle's workspace (raise max_batch)");
  // window ranges per segment
  std::vector<int> first(n_seg + 1, n_win);
  for (int w = n_win - 1; w >= 0; --w) first[win_seg[w]] = w;
  for (int sg = n_seg - 1; sg >= 0; --sg) first[sg] = std::min(first[sg], first[sg + 1]);
  if (n_win > h->win_cap) {
    for (int** b : {&h->win_seg_d, &h->win_off_d, &h->win_row_d, &h->alt_w_d, &h->copy_w_d, &h->fc_perm_d}) {
      if (*b) EXPECTO_HIP_CHECK(hipFree(*b));
      *b = nullptr;
    }
    h->win_cap = 0;
    for (int** b : {&h->win_seg_d, &h->win_off_d, &h->win_row_d, &h->alt_w_d, &h->copy_w_d})
      EXPECTO_HIP_CHECK(hipMalloc(b, n_win * sizeof(int)));
    EXPECTO_HIP_CHECK(hipMalloc(&h->fc_perm_d, 4 * n_win * sizeof(int)));   // per strand: FC order, alt order
    h->win_cap = n_win;
  }
  std::vector<int> alt_w, copy_w;
  if (pr) {
    for (int sg = 0; sg < n_seg; ++sg)
      EXPECTO_REQUIRE(pr->var_pos[sg] >= 0 && pr->var_pos[sg] < L, "variant position outside its segment");
    for (int w = 0; w < n_win; ++w) {
      const int q = pr->var_pos[win_seg[w]];
      (win_off[w] <= q && q < win_off[w] + kLen ? alt_w : copy_w).push_back(w);
    }
    if (n_seg > h->seg_var_cap) {
      if (h->seg_var_d) EXPECTO_HIP_CHECK(hipFree(h->seg_var_d));
      h->seg_var_d = nullptr;
      h->seg_var_cap = 0;
      EXPECTO_HIP_CHECK(hipMalloc(&h->seg_var_d, n_seg * sizeof(int)));
      h->seg_var_cap = n_seg;
    }
  }
  std::vector<HostCopy> copies;   // staged once the FC row order is known (below)
  if (pr) {
    copies.push_back({h->seg_var_d, pr->var_pos, n_seg * sizeof(int)});
    copies.push_back({h->alt_w_d, alt_w.data(), alt_w.size() * sizeof(int)});
    copies.push_back({h->copy_w_d, copy_w.data(), copy_w.size() * sizeof(int)});
  }
  if (win_row) {
    for (int w = 0; w < n_win; ++w) EXPECTO_REQUIRE(win_row[w] >= 0 && win_row[w] < n_win, "window row out of range");
    copies.push_back({h->win_row_d, win_row, n_win * sizeof(int)});
  }
  copies.push_back({h->win_seg_d, win_seg, n_win * sizeof(int)});
  copies.push_back({h->win_off_d, win_off, n_win * sizeof(int)});
  const int strands = mode == EXPECTO_STRAND_BOTH ? 2 : 1;
  // alt runs: one block per segment (conv1..4) or per (segment, phase) (pool2, conv5, conv6)
  const int blk_per_seg = pr ? std::max(n_ph, 1) : 0;
  // chunks of whole segments: grow while the segment buffers and the alt-run buffers (<= max_batch
  // blocks) fit.  The FC stage of a chunk runs in slices of <= max_batch windows (its workspace),
  // so a chunk is not bounded by its window count: one large chunk instead of several keeps every
  // conv launch's last partial round of 256 workgroups to one per chunk (the 200-window workload:
  // 96 segments per strand in one chunk instead of 40 + 40 + 16)
  std::vector<std::pair<int, int>> chunks;
  for (int s0 = 0; s0 < n_seg;) {
    int s1 = s0 + 1;
    while (s1 < n_seg && s1 - s0 < seg_cap && (long long)(s1 + 1 - s0) * blk_per_seg <= h->max_batch &&
           (h->seg_chunk_windows <= 0 || first[s1 + 1] - first[s0] <= h->seg_chunk_windows))
      ++s1;
    chunks.push_back({s0, s1});
    s0 = s1;
  }
  // Segment pairs: the FC rows of a chunk are its alt windows sorted by the SNV's position in
  // the window, then the other windows.  The ref FC1 runs in that order, and the alt FC1 over
  // the first rows recomputes only the split-K slabs its changed conv6 rows touch (a 256-row
  // tile then holds windows with nearly the same changed rows), reusing the ref partials.
  std::vector<int> fc_perm;
  if (pr) {
    fc_perm.resize((size_t)strands * n_win);
    std::vector<char> is_alt(n_win, 0);
    for (int w : alt_w) is_alt[w] = 1;
    for (int sd = 0; sd < strands; ++sd) {
      const bool rcs = (mode == EXPECTO_STRAND_RC) || sd == 1;
      int* out = fc_perm.data() + (size_t)sd * n_win;
      for (const auto& c : chunks) {
        const int w0 = first[c.first], w1 = first[c.second];
        int k = w0;
        std::vector<int> a;
        for (int w = w0; w < w1; ++w)
          if (is_alt[w]) a.push_back(w);
        std::stable_sort(a.begin(), a.end(), [&](int x, int y) {
          const int px = pr->var_pos[win_seg[x]] - win_off[x], py = pr->var_pos[win_seg[y]] - win_off[y];
          return rcs ? px > py : px < py;
        });
        for (int w : a) out[k++] = w;
        for (int w = w0; w < w1; ++w)
          if (!is_alt[w]) out[k++] = w;
      }
    }
    copies.push_back({h->fc_perm_d, fc_perm.data(), fc_perm.size() * sizeof(int)});
  }
  // FC1 as the block Karatsuba (f16x3): per strand and chunk the windows in group order (conv6
  // block, group start, role), the FC order of every launch and (segment pairs) the alt windows in
  // the same order; fc_perm_d holds [strand][n_win] FC orders, then [strand][n_win] alt orders
  // Segment pairs where more than a third of the windows hold the SNV (short sweeps: +-800, every
  // window) run the direct FC1 (role 4): an alt window's Karatsuba products mix rows 25-75 apart, so
  // nearly all of them reach the changed rows and the alt recompute outweighs the saving
  // (configs[2]: 14.4 k vs 16.6 k variants/s); the 200-window sweeps (5 % alt windows) gain.
  const bool fkm = fk_use_seg(h) && !(pr && 3 * alt_w.size() > (size_t)n_win);
  std::vector<std::vector<FkWin>> fk_ref, fk_alt;   // [strand * chunks + chunk]
  std::vector<char> fk_is_alt(pr ? n_win : 0, 0);
  for (int w : alt_w) fk_is_alt[w] = 1;
  if (fkm) {
    fc_perm.assign((size_t)4 * n_win, 0);
    for (int sd = 0; sd < strands; ++sd) {
      const bool rcs = (mode == EXPECTO_STRAND_RC) || sd == 1;
      for (const auto& c : chunks) {
        const int w0 = first[c.first], w1 = first[c.second];
        // group order: (segment pairs) the groups holding an alt window first, ordered by where the
        // SNV falls in the group (so an M tile of the in-place alt FC1 holds groups whose changed
        // products are the same and its masks stay sparse), then every other group; in a group its
        // windows by role
        struct Key {
          int cls;
          long long rel;
          int blk, G, off6, w;
        };
        std::vector<FkWin> ref, alt;
        std::vector<Key> key;
        std::map<std::pair<int, int>, int> galt;   // (block, group start) -> holds an alt window
        for (int w = w0; w < w1; ++w) {
          const FkWin fw = fk_win(w, win_seg, win_off, c.first, rcs, L, n_ph, ph_idx);
          ref.push_back(fw);
          if (pr && fk_is_alt[w]) {
            alt.push_back(fw);
            galt[{fw.blk, fw.off6 - 25 * fk_role_of(fw.off6)}] = 1;
          }
        }
        for (const FkWin& fw : ref) {
          const int G = fw.off6 - 25 * fk_role_of(fw.off6);
          const bool ga = pr && galt.count({fw.blk, G});
          long long rel = 0;
          if (ga) {
            const int q = pr->var_pos[win_seg[fw.w]];
            rel = (long long)(rcs ? L - 1 - q : q) - 16LL * G;
          }
          key.push_back({ga ? 0 : 1, rel, fw.blk, G, fw.off6, fw.w});
        }
        std::vector<int> ord(ref.size());
        for (size_t k = 0; k < ord.size(); ++k) ord[k] = (int)k;
        std::sort(ord.begin(), ord.end(), [&](int a, int b) {
          const Key &x = key[a], &y = key[b];
          return std::tie(x.cls, x.rel, x.blk, x.G, x.off6, x.w) < std::tie(y.cls, y.rel, y.blk, y.G, y.off6, y.w);
        });
        std::vector<FkWin> sorted;
        for (int k : ord) sorted.push_back(ref[k]);
        for (size_t k = 0; k < sorted.size(); ++k) fc_perm[(size_t)sd * n_win + w0 + k] = sorted[k].w;
        fk_ref.push_back(std::move(sorted));
        fk_alt.push_back(std::move(alt));
      }
    }
    if (pr) copies.pop_back();   // the pair order above is replaced by the group order
    copies.push_back({h->fc_perm_d, fc_perm.data(), fc_perm.size() * sizeof(int)});
  }
  // the tables are caller-owned (and local) host memory: stage them through pinned memory
  if ((rc = stage_copies(h, copies, st))) return rc;
  const long long strand_rows = pr ? pr->strand_stride : n_win;
  const int eb = act_bytes();
  hipStream_t sa = (pr && h->st2) ? h->st2 : st;     // alt runs of segment pairs
  const SegDims gd{L, g.T1, g.P1, g.T3, g.T4, g.S5, g.T5, g.T6};
  const int4 ph4 = make_int4(ph[0], ph[1], ph[2], ph[3]);
  for (int sd = 0; sd < strands; ++sd) {
    const bool is_rc = (mode == EXPECTO_STRAND_RC) || sd == 1;
    for (const auto& chunk : chunks) {
      const int s0 = chunk.first, s1 = chunk.second;
      const int w0 = first[s0], nw = first[s1] - first[s0];
      const int ns = s1 - s0;
      const long long nb = (long long)ns * n_ph;
      // Alt runs (segment pairs) on the handle's second stream `sa`: the alt input patch of
      // layer l is assembled from the ref input of layer l (`ref`, ref_rows per block; the
      // ref layer l reads it concurrently) and the previous alt run, then the layer's GEMM runs
      // on it beside the next ref layers.  The ref launch that next overwrites `ref` (ping-
      // pong) waits for the assembly (event `done`).  Same kernels, K order and weights.
      auto alt_asm = [&](int l, const float* ref, int ref_rows, const float* dprev, int wprev, int nbk, int ib,
                         int mult, int irp, int arows, hipEvent_t ready, hipEvent_t done) -> int {
        if (sa != st) {
          EXPECTO_HIP_CHECK(hipEventRecord(ready, st));
          EXPECTO_HIP_CHECK(hipStreamWaitEvent(sa, ready, 0));
        }
        const int row16 = kConv[l].cin * eb / 16;
        seg_delta_assemble<<<dim3(ns * nbk), dim3(256), 0, sa>>>(ref, ref_rows, dprev, wprev, h->seg_tab, nbk,
                                                                      ib, mult, irp, arows, row16, h->DA);
        int r = check_launch("seg_delta_assemble");
        if (!r && sa != st) EXPECTO_HIP_CHECK(hipEventRecord(done, sa));
        return r;
      };
      auto alt_gemm = [&](int l, int nbk, int arows, int w, bool pool, float* dnext) -> int {
        DeltaScope ds(h);
        return run_conv(h, l, h->DA, dnext, (long long)ns * nbk, arows, w, w, pool, sa);
      };
      auto st_wait = [&](hipEvent_t e) -> int {   // st: the alt work recorded in e is done
        if (sa != st) EXPECTO_HIP_CHECK(hipStreamWaitEvent(st, e, 0));
        return EXPECTO_OK;
      };
      if (pr && sa != st) {   // sa: the previous chunk's use of the alt buffers on st is done
        EXPECTO_HIP_CHECK(hipEventRecord(h->pev[0], st));
        EXPECTO_HIP_CHECK(hipStreamWaitEvent(sa, h->pev[0], 0));
      }
      // conv1 from codes: virtual rows = segments; rc mode mirrors inside the kernel (fused: inside
      // the conv2 launch)
      const bool kmer = use_kmer(h, nullptr);
      const bool fuse = !kmer && fuse_conv1(h, nullptr);
      const C1Src f1{codes + (long long)s0 * code_stride, code_stride, ns, is_rc ? EXPECTO_STRAND_RC : EXPECTO_STRAND_FWD,
                     0, L};
      if (!kmer && !fuse && (rc = run_conv1(h, nullptr, f1.codes, code_stride, ns, f1.mode, 0, ns, L, g.S1, st)))
        return rc;
      if (pr) {
        seg_delta_table<<<dim3((ns + 255) / 256), dim3(256), 0, sa>>>(h->seg_var_d, s0, ns, is_rc ? 1 : 0, gd, n_ph,
                                                                     ph4, h->seg_tab);
        if ((rc = check_launch("seg_delta_table"))) return rc;
        if (kmer || fuse) {   // the alt conv2 patch straight from the alt codes (k-mer table, or conv1 -> DA)
          seg_delta_codes2<<<dim3((ns + 4) / 5), dim3(5 * kC1PatStride), 0, sa>>>(
              codes, code_stride, pr->alt_code, s0, ns, is_rc ? 1 : 0, L, h->seg_tab, h->delta_codes);
          if ((rc = check_launch("seg_delta_codes2"))) return rc;
          DeltaScope ds(h);
          if (fuse && (rc = run_conv1(h, nullptr, h->delta_codes, kC1PatStride, ns, EXPECTO_STRAND_FWD, 0, ns, kC1Pat,
                                      kDA[2], sa, h->DA)))
            return rc;
        } else {
          seg_delta_codes<<<dim3((ns + 15) / 16), dim3(256), 0, sa>>>(codes, code_stride, pr->alt_code, s0, ns,
                                                                     is_rc ? 1 : 0, L, h->seg_tab, h->delta_codes);
          if ((rc = check_launch("seg_delta_codes"))) return rc;
          DeltaScope ds(h);
          if ((rc = run_conv1(h, nullptr, h->delta_codes, 16, ns, EXPECTO_STRAND_FWD, 0, ns, kDA[1], kDW[1], sa,
                              h->D0)))
            return rc;
        }
      }
      // conv2 + pool1 (P -> Q), conv3 (Q -> P), conv4 unpooled (P -> Q); alt runs D0 <-> D1
      if (pr && !kmer && !fuse && (rc = alt_asm(0, h->P, g.S1, h->D0, kDW[1], 1, 2, 4, 1, kDA[2], h->pev[1], h->pev[2])))
        return rc;
      if (kmer)
        rc = run_conv2_kmer(h, f1, ns, g.P1, g.P1, h->Q, st);
      else
        rc = run_conv(h, 0, h->P, h->Q, ns, g.S1, g.P1, g.P1, true, st, fuse ? &f1 : nullptr);
      if (rc) return rc;
      if (pr && kmer) {   // alt pooled conv2 rows [r2, r2 + kDW[2]) of each segment into D1
        DeltaScope ds(h);
        const C1Src fa{h->delta_codes, kC1PatStride, ns, EXPECTO_STRAND_FWD, 0, kC1Pat};
        if ((rc = run_conv2_kmer(h, fa, ns, kDW[2], kDW[2], h->D1, sa))) return rc;
      } else if (pr && ((!fuse && (rc = st_wait(h->pev[2]))) || (rc = alt_gemm(0, 1, kDA[2], kDW[2], true, h->D1)))) {
        return rc;
      }
      if (pr && (rc = alt_asm(1, h->Q, g.P1, h->D1, kDW[2], 1, 3, 1, 2, kDA[3], h->pev[3], h->pev[4]))) return rc;
      // conv3 rows at a 4-aligned stride per segment (T3p >= T3), so conv4's rows of every segment
      // start 4-aligned in its M index space: pool2 groups are then lane-local (epilogue_pool_ph02)
      const int T3p = (g.T3 + 3) & ~3;
      if ((rc = run_conv(h, 1, h->Q, h->P, ns, g.P1, g.T3, T3p, false, st))) return rc;
      if (pr && ((rc = st_wait(h->pev[4])) || (rc = alt_gemm(1, 1, kDA[3], kDW[3], false, h->D0)))) return rc;
      if (pr && (rc = alt_asm(2, h->P, T3p, h->D0, kDW[3], 1, 4, 1, 3, kA4u, h->pev[5], h->pev[6]))) return rc;
      // pool2 fused into conv4 (P -> phase blocks in Q, then P and Q trade roles for the rest of
      // the chunk: conv5 Q -> P, conv6 P -> Q, ... -- both hold a chunk's conv5 / conv6 rows, see
      // seg_geo), else conv4 unpooled (P -> Q) and a pool pass (Q -> P)
      const bool pfused = conv4_pool_fused(h, (long long)ns * T3p, n_ph, ph);
      struct PQSwap {
        expecto_beluga* h;
        bool on;
        ~PQSwap() {
          if (on) std::swap(h->P, h->Q);
        }
      } pq{h, false};
      if (pfused) {
        if ((rc = run_conv4_pool_fused(h, h->P, h->Q, ns, T3p, g.T4, g.S5, pr ? h->seg_tab : nullptr, st))) return rc;
        std::swap(h->P, h->Q);
        pq.on = true;
      } else if ((rc = run_conv(h, 2, h->P, h->Q, ns, T3p, g.T4, g.T4, false, st))) {
        return rc;
      }
      if (pr && ((rc = st_wait(h->pev[6])) || (rc = alt_gemm(2, 1, kA4u, kW4u, false, h->D1)))) return rc;
      if (!pfused) {  // pool2 phases (Q -> P)
        LayerTimer lt(h, 3, st);
        if (act_fmt() == 2 && h->pool_one_pass) {   // all phases in one pass over the conv4 rows
          dim3 grid((g.S5 + 3) / 4, ns);
          pool4_phases_h2m<<<grid, dim3(256), 0, st>>>(h->Q, g.T4, g.T4, 480, n_ph, ph4, g.S5, h->P);
        } else if (act_fmt() == 2) {
          dim3 grid((g.S5 + 3) / 4, ns * n_ph);
          pool4_phases_h2<<<grid, dim3(256), 0, st>>>(h->Q, g.T4, g.T4, 480, n_ph, ph4, g.S5, h->P);
        } else {
          dim3 grid(g.S5, ns * n_ph);
          pool4_phases<<<grid, dim3(480), 0, st>>>(h->Q, ns, g.T4, g.T4, 480, n_ph, ph4, g.S5, h->P, act_fmt());
        }
        if ((rc = check_launch("pool4_phases"))) return rc;
      }
      if (pr) {   // alt pool2 phases from the unpooled conv4 rows (Q) and the alt conv4 run
        if (sa != st) {
          EXPECTO_HIP_CHECK(hipEventRecord(h->pev[7], st));
          EXPECTO_HIP_CHECK(hipStreamWaitEvent(sa, h->pev[7], 0));
        }
        seg_delta_pool<<<dim3(kDW[4], (unsigned)nb), dim3(480), 0, sa>>>(pfused ? h->edge : h->Q, g.T4, h->D1, n_ph,
                                                                         ph4, h->seg_tab, act_fmt(), h->D0,
                                                                         pfused ? 1 : 0);
        if ((rc = check_launch("seg_delta_pool"))) return rc;
        if (sa != st) EXPECTO_HIP_CHECK(hipEventRecord(h->pev[8], sa));
        if ((rc = alt_asm(3, h->P, g.S5, h->D0, kDW[4], n_ph, 9, 1, 5, kDA[5], h->pev[9], h->pev[10]))) return rc;
        if ((rc = st_wait(h->pev[8]))) return rc;    // conv5 overwrites Q
      }
      // conv5 (P -> Q), conv6 (Q -> P) over (segment, phase) blocks
      if ((rc = run_conv(h, 3, h->P, h->Q, nb, g.S5, g.T5, g.T5, false, st))) return rc;
      if (pr && ((rc = st_wait(h->pev[10])) || (rc = alt_gemm(3, n_ph, kDA[5], kDW[5], false, h->D1)))) return rc;
      if (pr && (rc = alt_asm(4, h->Q, g.T5, h->D1, kDW[5], n_ph, 13, 1, 9, kDA[6], h->pev[11], h->pev[12])))
        return rc;
      if ((rc = run_conv(h, 4, h->Q, h->P, nb, g.T5, g.T6, g.T6, false, st))) return rc;
      if (pr) {
        if ((rc = alt_gemm(4, n_ph, kDA[6], kDW[6], false, h->D0))) return rc;
        if (sa != st) EXPECTO_HIP_CHECK(hipEventRecord(h->pev[13], sa));   // all alt runs of the chunk
      }
      if (nw > 0 && fkm) {
        // FC1 as the block Karatsuba: the conv6 blocks' D1 / D2 / DD, then slices of whole window
        // groups (<= fk_cap windows) in group order: window starts and output rows (seg_a_rows),
        // the slice's product and partial-row tables (host, staged), one grouped FC1 launch, FC2.
        // Segment pairs: the groups holding alt windows come first in the first slice; right after
        // it, the alt FC1 runs IN PLACE over that slice's partial rows -- the alt blocks' sequences
        // (Q), only the (product, slab, tail) partials the SNV's changed conv6 rows reach (masks per
        // M tile), the ref partials for the rest -- and the alt windows' rows are reduced and FC2'd.
        const int4 phi = make_int4(ph_idx[0], ph_idx[1], ph_idx[2], ph_idx[3]);
        const long long row_base = (long long)sd * strand_rows;
        const size_t ci = (size_t)sd * chunks.size() + (size_t)(&chunk - chunks.data());
        const long long cap = fk_cap(h);
        const std::vector<FkWin>& ws = fk_ref[ci];
        const int* perm = h->fc_perm_d + (size_t)sd * n_win + w0;
        // per conv6 block: its groups' start residue mod 100 (all equal on 200-bp sweeps), so the
        // sequences are formed only on the rows the products read; -2: a block no window reads
        std::vector<int> gres((size_t)nb, -2);
        for (const FkWin& w : ws) {
          const int r = (w.off6 - 25 * fk_role_of(w.off6)) % 100;
          int& e = gres[(size_t)w.blk];
          e = e == -2 ? r : (e == r ? r : -1);
        }
        if (nb > h->fk_gres_cap) {
          if (h->fk_gres) EXPECTO_HIP_CHECK(hipFree(h->fk_gres));
          h->fk_gres = nullptr;
          h->bytes -= (size_t)h->fk_gres_cap * sizeof(int);
          h->fk_gres_cap = 0;
          EXPECTO_HIP_CHECK(hipMalloc(&h->fk_gres, (size_t)nb * sizeof(int)));
          h->fk_gres_cap = nb;
          h->bytes += (size_t)nb * sizeof(int);
        }
        if ((rc = stage_copies(h, {{h->fk_gres, gres.data(), gres.size() * sizeof(int)}}, st)) || (rc = fk_tables(h)) ||
            (rc = fk_seg_buffers(h)) || (rc = fk_sequences(h, h->P, nb, g.T6, g.T6, nullptr, n_ph, st, h->fk_gres)))
          return rc;
        const bool has_alt = pr && !fk_alt[ci].empty();
        bool alt_ready = false;   // alt conv6 blocks (Q) and their sequences formed (once per chunk)
        for (size_t i0 = 0; i0 < ws.size();) {
          size_t i1 = i0;
          while (i1 < ws.size()) {   // whole groups, <= fk_cap windows
            size_t j = i1 + 1;
            while (j < ws.size() && fk_same_group(ws[j], ws[i1])) ++j;
            if (j - i0 > (size_t)cap && i1 > i0) break;
            i1 = j;
          }
          EXPECTO_REQUIRE(i1 - i0 <= (size_t)cap, "a Karatsuba FC1 window group exceeds the FC1 slice");
          const int fn = (int)(i1 - i0);
          std::vector<long long> grows;
          std::vector<int> prow, rgrp, ginfo;
          FkProducts prd{h->fk_grows, {}, {}, {}};
          fk_slice_tables(ws, (int)i0, (int)i1, g.T6, grows, prd, prow, &rgrp, &ginfo);
          if ((rc = stage_copies(h, {{h->fk_grows, grows.data(), grows.size() * sizeof(long long)},
                                     {h->fk_prow, prow.data(), prow.size() * sizeof(int)}}, st)))
            return rc;
          seg_a_rows<<<dim3((fn + 255) / 256), dim3(256), 0, st>>>(
              h->win_seg_d, h->win_off_d, win_row ? h->win_row_d : nullptr, perm + i0, 0, fn, s0, is_rc ? 1 : 0, L,
              n_ph, phi, g.T6, row_base, h->fk_arows, h->fk_crows);
          if ((rc = check_launch("seg_a_rows")) ||
              (rc = fk_fc1(h, h->P, h->fk_seq, prd, h->fk_arows, fn, h->fk_prow, h->fk_h1, st, nullptr, 0, h->fk_part,
                           kFkParts * cap)))
            return rc;
          for (int r0 = 0; r0 < fn; r0 += h->max_batch)   // FC2 over its workspace's max_batch rows at a time
            if ((rc = run_fc2(h, h->fk_h1 + (long long)r0 * kHidLd, std::min(h->max_batch, fn - r0), y, st,
                              h->fk_crows + r0)))
              return rc;
          // the slice's first groups holding alt windows (the alt groups lead the chunk's order, so
          // they fill the first slices) and their windows
          int n_ag = 0;
          size_t nw_pre = 0;
          for (size_t i = i0; has_alt && i < i1; ++i) {
            bool galt = false;
            size_t j = i;
            for (; j < i1 && fk_same_group(ws[j], ws[i]); ++j) galt |= fk_is_alt[ws[j].w] != 0;
            if (!galt) break;
            ++n_ag;
            nw_pre = j - i0;
            i = j - 1;
          }
          if (n_ag > 0) {
            FkProducts pa = prd;   // the alt groups' prefix of every product list, in the ref layout
            FkMaskDesc md{};
            for (int gq = 0; gq < 9; ++gq) {
              int c = 0;
              for (int i = 0; i < prd.cnt[gq]; ++i)
                if (rgrp[prd.off[gq] + i] < n_ag) ++c;
              pa.cnt[gq] = c;
              pa.lay[gq] = prd.cnt[gq];
              for (int sb = 0; prd.cnt[gq] > 0 && sb < kFkSlabs; ++sb) {
                md.g[md.n] = gq;
                md.s[md.n] = sb;
                md.off[md.n] = prd.off[gq];
                md.cnt[md.n] = c;
                ++md.n;
              }
            }
            md.nw = (int)nw_pre;
            std::vector<int> winfo, aperm, aprow;
            for (size_t i = 0; i < nw_pre; ++i) {
              winfo.push_back(ws[i0 + i].blk);
              winfo.push_back(ws[i0 + i].off6);
              if (fk_is_alt[ws[i0 + i].w]) {
                aperm.push_back(ws[i0 + i].w);
                aprow.insert(aprow.end(), prow.begin() + (long long)i * kFkParts, prow.begin() + (long long)(i + 1) * kFkParts);
              }
            }
            const int na = (int)aperm.size();
            const int tiles = (int)(cap / 256 + 1);
            if ((rc = stage_copies(h, {{h->fk_rgrp, rgrp.data(), rgrp.size() * sizeof(int)},
                                       {h->fk_ginfo, ginfo.data(), ginfo.size() * sizeof(int)},
                                       {h->fk_winfo, winfo.data(), winfo.size() * sizeof(int)},
                                       {h->fk_aperm, aperm.data(), aperm.size() * sizeof(int)},
                                       {h->fk_aprow, aprow.data(), aprow.size() * sizeof(int)}}, st)))
              return rc;
            if (!alt_ready) {
              if ((rc = st_wait(h->pev[13]))) return rc;   // alt conv6 runs (and the Q reads of their patches)
              seg_alt_blocks<<<dim3(kAltRows6, (unsigned)nb), dim3(64), 0, st>>>(h->P, h->D0, n_ph, g.T6, h->seg_tab,
                                                                                640 * eb / 16, h->Q);
              if ((rc = check_launch("seg_alt_blocks"))) return rc;
              DeltaScope ds(h);
              if ((rc = fk_sequences(h, h->Q, nb, g.T6, g.T6, h->seg_tab, n_ph, st, h->fk_gres, 1))) return rc;
              alt_ready = true;
            }
            EXPECTO_HIP_CHECK(hipMemsetAsync(h->fk_smask, 0, (size_t)(md.n + 1) * tiles * sizeof(unsigned), st));
            int rows_max = md.nw;
            for (int i = 0; i < md.n; ++i) rows_max = std::max(rows_max, md.cnt[i]);
            if (rows_max > 0) {
              fk_seg_mask<<<dim3((rows_max + 255) / 256, md.n + 1), dim3(256), 0, st>>>(
                  md, h->fk_rgrp, h->fk_ginfo, h->fk_winfo, h->seg_tab, n_ph, make_int4(0, 0, 0, 0), tiles, h->fk_smask);
              if ((rc = check_launch("fk_seg_mask"))) return rc;
            }
            DeltaScope ds(h);
            if ((rc = fk_fc1(h, h->Q, h->fk_aseq, pa, h->fk_arows, (int)nw_pre, nullptr, h->fk_h1, st, h->fk_smask, tiles,
                             h->fk_part, kFkParts * cap)) ||
                (na > 0 && (rc = fk_reduce(h, h->fk_part, h->fk_aprow, na, h->fk_h1, st))))
              return rc;
            if (na > 0) {
              seg_a_rows<<<dim3((na + 255) / 256), dim3(256), 0, st>>>(
                  h->win_seg_d, h->win_off_d, win_row ? h->win_row_d : nullptr, h->fk_aperm, 0, na, s0, is_rc ? 1 : 0,
                  L, n_ph, phi, g.T6, row_base, h->fk_arows, h->fk_crows);
              if ((rc = check_launch("seg_a_rows"))) return rc;
              for (int r0 = 0; r0 < na; r0 += h->max_batch)
                if ((rc = run_fc2(h, h->fk_h1 + (long long)r0 * kHidLd, std::min(h->max_batch, na - r0), pr->y_alt, st,
                                  h->fk_crows + r0)))
                  return rc;
            }
          }
          i0 = i1;
        }
        if (pr) {
          const int ic0 = (int)(std::lower_bound(copy_w.begin(), copy_w.end(), w0) - copy_w.begin());
          const int ic1 = (int)(std::lower_bound(copy_w.begin(), copy_w.end(), w0 + nw) - copy_w.begin());
          if (ic1 > ic0) {
            copy_rows<<<dim3(ic1 - ic0), dim3(256), 0, st>>>(y, pr->y_alt, h->copy_w_d + ic0,
                                                             win_row ? h->win_row_d : nullptr, row_base);
            if ((rc = check_launch("copy_rows"))) return rc;
          }
        }
      } else if (nw > 0) {
        const int4 phi = make_int4(ph_idx[0], ph_idx[1], ph_idx[2], ph_idx[3]);
        const long long row_base = (long long)sd * strand_rows;
        const int* widx = pr ? h->fc_perm_d + (size_t)sd * n_win + w0 : nullptr;   // FC row order
        // windows of this chunk holding the SNV (alt FC: the first n_alt FC rows, widx order) and
        // the others (copies of the ref rows)
        int n_alt = 0, ic0 = 0, ic1 = 0;
        if (pr) {
          n_alt = (int)(std::lower_bound(alt_w.begin(), alt_w.end(), w0 + nw) -
                        std::lower_bound(alt_w.begin(), alt_w.end(), w0));
          ic0 = (int)(std::lower_bound(copy_w.begin(), copy_w.end(), w0) - copy_w.begin());
          ic1 = (int)(std::lower_bound(copy_w.begin(), copy_w.end(), w0 + nw) - copy_w.begin());
        }
        // FC1 slices of <= max_batch rows (the FC1 workspace); the alt FC of a slice's alt rows
        // reuses that slice's ref partials, so it runs right after the slice's ref FC1.  FC2
        // unsplit: the slices' h1 rows (and FC2 output rows) gather into one FC2 launch of up to
        // fc2_rows rows (split FC2: per slice)
        const bool gather2 = h->fc2_splits == 1;
        int pend = 0;   // gathered h1 rows awaiting FC2
        auto flush2 = [&]() -> int {
          const int n2 = pend;
          pend = 0;
          return n2 ? run_fc2(h, h->h1, n2, y, st, h->c_rows) : EXPECTO_OK;
        };
        for (int f0 = 0; f0 < nw; f0 += h->max_batch) {
          const int fn = std::min(h->max_batch, nw - f0);
          if (gather2 && pend + fn > h->fc2_rows && (rc = flush2())) return rc;
          long long* crow = h->c_rows + (gather2 ? pend : 0);
          seg_a_rows<<<dim3((fn + 255) / 256), dim3(256), 0, st>>>(
              h->win_seg_d, h->win_off_d, win_row ? h->win_row_d : nullptr, widx ? widx + f0 : nullptr, w0 + f0,
              fn, s0, is_rc ? 1 : 0, L, n_ph, phi, g.T6, row_base, h->a_rows, crow);
          if ((rc = check_launch("seg_a_rows"))) return rc;
          if (gather2) {
            if ((rc = run_fc1(h, h->P, h->a_rows, fn, h1_rows(h, pend), st))) return rc;
            pend += fn;
          } else if ((rc = run_fc(h, h->P, h->a_rows, fn, y, st, h->c_rows))) {
            return rc;
          }
          const int na = std::min(n_alt - f0, fn);   // alt rows of this slice: [f0, f0 + na)
          if (na <= 0) continue;
          if (f0 == 0) {
            if ((rc = st_wait(h->pev[13]))) return rc;   // alt conv6 runs (and the Q reads of their patches)
            // alt conv6 blocks into Q (conv5 rows are dead): only the rows the alt windows read
            seg_alt_blocks<<<dim3(kAltRows6, (unsigned)nb), dim3(64), 0, st>>>(h->P, h->D0, n_ph, g.T6, h->seg_tab,
                                                                              640 * eb / 16, h->Q);
            if ((rc = check_launch("seg_alt_blocks"))) return rc;
          }
          long long* acrow = gather2 ? h->c_rows + h->fc2_rows : h->c_rows;   // alt rows apart
          seg_a_rows<<<dim3((na + 255) / 256), dim3(256), 0, st>>>(
              h->win_seg_d, h->win_off_d, win_row ? h->win_row_d : nullptr, widx + f0, 0, na, s0, is_rc ? 1 : 0,
              L, n_ph, phi, g.T6, row_base, h->a_rows, acrow);
          if ((rc = check_launch("seg_a_rows"))) return rc;
          const unsigned* mask = nullptr;
          double frac = 1.0;
          if (planes_gemm()) {
            const int tiles = (int)((na + gemm_bm() - 1) / gemm_bm());
            unsigned* md = reinterpret_cast<unsigned*>(h->slab_mask);
            EXPECTO_HIP_CHECK(hipMemsetAsync(md, 0, tiles * sizeof(unsigned), st));
            fc1_slab_mask_seg<<<dim3((na + 255) / 256), dim3(256), 0, st>>>(
                widx + f0, na, h->win_seg_d, h->win_off_d, s0, is_rc ? 1 : 0, L, phi, h->seg_tab, (int)gemm_bm(),
                kFc1In / h->fc_splits, md);
            if ((rc = check_launch("fc1_slab_mask_seg"))) return rc;
            mask = md;
            if (h->profiling) {   // executed share of the slabs, counted on the device (no sync)
              if ((rc = count_slab_macs(h, md, tiles, na, st))) return rc;
              frac = 0.0;
            }
          }
          DeltaScope ds(h);
          if (gather2) {
            float* h1a = h1_rows(h, h->fc2_rows);
            if ((rc = run_fc1(h, h->Q, h->a_rows, na, h1a, st, mask, frac, fn)) ||
                (rc = run_fc2(h, h1a, na, pr->y_alt, st, acrow)))
              return rc;
          } else if ((rc = run_fc(h, h->Q, h->a_rows, na, pr->y_alt, st, h->c_rows, mask, frac, fn))) {
            return rc;
          }
        }
        if ((rc = flush2())) return rc;   // the ref rows are read by copy_rows below
        if (pr) {
          if (ic1 > ic0) {
            copy_rows<<<dim3(ic1 - ic0), dim3(256), 0, st>>>(y, pr->y_alt, h->copy_w_d + ic0,
                                                             win_row ? h->win_row_d : nullptr, row_base);
            if ((rc = check_launch("copy_rows"))) return rc;
          }
        }
      }
      if (pr && (rc = st_wait(h->pev[13]))) return rc;   // every alt run of the chunk joined
    }
  }
  return EXPECTO_OK;
}
int forward_pairs(expecto_beluga* h, const uint8_t* ref, const uint8_t* alt, int n, long long stride,
                  const int* var_pos, int mode, float* y_ref, float* y_alt, long long strand_stride, hipStream_t st) {
  g_precision = h->precision;
  g_conv_ea = h->conv_ea;
  const int strands = mode == EXPECTO_STRAND_BOTH ? 2 : 1;
  int rc;
  if ((rc = ensure_delta(h))) return rc;
  const int eb = act_bytes();   // bytes per activation element
  const int nv_max = std::max(1, h->max_batch / strands);
  // Alt-delta launches go to a second stream (st2) so their few workgroups fill the rounds the
  // ref launches leave partly empty: alt layer l needs the ref layer l-1 output (event after the
  // ref launch that wrote it) and the ref layer l+1 launch, which overwrites that buffer (ping-
  // pong), waits until the alt patch of layer l has been assembled.
  hipStream_t sa = h->st2 ? h->st2 : st;
  auto order = [&](hipStream_t from, hipStream_t to, hipEvent_t e) -> int {
    if (from == to) return EXPECTO_OK;
    EXPECTO_HIP_CHECK(hipEventRecord(e, from));
    EXPECTO_HIP_CHECK(hipStreamWaitEvent(to, e, 0));
    return EXPECTO_OK;
  };
  for (int v0 = 0; v0 < n; v0 += nv_max) {
    const int nv = std::min(nv_max, n - v0), R = strands * nv;
    if ((rc = order(st, sa, h->pev[0]))) return rc;   // caller's inputs (and the previous chunk)
    // conv1: ref windows (full; fused: inside the conv2 launch) and the alt runs (15 codes -> 8
    // rows; fused: the whole alt conv2 patch, kC1Pat codes -> kDA[2] rows)
    const bool kmer = use_kmer(h, nullptr);
    const bool fuse = !kmer && fuse_conv1(h, nullptr);
    const C1Src f1{ref + (long long)v0 * stride, stride, nv, mode, 0, kLen};
    if (!kmer && !fuse && (rc = run_conv1(h, nullptr, f1.codes, stride, nv, mode, 0, R, kLen, kS1, st))) return rc;
    if (kmer || fuse) {
      delta_codes2<<<dim3((R + 4) / 5), dim3(5 * kC1PatStride), 0, sa>>>(alt, stride, nv, v0, var_pos, h->delta_codes, R);
      if ((rc = check_launch("delta_codes2"))) return rc;
      DeltaScope ds(h);
      if (fuse && (rc = run_conv1(h, nullptr, h->delta_codes, kC1PatStride, R, EXPECTO_STRAND_FWD, 0, R, kC1Pat, kDA[2],
                                  sa, h->DA)))
        return rc;
    } else {
      delta_codes<<<dim3((R + 15) / 16), dim3(256), 0, sa>>>(alt, stride, nv, v0, var_pos, h->delta_codes, R);
      if ((rc = check_launch("delta_codes"))) return rc;
      DeltaScope ds(h);
      if ((rc = run_conv1(h, nullptr, h->delta_codes, 16, R, EXPECTO_STRAND_FWD, 0, R, kDA[1], kDW[1], sa, h->D0)))
        return rc;
    }
    float* src = h->P;
    float* dst = h->Q;
    float* dprev = h->D0;
    float* dnext = h->D1;
    for (int l = 0; l < 5; ++l) {   // conv2..conv6 (layer index l+2 in the delta tables)
      const ConvGeo& g = kConv[l];
      const int L = l + 2;
      if ((rc = order(st, sa, h->pev[1 + 2 * l]))) return rc;   // src (ref layer l-1) written
      const bool fused = l == 0 && fuse;   // the alt conv2 patch is already in DA
      const bool tab = l == 0 && kmer;     // conv2 from the k-mer table (ref windows and alt patches)
      if (tab)
        rc = run_conv2_kmer(h, f1, R, g.t_valid, g.s_out, dst, st);
      else
        rc = run_conv(h, l, src, dst, R, g.s_in, g.t_valid, g.s_out, g.pool != 0, st, fused ? &f1 : nullptr);
      if (rc) return rc;
      const int row16 = g.cin * eb / 16;
      if (!fused && !tab) {
        delta_assemble<<<dim3(R), dim3(256), 0, sa>>>(src, g.s_in, dprev, L, row16, nv, v0, var_pos, h->DA);
        if ((rc = check_launch("delta_assemble"))) return rc;
      }
      if ((rc = order(sa, st, h->pev[2 + 2 * l]))) return rc;   // src read: ref l+1 may overwrite it
      DeltaScope ds(h);
      if (tab) {
        const C1Src fa{h->delta_codes, kC1PatStride, R, EXPECTO_STRAND_FWD, 0, kC1Pat};
        if ((rc = run_conv2_kmer(h, fa, R, kDW[L], kDW[L], dnext, sa))) return rc;
      } else if ((rc = run_conv(h, l, h->DA, dnext, R, kDA[L], kDW[L], kDW[L], g.pool != 0, sa))) {
        return rc;
      }
      std::swap(src, dst);
      std::swap(dprev, dnext);
    }
    if ((rc = order(sa, st, h->pev[11]))) return rc;   // alt conv6 runs done
    float* act6 = src;   // ref conv6 rows; dprev = the alt runs' conv6 rows
    pair_rows<<<dim3((R + 255) / 256), dim3(256), 0, st>>>(h->c_rows, R, nv, v0, strand_stride);
    if ((rc = check_launch("pair_rows"))) return rc;
    const bool fk = fk_use(h);
    if ((rc = fk ? fk_windows(h, act6, R, y_ref, st, h->c_rows) : run_fc(h, act6, nullptr, R, y_ref, st, h->c_rows)))
      return rc;
    pair_patch_apply<<<dim3(R), dim3(256), 0, st>>>(dprev, act6, nv, v0, var_pos, 640 * eb / 16);
    if ((rc = check_launch("pair_patch_apply"))) return rc;
    if (fk) {   // alt FC1: only the partials (product, slab, tail) the 20 changed conv6 rows reach, in place
      const int tiles = (R + X6P_BM - 1) / X6P_BM;
      EXPECTO_HIP_CHECK(hipMemsetAsync(h->fk_mask, 0, (size_t)kFkParts * tiles * sizeof(unsigned), st));
      fk_window_mask<<<dim3((R + 255) / 256), dim3(256), 0, st>>>(var_pos, nv, v0, R, h->fk_role, tiles, h->fk_mask);
      if ((rc = check_launch("fk_window_mask"))) return rc;
      DeltaScope ds(h);
      if ((rc = fk_windows(h, act6, R, y_alt, st, h->c_rows, h->fk_mask, tiles))) return rc;
      continue;
    }
    // alt FC1: only the split-K slabs the 20 changed conv6 rows touch (planes GEMMs)
    const unsigned* mask = nullptr;
    double frac = 1.0;
    if (planes_gemm()) {
      const int tiles = (int)((R + gemm_bm() - 1) / gemm_bm());
      unsigned* md = reinterpret_cast<unsigned*>(h->slab_mask);
      EXPECTO_HIP_CHECK(hipMemsetAsync(md, 0, tiles * sizeof(unsigned), st));
      fc1_slab_mask<<<dim3((R + 255) / 256), dim3(256), 0, st>>>(var_pos, nv, v0, R, (int)gemm_bm(),
                                                                  kFc1In / h->fc_splits, md);
      if ((rc = check_launch("fc1_slab_mask"))) return rc;
      mask = md;
      if (h->profiling) {   // executed share of the slabs, counted on the device (no sync)
        if ((rc = count_slab_macs(h, md, tiles, R, st))) return rc;
        frac = 0.0;
      }
    }
    DeltaScope ds(h);
    if ((rc = run_fc(h, act6, nullptr, R, y_alt, st, h->c_rows, mask, frac))) return rc;
  }
  return EXPECTO_OK;
}

// ---- f16x3 set-up: fp16 weight planes + activation-scale calibration -----------------------
constexpr int kCalibWindows = 256;

// column scales of every GEMM layer from the current sx[] and the weight exponents
int f16_col_scales(expecto_beluga* h, hipStream_t st) {
  const int np[7] = {npad_of(320), npad_of(480), npad_of(480), npad_of(640), npad_of(640), npad_of(kFc1Out),
                     npad_of(kNFeat)};
  for (int g = 0; g < 7; ++g) {
    col_scales<<<dim3((np[g] + 255) / 256), dim3(256), 0, st>>>(h->swd[g], np[g], h->sx[g], h->cs[g]);
    int rc = check_launch("col_scales");
    if (rc) return rc;
  }
  if (h->fkw) {   // the Karatsuba FC1 weights: FC1's input scale, their own row exponents
    col_scales<<<dim3((np[5] + 255) / 256), dim3(256), 0, st>>>(h->fk_sw, np[5], h->sx[5], h->fk_cs);
    return check_launch("col_scales (FC1 Karatsuba)");
  }
  return EXPECTO_OK;
}

// sx[b] = target - e, with the calibration maximum of boundary b = m * 2^e (m in [0.5, 1)):
// that maximum lands in (2^(target-1), 2^target] after scaling.
int f16_calibrate(expecto_beluga* h, hipStream_t st) {
  const int nb = std::min(kCalibWindows, h->max_batch);
  int rc;
  if (!h->calib && (rc = dalloc(h, &h->calib, (size_t)nb * kNFeat + (size_t)nb * kLen / 4 + 64))) return rc;
  float* buf = h->calib;
  float* y = buf;
  uint8_t* codes = reinterpret_cast<uint8_t*>(buf + (size_t)nb * kNFeat);
  unsigned* amax = reinterpret_cast<unsigned*>(buf + (size_t)nb * kNFeat + (size_t)nb * kLen / 4);
  EXPECTO_HIP_CHECK(hipMemsetAsync(amax, 0, 8 * sizeof(unsigned), st));
  const long long nc = (long long)nb * kLen;
  calib_codes<<<dim3((unsigned)((nc + 255) / 256)), dim3(256), 0, st>>>(codes, nc, 0x5eed1234u);
  if ((rc = check_launch("calib_codes"))) return rc;
  const int saved = g_precision;
  const bool prof = h->profiling;
  h->profiling = false;
  g_precision = EXPECTO_PRECISION_BF16X6;
  auto amax_of = [&](const float* A, long long groups, int s_rows, int t_valid, int C, int b) {
    act_max<<<dim3(1024), dim3(256), 0, st>>>(A, groups, s_rows, t_valid, C, C, amax + b);
    return check_launch("act_max");
  };
  rc = run_conv1(h, nullptr, codes, kLen, nb, EXPECTO_STRAND_FWD, 0, nb, kLen, kS1, st);
  if (!rc) rc = amax_of(h->P, nb, kS1, kLen - 7, 320, 0);
  float* src = h->P;
  float* dst = h->Q;
  for (int l = 0; l < 5 && !rc; ++l) {
    const ConvGeo& g = kConv[l];
    rc = run_conv(h, l, src, dst, nb, g.s_in, g.t_valid, g.s_out, g.pool != 0, st);
    if (!rc) rc = amax_of(dst, nb, g.s_out, g.t_valid, g.cout, l + 1);
    std::swap(src, dst);
  }
  if (!rc) rc = run_fc(h, src, nullptr, nb, y, st);
  if (!rc) {
    act_max<<<dim3(1024), dim3(256), 0, st>>>(h->h1, nb, 1, 1, kHidLd, kFc1Out, amax + 6);
    rc = check_launch("act_max");
  }
  g_precision = saved;
  h->profiling = prof;
  if (rc) return rc;
  unsigned bits[7];
  EXPECTO_HIP_CHECK(hipMemcpyAsync(bits, amax, sizeof(bits), hipMemcpyDeviceToHost, st));
  EXPECTO_HIP_CHECK(hipStreamSynchronize(st));
  for (int b = 0; b < 7; ++b) {
    float m;
    std::memcpy(&m, &bits[b], sizeof(float));
    int e = 0;
    (void)std::frexp(m, &e);
    h->sx[b] = (m > 0.f && std::isfinite(m)) ? std::min(40, std::max(-40, h->f16_target - e)) : 0;
  }
  return f16_col_scales(h, st);
}

int f16_prepare(expecto_beluga* h, hipStream_t st) {
  if (h->f16_ready) return EXPECTO_OK;
  int rc;
  struct L {
    const float* w;
    int rows;
    long long K;
  } layers[7] = {{h->wt[0], npad_of(320), 8LL * 320}, {h->wt[1], npad_of(480), 8LL * 320},
                 {h->wt[2], npad_of(480), 8LL * 480}, {h->wt[3], npad_of(640), 8LL * 480},
                 {h->wt[4], npad_of(640), 8LL * 640}, {h->fc1w, npad_of(kFc1Out), kFc1In},
                 {h->fc2w, npad_of(kNFeat), kHidLd}};
  if (!h->ovf) {
    float* f = nullptr;
    if ((rc = dalloc(h, &f, 1))) return rc;
    h->ovf = reinterpret_cast<int*>(f);
    EXPECTO_HIP_CHECK(hipMemsetAsync(h->ovf, 0, sizeof(int), st));
  }
  for (int g = 0; g < 7; ++g) {
    const L& y = layers[g];
    float* swf = nullptr;
    // conv3 / conv4: 32 zero rows past the 480 (4 N tiles of 128 columns for small batches, conv_narrow)
    const int zrows = (g == 1 || g == 2) ? 4 * 128 - y.rows : 0;
    if ((rc = dalloc(h, &swf, y.rows)) || (rc = dalloc(h, &h->cs[g], y.rows)) ||
        (rc = dalloc(h, &h->wh[g], (size_t)(y.rows + zrows) * y.K)))
      return rc;
    h->swd[g] = reinterpret_cast<int*>(swf);
    row_scale_exp<<<dim3(y.rows), dim3(256), 0, st>>>(y.w, (int)y.K, h->swd[g]);
    if ((rc = check_launch("row_scale_exp"))) return rc;
    const long long n4 = (long long)y.rows * y.K / 4;
    split_planes_h2<<<dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st>>>(
        y.w, y.rows, (int)y.K, h->swd[g], reinterpret_cast<_Float16*>(h->wh[g]));
    if ((rc = check_launch("split_planes_h2"))) return rc;
  }
  {  // conv1 (beluga_conv1_h3): weights repacked to k = tap*4 + ci, per-row scaled planes
    float *w1r = nullptr, *sw1 = nullptr;
    if ((rc = dalloc(h, &w1r, 320 * 32)) || (rc = dalloc(h, &sw1, 320)) || (rc = dalloc(h, &h->cs1, 320)) ||
        (rc = dalloc(h, &h->w1h, 320 * 32)))
      return rc;
    repack_conv1<<<dim3(40), dim3(256), 0, st>>>(h->w1, w1r);
    row_scale_exp<<<dim3(320), dim3(256), 0, st>>>(w1r, 32, reinterpret_cast<int*>(sw1));
    split_planes_h2<<<dim3(10), dim3(256), 0, st>>>(w1r, 320, 32, reinterpret_cast<int*>(sw1),
                                                    reinterpret_cast<_Float16*>(h->w1h));
    col_scales<<<dim3(2), dim3(256), 0, st>>>(reinterpret_cast<int*>(sw1), 320, 0, h->cs1);
    if ((rc = check_launch("conv1 planes"))) return rc;
  }
  if (h->fk_on) {   // FC1 block Karatsuba: the 9 products' weights + the tail, fp64 sums rounded once,
    const int np1 = npad_of(kFc1Out);   // one exponent per row over all of them (a shared column unscale)
    float* wk = nullptr;
    EXPECTO_HIP_CHECK(hipMalloc(&wk, (size_t)np1 * kFkKTotal * sizeof(float)));
    float *swf = nullptr;
    if ((rc = dalloc(h, &swf, np1)) || (rc = dalloc(h, &h->fk_cs, np1)) ||
        (rc = dalloc(h, &h->fkw, (size_t)np1 * kFkKTotal))) {
      (void)hipFree(wk);
      return rc;
    }
    h->fk_sw = reinterpret_cast<int*>(swf);
    const long long tot = (long long)np1 * kFkKTotal;
    fk_weights<<<dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st>>>(h->fc1w, np1, wk);
    row_scale_exp<<<dim3(np1), dim3(256), 0, st>>>(wk, (int)kFkKTotal, h->fk_sw);
    split_planes_h2<<<dim3((unsigned)((tot / 4 + 255) / 256)), dim3(256), 0, st>>>(
        wk, np1, (int)kFkKTotal, h->fk_sw, reinterpret_cast<_Float16*>(h->fkw));
    rc = check_launch("FC1 Karatsuba weights");
    (void)hipStreamSynchronize(st);
    (void)hipFree(wk);
    if (rc) return rc;
  }
  if ((rc = f16_calibrate(h, st))) return rc;
  h->f16_ready = true;
  return EXPECTO_OK;
}

// Run one public call; on the f16x3 path check the overflow flag afterwards and, if an
// activation did not fit fp16, recompute the whole call with bf16x6.  In deferred mode the
// flag stays on the device for expecto_beluga_overflow_pending (the caller's release point).
// The per-call checks' flag words into pinned, device-mapped host memory (out[0] the f16x3 overflow
// flag, out[1] the one-hot check flag, which is reset for the next call): one tiny kernel on the
// call's stream instead of a copy-engine blit per flag plus a memset; visible to the host after the
// stream sync that follows.
__global__ void take_flags(const int* __restrict__ ovf, int* __restrict__ bad, int* __restrict__ out) {
  if (threadIdx.x != 0) return;
  // agent-scope loads: vector loads past the CU's caches (the flags were stored by earlier kernels)
  if (ovf) out[0] = __hip_atomic_load(ovf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (bad) {
    out[1] = __hip_atomic_load(bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *bad = 0;
  }
}

template <class F>
int run_checked(expecto_beluga* h, hipStream_t st, F&& fn) {
  if (h->precision != EXPECTO_PRECISION_F16X3 || h->ovf_deferred) return fn();
  int rc = fn();
  if (rc) return rc;
  int* flag = h->hflags;   // pinned, device-mapped: one tiny kernel writes it (no copy-engine blit)
  take_flags<<<1, 64, 0, st>>>(h->ovf, nullptr, h->hflags_d);
  EXPECTO_HIP_CHECK(hipGetLastError());
  EXPECTO_HIP_CHECK(hipStreamSynchronize(st));
  if (!*flag) return EXPECTO_OK;
  EXPECTO_HIP_CHECK(hipMemsetAsync(h->ovf, 0, sizeof(int), st));
  h->fallbacks += 1;
  h->precision = EXPECTO_PRECISION_BF16X6;
  rc = fn();
  h->precision = EXPECTO_PRECISION_F16X3;
  return rc;
}
}  // namespace

extern "C" {

int expecto_beluga_create(int device, const float* const* params, int max_batch, void* stream,
                          expecto_beluga_t* out) {
  EXPECTO_REQUIRE(out != nullptr && params != nullptr, "null argument");
  EXPECTO_REQUIRE(max_batch > 0 && max_batch <= (1 << 16), "max_batch out of range");
  for (int i = 0; i < EXPECTO_BELUGA_NPARAMS; ++i) EXPECTO_REQUIRE(params[i] != nullptr, "null parameter pointer");
  EXPECTO_HIP_CHECK(hipSetDevice(device));
  hipStream_t st = as_stream(stream);
  auto* h = new expecto_beluga();
  h->device = device;
  h->max_batch = max_batch;
  if (hipDeviceGetAttribute(&h->cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) h->cus = 0;
  int rc = 0;
  auto fail = [&](int code) {
    expecto_beluga_destroy(h);
    return code;
  };
  if ((rc = dalloc(h, &h->w1, 320 * 32)) || (rc = dalloc(h, &h->b1, 320))) return fail(rc);
  if (hipHostMalloc(&h->hflags, 4 * sizeof(int), hipHostMallocMapped) != hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&h->hflags_d), h->hflags, 0) != hipSuccess) {
    set_error("hipHostMalloc (flag words)");
    return fail(EXPECTO_ENOMEM);
  }
  EXPECTO_HIP_CHECK(hipMemcpyAsync(h->w1, params[0], 320 * 32 * sizeof(float), hipMemcpyDeviceToDevice, st));
  EXPECTO_HIP_CHECK(hipMemcpyAsync(h->b1, params[1], 320 * sizeof(float), hipMemcpyDeviceToDevice, st));
  for (int l = 0; l < 5; ++l) {
    const ConvGeo& g = kConv[l];
    const int np = npad_of(g.cout);
    const long long K = 8LL * g.cin;
    if ((rc = dalloc(h, &h->wt[l], (size_t)np * K)) || (rc = dalloc(h, &h->bt[l], np))) return fail(rc);
    const long long tot = np * K;
    repack_conv<<<dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st>>>(params[2 + 2 * l], g.cout, g.cin, np,
                                                                          h->wt[l]);
    pad_copy<<<dim3((np + 255) / 256), dim3(256), 0, st>>>(params[3 + 2 * l], g.cout, np, h->bt[l]);
    if ((rc = make_planes(h, h->wt[l], np, K, &h->wp[l], st))) return fail(rc);
  }
  const int np1 = npad_of(kFc1Out), np2 = npad_of(kNFeat);
  if ((rc = dalloc(h, &h->fc1w, (size_t)np1 * kFc1In)) || (rc = dalloc(h, &h->fc1b, np1)) ||
      (rc = dalloc(h, &h->fc2w, (size_t)np2 * kHidLd)) || (rc = dalloc(h, &h->fc2b, np2)))
    return fail(rc);
  {
    const long long tot = (long long)np1 * kFc1In;
    repack_fc1<<<dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st>>>(params[12], np1, h->fc1w);
    pad_copy<<<dim3((np1 + 255) / 256), dim3(256), 0, st>>>(params[13], kFc1Out, np1, h->fc1b);
    const long long tot2 = (long long)np2 * kHidLd;
    repack_fc2<<<dim3((unsigned)((tot2 + 255) / 256)), dim3(256), 0, st>>>(params[14], np2, h->fc2w);
    pad_copy<<<dim3((np2 + 255) / 256), dim3(256), 0, st>>>(params[15], kNFeat, np2, h->fc2b);
    if ((rc = make_planes(h, h->fc1w, np1, kFc1In, &h->fc1p, st)) ||
        (rc = make_planes(h, h->fc2w, np2, kHidLd, &h->fc2p, st)))
      return fail(rc);
  }
  if ((rc = check_launch("repack"))) return fail(rc);
  const size_t pf = p_floats(max_batch), qf = q_floats(max_batch);
  if (const char* e = getenv("EXPECTO_FC1_SPLITS")) {   // tuning knob (fixed per handle: sums never
    const int v = atoi(e);                               // depend on the batch)
    EXPECTO_REQUIRE(v >= 1 && v <= 32 && (kFc1In / GBK) % v == 0, "EXPECTO_FC1_SPLITS must divide 2120 and be <= 32");
    h->fc_splits = v;
  }
  if (const char* e = getenv("EXPECTO_FC2_SPLITS")) {   // tuning knob (fixed per handle, like FC1's)
    const int v = atoi(e);
    EXPECTO_REQUIRE(v >= 1 && 63 % v == 0, "EXPECTO_FC2_SPLITS must divide 63");
    h->fc2_splits = v;
  }
  if (const char* e = getenv("EXPECTO_FC1_M_ORDER_MB")) h->fc1_m_order_mb = atof(e);   // same bits either way
  if (const char* e = getenv("EXPECTO_FC1_ORDER")) h->fc1_order = atoi(e);              // same bits either way
  if (const char* e = getenv("EXPECTO_FC1_M_GROUP")) h->fc1_m_group = std::max(1, atoi(e));   // same bits
  if (const char* e = getenv("EXPECTO_FC_WIDE")) h->fc_wide = atoi(e) != 0;                   // same bits
  if (const char* e = getenv("EXPECTO_OVERLAP")) h->overlap = atoi(e) != 0;   // same bits either way
  if (const char* e = getenv("EXPECTO_POOL_ONE_PASS")) h->pool_one_pass = atoi(e) != 0;   // same bits either way
  if (const char* e = getenv("EXPECTO_POOL_FUSED")) h->pool_fused = atoi(e) != 0;         // same bits either way
  if (const char* e = getenv("EXPECTO_FUSE_CONV1")) h->fuse_conv1 = atoi(e) != 0;         // same bits either way
  if (const char* e = getenv("EXPECTO_CONV2_TABLE")) h->kmer_on = atoi(e) != 0;   // conv2 on the MFMAs (parity, not bits)
  if (const char* e = getenv("EXPECTO_KMER_QUAD")) h->kmer_quad = atoi(e) != 0;    // pair tables only (parity, not bits)
  if (const char* e = getenv("EXPECTO_ONEHOT_CODES")) h->onehot_as_codes = atoi(e) != 0;   // parity, not bits
  if (const char* e = getenv("EXPECTO_FC1_KARATSUBA")) h->fk_on = atoi(e) != 0;       // parity, not bits
  if (const char* e = getenv("EXPECTO_FC1K_SLICE")) h->fk_slice = std::max(1, atoi(e));  // same bits either way
  if (const char* e = getenv("EXPECTO_FC1_ROLE")) {    // per-window forwards' Karatsuba role (tests)
    const int v = atoi(e);
    EXPECTO_REQUIRE(v >= 0 && v <= 4, "EXPECTO_FC1_ROLE must be 0..4");
    h->fk_role = v;
  }
  if (const char* e = getenv("EXPECTO_SEG_CHUNK_WINDOWS")) h->seg_chunk_windows = atoi(e);   // same bits either way
  if (const char* e = getenv("EXPECTO_CONV_NARROW")) {   // conv5 / conv6 tile width (same bits either way)
    const int v = atoi(e);
    EXPECTO_REQUIRE(v >= -1 && v <= 1, "EXPECTO_CONV_NARROW must be -1 (auto), 0 or 1");
    h->conv_narrow = v;
  }
  if (const char* e = getenv("EXPECTO_FC1_NARROW")) {   // grouped FC1 tile width (same bits either way)
    const int v = atoi(e);
    EXPECTO_REQUIRE(v >= -1 && v <= 1, "EXPECTO_FC1_NARROW must be -1 (auto), 0 or 1");
    h->fc1_narrow = v;
  }
  if (const char* e = getenv("EXPECTO_CONV_EA")) h->conv_ea = atoi(e) != 0;   // same bits either way
  if (const char* e = getenv("EXPECTO_FC_SKINNY")) h->fc_skinny = atoi(e) != 0;   // same bits either way
  if (const char* e = getenv("EXPECTO_CONV_TILE")) {    // tuning knob: f16x3 conv M tile (same bits)
    const int v = atoi(e);
    EXPECTO_REQUIRE(v == 0 || v == 256 || v == 384, "EXPECTO_CONV_TILE must be 0 (auto), 256 or 384");
    h->conv_tile = v;
  }
  // segment path with FC2 unsplit: the FC1 slices' h1 rows of a chunk are gathered into one FC2
  // launch of up to fc2_rows rows (a 2,016-deep GEMM fills whole rounds of the chip only at
  // ~20 k rows; EXPECTO_FC2_ROWS, same bits for any value)
  h->fc2_rows = h->fc2_splits == 1 ? 4 * max_batch : max_batch;
  if (const char* e = getenv("EXPECTO_FC2_ROWS"))
    if (h->fc2_splits == 1) h->fc2_rows = std::max(max_batch, atoi(e));
  // split-K partial rows: FC1's slabs, or the Karatsuba FC1's <= kFkParts partial rows per window
  const size_t partf = (size_t)std::max(h->fc_splits, kFkParts) * max_batch * kHidLd;
  const size_t h1_rows = (size_t)h->fc2_rows + (h->fc2_splits == 1 ? max_batch : 0);
  if ((rc = dalloc(h, &h->P, act_alloc(pf))) || (rc = dalloc(h, &h->Q, act_alloc(qf))) ||
      (rc = dalloc(h, &h->part, partf)) || (rc = dalloc(h, &h->h1, act_alloc(h1_rows * kHidLd))) ||
      (rc = dalloc(h, &h->part2, (size_t)h->fc2_splits * max_batch * kHidLd)))
    return fail(rc);
  {
    float* rows = nullptr;
    if ((rc = dalloc(h, &rows, (size_t)(max_batch + h1_rows) * 2))) return fail(rc);
    h->a_rows = reinterpret_cast<long long*>(rows);
    h->c_rows = h->a_rows + max_batch;
  }
  EXPECTO_HIP_CHECK(hipMemsetAsync(h->P, 0, act_alloc(pf) * sizeof(float), st));
  EXPECTO_HIP_CHECK(hipMemsetAsync(h->Q, 0, act_alloc(qf) * sizeof(float), st));
  // default arithmetic: f16x3 (fp16 weight planes + activation-scale calibration now)
  if ((rc = f16_prepare(h, st))) return fail(rc);
  if (h->kmer_on && (rc = kmer_acquire(h, params, st))) return fail(rc);
  h->precision = EXPECTO_PRECISION_F16X3;
  EXPECTO_HIP_CHECK(hipStreamSynchronize(st));
  *out = h;
  return EXPECTO_OK;
}

void expecto_beluga_destroy(expecto_beluga_t h) {
  if (!h) return;
  kmer_release(h);
  if (h->win_seg_d) (void)hipFree(h->win_seg_d);
  if (h->alt_w_d) (void)hipFree(h->alt_w_d);
  if (h->copy_w_d) (void)hipFree(h->copy_w_d);
  if (h->fc_perm_d) (void)hipFree(h->fc_perm_d);
  if (h->seg_var_d) (void)hipFree(h->seg_var_d);
  if (h->win_off_d) (void)hipFree(h->win_off_d);
  if (h->win_row_d) (void)hipFree(h->win_row_d);
  for (float* p : h->fk_seq)
    if (p) (void)hipFree(p);
  for (float* p : h->fk_aseq)
    if (p) (void)hipFree(p);
  if (h->fk_gres) (void)hipFree(h->fk_gres);
  if (h->seam) (void)hipFree(h->seam);
  if (h->edge) (void)hipFree(h->edge);
  for (void* p : h->allocs) (void)hipFree(p);
  for (hipEvent_t e : h->ev_pool) (void)hipEventDestroy(e);
  for (hipEvent_t e : h->pev)
    if (e) (void)hipEventDestroy(e);
  if (h->st2) (void)hipStreamDestroy(h->st2);
  for (int s = 0; s < 2; ++s) {
    if (h->stage_ev[s]) (void)hipEventSynchronize(h->stage_ev[s]);
    if (h->stage_buf[s]) (void)hipHostFree(h->stage_buf[s]);
    if (h->stage_ev[s]) (void)hipEventDestroy(h->stage_ev[s]);
  }
  if (h->hflags) (void)hipHostFree(h->hflags);
  delete h;
}

size_t expecto_beluga_device_bytes(expecto_beluga_t h) {
  return h ? h->bytes + kmer_reported_bytes(h) : 0;
}

int expecto_beluga_conv2_table_active(expecto_beluga_t h, int* reason) {
  EXPECTO_REQUIRE(h != nullptr, "null handle");
  if (reason) *reason = h->kmer_state;
  return h->kmer ? 1 : 0;
}

int expecto_beluga_set_fc1_role(expecto_beluga_t h, int role) {
  EXPECTO_REQUIRE(h != nullptr, "null handle");
  EXPECTO_REQUIRE(role >= 0 && role <= 4, "FC1 role must be 0..4");
  h->fk_role = role;
  return EXPECTO_OK;
}

int expecto_beluga_forward_onehot(expecto_beluga_t h, const float* x, int n, float* y, void* stream) {
  EXPECTO_REQUIRE(h != nullptr, "null handle");
  EXPECTO_REQUIRE(n >= 0, "negative batch");
  if (n == 0) return EXPECTO_OK;
  EXPECTO_REQUIRE(x != nullptr && y != nullptr, "null input/output");
  EXPECTO_HIP_CHECK(hipSetDevice(h->device));
  hipStream_t st = as_stream(stream);
  // The reference's own call (Beluga.forward on encodeSeqs' one-hot floats, chromatin.py:266-279):
  // when every column of x is an exact one-hot or all-zero column, the call runs as
  // forward_codes(FWD) on codes converted chunk by chunk -- conv1 + conv2 + pool1 from the k-mer
  // tables, the same bits as forward_codes -- else conv1 / conv2 stay on the MFMAs (any fp32
  // input, like the reference).  With the per-call overflow check the codes path runs at once and
  // the conversion's flag is read with the overflow flag at the end (one sync; an input that is not
  // one-hot reruns on the MFMA path, and the handle then checks its next inputs first until one is
  // one-hot again, so a stream of soft inputs costs one check pass each, not a second forward);
  // with the deferred check, one check pass and a sync first (include/expecto_hip.h).  Either way
  // an input's path -- and so its bits -- depends only on the input.
  const bool candidate = h->onehot_as_codes && h->kmer && (reinterpret_cast<uintptr_t>(x) & 15) == 0 &&
                         (h->precision == EXPECTO_PRECISION_F16X3 || h->precision == EXPECTO_PRECISION_BF16X6);
  if (candidate && !h->oh_codes) {
    float *c = nullptr, *f = nullptr;
    int rc;
    if ((rc = dalloc(h, &c, ((size_t)h->max_batch * kLen + 3) / 4)) || (rc = dalloc(h, &f, 1))) return rc;
    h->oh_codes = reinterpret_cast<uint8_t*>(c);
    h->oh_bad = reinterpret_cast<int*>(f);
  }
  // all chunks, conv1 input from codes converted per chunk (bad: also flag non-one-hot columns) or x
  auto run = [&](bool as_codes, int* bad) {
    for (long long r0 = 0; r0 < n; r0 += h->max_batch) {
      const int nb = (int)std::min<long long>(h->max_batch, n - r0);
      int rc;
      if (as_codes) {
        {
          LayerTimer lt(h, 0, st);
          const long long q = (long long)nb * (kLen / 4);
          onehot_codes<<<dim3((unsigned)((q + 255) / 256)), dim3(256), 0, st>>>(x + r0 * 4 * kLen, nb, kLen,
                                                                              h->oh_codes, bad);
          if ((rc = check_launch("onehot_codes"))) return rc;
        }
        rc = forward_chunk(h, nullptr, h->oh_codes, kLen, nb, EXPECTO_STRAND_FWD, 0, nb, y + r0 * kNFeat, st);
      } else {
        rc = forward_chunk(h, x, nullptr, 0, 0, 0, r0, nb, y + r0 * kNFeat, st);
      }
      if (rc) return rc;
    }
    return (int)EXPECTO_OK;
  };
  if (candidate && h->precision == EXPECTO_PRECISION_F16X3 && !h->ovf_deferred && !h->oh_hint_bad) {
    // (oh_bad is 0 here: zeroed at allocation, and every path that sets it resets it in take_flags)
    int rc = run(true, h->oh_bad);
    if (rc) return rc;
    int* flags = h->hflags;   // pinned, device-mapped host words: ovf, oh_bad (then reset on the device)
    take_flags<<<1, 64, 0, st>>>(h->ovf, h->oh_bad, h->hflags_d);
    EXPECTO_HIP_CHECK(hipGetLastError());
    EXPECTO_HIP_CHECK(hipStreamSynchronize(st));
    if (flags[1]) {   // not one-hot: the whole call on the MFMA path (its own overflow check)
      h->oh_hint_bad = true;
      EXPECTO_HIP_CHECK(hipMemsetAsync(h->ovf, 0, sizeof(int), st));
      return run_checked(h, st, [&]() { return run(false, nullptr); });
    }
    if (!flags[0]) return EXPECTO_OK;
    EXPECTO_HIP_CHECK(hipMemsetAsync(h->ovf, 0, sizeof(int), st));   // as run_checked: bf16x6 redo
    h->fallbacks += 1;
    h->precision = EXPECTO_PRECISION_BF16X6;
    rc = run(true, nullptr);
    h->precision = EXPECTO_PRECISION_F16X3;
    return rc;
  }
  bool as_codes = false;
  if (candidate) {
    int bad = 0;
    {
      LayerTimer lt(h, 0, st);
      EXPECTO_HIP_CHECK(hipMemsetAsync(h->oh_bad, 0, sizeof(int), st));
      const long long q = (long long)n * (kLen / 4);
      onehot_codes<<<dim3((unsigned)((q + 255) / 256)), dim3(256), 0, st>>>(x, n, kLen, nullptr, h->oh_bad);
      int rc = check_launch("onehot_codes check");
      if (rc) return rc;
    }
    take_flags<<<1, 64, 0, st>>>(nullptr, h->oh_bad, h->hflags_d);   // (resets oh_bad)
    EXPECTO_HIP_CHECK(hipGetLastError());
    EXPECTO_HIP_CHECK(hipStreamSynchronize(st));
    bad = h->hflags[1];
    as_codes = bad == 0;
    h->oh_hint_bad = !as_codes;
  }
  return run_checked(h, st, [&]() { return run(as_codes, nullptr); });
}

int expecto_beluga_forward_codes(expecto_beluga_t h, const uint8_t* codes, int n, long long code_stride,
                                 int strand_mode, float* y, void* stream) {
  EXPECTO_REQUIRE(h != nullptr, "null handle");
  EXPECTO_REQUIRE(n >= 0, "negative batch");
  EXPECTO_REQUIRE(strand_mode >= 0 && strand_mode <= 2, "bad strand mode");
  if (n == 0) return EXPECTO_OK;
  EXPECTO_REQUIRE(codes != nullptr && y != nullptr, "null input/output");
  EXPECTO_REQUIRE(code_stride >= kLen, "code_stride < 2000");
  EXPECTO_HIP_CHECK(hipSetDevice(h->device));
  hipStream_t st = as_stream(stream);
  const long long rows = strand_mode == EXPECTO_STRAND_BOTH ? 2LL * n : n;
  return run_checked(h, st, [&]() {
    for (long long r0 = 0; r0 < rows; r0 += h->max_batch) {
      const int nb = (int)std::min<long long>(h->max_batch, rows - r0);
      int rc = forward_chunk(h, nullptr, codes, code_stride, n, strand_mode, r0, nb, y + r0 * kNFeat, st);
      if (rc) return rc;
    }
    return (int)EXPECTO_OK;
  });
}

int expecto_beluga_forward_segments(expecto_beluga_t h, const uint8_t* codes, int n_seg, int seg_len,
                                    long long code_stride, int strand_mode, const int* win_seg, const int* win_off,
                                    const int* win_row, int n_win, float* y, void* stream) {
  EXPECTO_REQUIRE(h != nullptr, "null handle");
  EXPECTO_REQUIRE(n_seg >= 0 && n_win >= 0, "negative count");
  EXPECTO_REQUIRE(strand_mode >= 0 && strand_mode <= 2, "bad strand mode");
  if (n_win == 0 || n_seg == 0) return EXPECTO_OK;
  EXPECTO_REQUIRE(codes && y && win_seg && win_off, "null argument");
  EXPECTO_REQUIRE(code_stride >= seg_len, "code_stride < seg_len");
  EXPECTO_HIP_CHECK(hipSetDevice(h->device));
  hipStream_t st = as_stream(stream);
  return run_checked(h, st, [&]() {
    return forward_segments(h, codes, n_seg, seg_len, code_stride, strand_mode, win_seg, win_off, win_row, n_win, y,
                            st);
  });
}

int expecto_beluga_forward_segment_pairs(expecto_beluga_t h, const uint8_t* codes, const int* var_pos,
                                         const uint8_t* alt_code, int n_seg, int seg_len, long long code_stride,
                                         int strand_mode, const int* win_seg, const int* win_off, const int* win_row,
                                         int n_win, float* y_ref, float* y_alt, long long strand_stride,
                                         void* stream) {
  EXPECTO_REQUIRE(h != nullptr, "null handle");
  EXPECTO_REQUIRE(n_seg >= 0 && n_win >= 0, "negative count");
  EXPECTO_REQUIRE(strand_mode >= 0 && strand_mode <= 2, "bad strand mode");
  if (n_win == 0 || n_seg == 0) return EXPECTO_OK;
  EXPECTO_REQUIRE(codes && var_pos && alt_code && y_ref && y_alt && win_seg && win_off, "null argument");
  EXPECTO_REQUIRE(code_stride >= seg_len, "code_stride < seg_len");
  EXPECTO_REQUIRE(strand_mode != EXPECTO_STRAND_BOTH || strand_stride >= n_win, "strand_stride < n_win");
  EXPECTO_HIP_CHECK(hipSetDevice(h->device));
  const SegPairs pr{var_pos, alt_code, y_alt, strand_stride};
  hipStream_t st = as_stream(stream);
  return run_checked(h, st, [&]() {
    return forward_segments(h, codes, n_seg, seg_len, code_stride, strand_mode, win_seg, win_off, win_row, n_win,
                            y_ref, st, &pr);
  });
}

int expecto_beluga_forward_pairs(expecto_beluga_t h, const uint8_t* ref_codes, const uint8_t* alt_codes, int n,
                                 long long code_stride, const int* var_pos, int strand_mode, float* y_ref,
                                 float* y_alt, long long strand_stride, void* stream) {
  EXPECTO_REQUIRE(h != nullptr, "null handle");
  EXPECTO_REQUIRE(n >= 0, "negative count");
  EXPECTO_REQUIRE(strand_mode == EXPECTO_STRAND_FWD || strand_mode == EXPECTO_STRAND_BOTH, "strand mode FWD or BOTH");
  if (n == 0) return EXPECTO_OK;
  EXPECTO_REQUIRE(ref_codes && alt_codes && var_pos && y_ref && y_alt, "null argument");
  EXPECTO_REQUIRE(code_stride >= kLen, "code_stride < 2000");
  EXPECTO_HIP_CHECK(hipSetDevice(h->device));
  hipStream_t st = as_stream(stream);
  return run_checked(h, st, [&]() {
    return forward_pairs(h, ref_codes, alt_codes, n, code_stride, var_pos, strand_mode, y_ref, y_alt, strand_stride,
                         st);
  });
}

int expecto_beluga_set_precision(expecto_beluga_t h, int precision) {
  EXPECTO_REQUIRE(h != nullptr, "null handle");
  EXPECTO_REQUIRE(precision == EXPECTO_PRECISION_FP32 || precision == EXPECTO_PRECISION_BF16X6 ||
                      precision == EXPECTO_PRECISION_F16X3,
                  "bad precision");
  if (precision == EXPECTO_PRECISION_F16X3) {
    EXPECTO_HIP_CHECK(hipSetDevice(h->device));
    int rc = f16_prepare(h, nullptr);
    if (rc) return rc;
    EXPECTO_HIP_CHECK(hipStreamSynchronize(nullptr));
  }
  h->precision = precision;
  return EXPECTO_OK;
}

int expecto_beluga_set_f16_target(expecto_beluga_t h, int target_log2) {
  EXPECTO_REQUIRE(h != nullptr, "null handle");
  EXPECTO_REQUIRE(target_log2 >= 0 && target_log2 <= 20, "target_log2 out of range");
  EXPECTO_HIP_CHECK(hipSetDevice(h->device));
  h->f16_target = target_log2;
  if (!h->f16_ready) return EXPECTO_OK;   // applied by the first f16_prepare
  const int saved = g_precision;
  int rc = f16_calibrate(h, nullptr);
  g_precision = saved;
  if (rc) return rc;
  EXPECTO_HIP_CHECK(hipStreamSynchronize(nullptr));
  return EXPECTO_OK;
}

long long expecto_beluga_f16_fallbacks(expecto_beluga_t h, int* sx) {
  if (!h) return EXPECTO_EINVAL;
  if (sx)
    for (int b = 0; b < 7; ++b) sx[b] = h->sx[b];
  return h->fallbacks;
}

int expecto_beluga_get_precision(expecto_beluga_t h) { return h ? h->precision : EXPECTO_EINVAL; }

int expecto_beluga_set_profiling(expecto_beluga_t h, int on) {
  EXPECTO_REQUIRE(h != nullptr, "null handle");
  if (on && h->ev_pool.empty()) {
    h->ev_pool.resize(1024);
    for (auto& e : h->ev_pool) EXPECTO_HIP_CHECK(hipEventCreate(&e));
  }
  if (!on) {
    int rc = resolve_events(h);
    if (rc) return rc;
  }
  h->profiling = on != 0;
  if (on) {
    if (h->macs_d) {
      EXPECTO_HIP_CHECK(hipDeviceSynchronize());
      EXPECTO_HIP_CHECK(hipMemset(h->macs_d, 0, 2 * kNumLayers * sizeof(double)));
    }
    std::fill(h->ms, h->ms + 2 * kNumLayers, 0.0);
    std::fill(h->calls, h->calls + 2 * kNumLayers, 0LL);
    std::fill(h->macs, h->macs + 2 * kNumLayers, 0.0);
    h->launch_stats.clear();
  }
  return EXPECTO_OK;
}

int expecto_beluga_main_launches(expecto_beluga_t h, int slot, long long* rows, double* ms, long long* calls,
                                 double* macs) {
  EXPECTO_REQUIRE(h != nullptr && rows && ms && calls && macs, "null argument");
  EXPECTO_REQUIRE(slot >= 0 && slot < 2 * kNumLayers, "slot out of range");
  int rc = resolve_events(h);
  if (rc) return rc;
  *rows = 0, *ms = 0.0, *calls = 0, *macs = 0.0;
  for (auto& kv : h->launch_stats)
    if (kv.first.first == slot && kv.first.second > *rows) {
      *rows = kv.first.second;
      *ms = kv.second[0];
      *calls = (long long)kv.second[1];
      *macs = kv.second[2];
    }
  return EXPECTO_OK;
}

int expecto_beluga_layer_times(expecto_beluga_t h, double* ms, long long* calls, double* macs, int max_layers) {
  EXPECTO_REQUIRE(h != nullptr, "null handle");
  int rc = resolve_events(h);
  if (rc) return rc;
  double dm[2 * kNumLayers] = {};
  if (h->macs_d) {   // device-side counts (alt FC1 slab share); the events above are resolved
    EXPECTO_HIP_CHECK(hipDeviceSynchronize());
    EXPECTO_HIP_CHECK(hipMemcpy(dm, h->macs_d, sizeof(dm), hipMemcpyDeviceToHost));
  }
  const int n = std::min(max_layers, 2 * kNumLayers);
  for (int i = 0; i < n; ++i) {
    if (ms) ms[i] = h->ms[i];
    if (calls) calls[i] = h->calls[i];
    if (macs) macs[i] = h->macs[i] + dm[i];
  }
  return 2 * kNumLayers;
}

int expecto_beluga_set_overflow_check(expecto_beluga_t h, int deferred) {
  EXPECTO_REQUIRE(h != nullptr, "null handle");
  EXPECTO_REQUIRE(deferred == 0 || deferred == 1, "deferred must be 0 or 1");
  h->ovf_deferred = deferred != 0;
  return EXPECTO_OK;
}

int expecto_beluga_overflow_take(expecto_beluga_t h, int* dst, void* stream) {
  EXPECTO_REQUIRE(h != nullptr && dst != nullptr, "null argument");
  EXPECTO_HIP_CHECK(hipSetDevice(h->device));
  hipStream_t st = as_stream(stream);
  EXPECTO_REQUIRE(h->ovf != nullptr, "no overflow flag (f16x3 never prepared)");
  EXPECTO_HIP_CHECK(hipMemcpyAsync(dst, h->ovf, sizeof(int), hipMemcpyDefault, st));
  EXPECTO_HIP_CHECK(hipMemsetAsync(h->ovf, 0, sizeof(int), st));
  return EXPECTO_OK;
}

int expecto_beluga_count_fallback(expecto_beluga_t h) {
  EXPECTO_REQUIRE(h != nullptr, "null handle");
  h->fallbacks += 1;
  return EXPECTO_OK;
}

int expecto_beluga_overflow_pending(expecto_beluga_t h, void* stream) {
  EXPECTO_REQUIRE(h != nullptr, "null handle");
  if (!h->ovf) return 0;
  EXPECTO_HIP_CHECK(hipSetDevice(h->device));
  hipStream_t st = as_stream(stream);
  int flag = 0;
  EXPECTO_HIP_CHECK(hipMemcpyAsync(&flag, h->ovf, sizeof(int), hipMemcpyDeviceToHost, st));
  EXPECTO_HIP_CHECK(hipStreamSynchronize(st));
  if (!flag) return 0;
  EXPECTO_HIP_CHECK(hipMemsetAsync(h->ovf, 0, sizeof(int), st));
  EXPECTO_HIP_CHECK(hipStreamSynchronize(st));
  h->fallbacks += 1;   // the caller recomputes the flagged calls with BF16X6
  return 1;
}

}  // extern "C"
