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
#include <cstring>
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
                                                    float* __restrict__ out, int out_rows, int len, int x3) {
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
    const float v = fmaxf(s + bco, 0.f);
    if (x3)
      store_act<true>(out, orow + t, 320, co, v);
    else
      store_act<false>(out, orow + t, 320, co, v);
  }
}

__global__ void fc1_reduce(const float* __restrict__ part, int splits, long long split_stride, long long count,
                           const float* __restrict__ bias, float* __restrict__ h1, int x3) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const long long row = i / kHidLd;
  const int n = (int)(i - row * kHidLd);
  float s = 0.f;
  for (int k = 0; k < splits; ++k) s += part[k * split_stride + i];
  const float v = n < kFc1Out ? fmaxf(s + bias[n], 0.f) : 0.f;
  if (x3)
    store_act<true>(h1, row, kHidLd, n, v);
  else
    h1[i] = v;
}

// MaxPool(1,4) floor mode at pool phases p (segment path, SURVEY.md 5 "trunk sharing"):
// out[(seg*n_ph + i)*s_out + g][c] = max_{j<4} in[seg*s_in + ph[i] + 4g + j][c],
// g < (t_in - ph[i]) / 4.  ReLU was applied by the producing conv (Beluga.py:32-34 order).
// One thread per channel; on the bf16x6 path the values are recovered exactly from their
// planes, pooled, and re-split (so the planes equal those of the pooled fp32 value).
__global__ void pool4_phases(const float* __restrict__ in, int n_seg, int s_in, int t_in, int C,
                             int n_ph, int4 ph, int s_out, float* __restrict__ out, int x3) {
  const int c = threadIdx.x;
  const int g = blockIdx.x;
  const int i = blockIdx.y % n_ph;
  const long long seg = blockIdx.y / n_ph;
  const int p = i == 0 ? ph.x : i == 1 ? ph.y : i == 2 ? ph.z : ph.w;
  if (c >= C || g >= (t_in - p) / 4) return;
  const long long r0 = seg * s_in + p + 4LL * g, orow = (seg * n_ph + i) * s_out + g;
  float m = x3 ? load_x3(in, r0, C, c) : in[r0 * C + c];
#pragma unroll
  for (int j = 1; j < 4; ++j) m = fmaxf(m, x3 ? load_x3(in, r0 + j, C, c) : in[(r0 + j) * C + c]);
  if (x3)
    store_act<true>(out, orow, C, c, m);
  else
    out[orow * C + c] = m;
}

// FC1 row table of the windows of one segment chunk: window m of the chunk reads conv6
// rows [off6, off6+106) of block (segment, pool2 phase).
__global__ void seg_a_rows(const int* __restrict__ win_seg, const int* __restrict__ win_off,
                           const int* __restrict__ win_row, int w0, int m_count, int seg_base, int rc, int seg_len,
                           int n_ph, int4 ph_idx, int s7, long long row_base, long long* __restrict__ a_rows,
                           long long* __restrict__ c_rows) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= m_count) return;
  const int w = w0 + m;
  c_rows[m] = row_base + (win_row ? win_row[w] : w);
  const int o = rc ? seg_len - 2000 - win_off[w] : win_off[w];
  const int q = o >> 2, p = q & 3, off6 = (q - p) >> 2;
  const int pi = p == 0 ? ph_idx.x : p == 1 ? ph_idx.y : p == 2 ? ph_idx.z : ph_idx.w;
  const long long blk = (long long)(win_seg[w] - seg_base) * n_ph + pi;
  a_rows[m] = (blk * s7 + off6) * 640;
}

// ---- alt-cone reuse for SNV ref/alt window pairs ---------------------------------------
// A conv6 row t of a window depends on input positions [16t, 16t+309] (receptive field 310).
// An SNV at window index p therefore changes only rows t in [ceil((p-309)/16), floor(p/16)]
// (at most 20 of 106).  The alt window is computed as: the ref window's conv6 rows, with the
// 20 rows starting at r0 replaced by the conv6 rows of a 616-bp "patch" sequence cut from the
// alt window at 16*r0 (16-aligned, so pool1/pool2 groups coincide with the window's).  Every
// row is produced by the same kernels from the same operands -> bit-identical alt outputs.
constexpr int kPatchLen = 616;   // 16*19 + 310 rounded up to 4 -> 20 conv6 rows
constexpr int kPatchRows = 20;
constexpr int kPatchMaxRow0 = 106 - kPatchRows;

__device__ __forceinline__ int patch_row0(int p) {
  const int t_lo = p >= 309 ? (p - 309 + 15) / 16 : 0;
  return t_lo < kPatchMaxRow0 ? t_lo : kPatchMaxRow0;
}

// m = strand*nv + (v - v0); strand 1 = reverse complement of the alt window.
__global__ void pair_patch_codes(const uint8_t* __restrict__ alt, long long stride, int nv, int v0,
                                 const int* __restrict__ var_pos, uint8_t* __restrict__ out) {
  const int m = blockIdx.y;
  const int s = m / nv, v = v0 + m % nv;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= kPatchLen) return;
  const int pv = min(max(var_pos[v], 0), kLen - 1);
  const int p = s ? kLen - 1 - pv : pv;
  const int start = 16 * patch_row0(p);
  const uint8_t* a = alt + (long long)v * stride;
  uint8_t c;
  if (s) {
    const uint8_t f = a[kLen - 1 - (start + i)];
    c = f < 4 ? (uint8_t)(3 - f) : f;
  } else {
    c = a[start + i];
  }
  out[(long long)m * kPatchLen + i] = c;
}

// act6[m][r0 + r][:] = patch6[m][r][:] for r < 20: one conv6 row = row16 16-byte lanes
// (640 fp32 = 160, or 640 channels of bf16 planes = 240)
__global__ void pair_patch_apply(const float* __restrict__ patch6, float* __restrict__ act6, int nv, int v0,
                                 const int* __restrict__ var_pos, int row16) {
  const int m = blockIdx.y;
  const int r = blockIdx.x;
  const int c4 = threadIdx.x;
  if (c4 >= row16) return;
  const int s = m / nv, v = v0 + m % nv;
  const int pv = min(max(var_pos[v], 0), kLen - 1);
  const int p = s ? kLen - 1 - pv : pv;
  const int r0 = patch_row0(p);
  const floatx4* src = reinterpret_cast<const floatx4*>(patch6) + ((long long)m * kPatchRows + r) * row16;
  floatx4* dst = reinterpret_cast<floatx4*>(act6) + ((long long)m * 106 + r0 + r) * row16;
  dst[c4] = src[c4];
}

__global__ void pair_rows(long long* __restrict__ c_rows, int M, int nv, int v0, long long strand_stride) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m < M) c_rows[m] = (long long)(m / nv) * strand_stride + v0 + m % nv;
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

}  // namespace expecto

using namespace expecto;

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
constexpr int kFcSplits[] = {1, 2, 4, 5, 8, 10};  // divisors of 67840/32 = 2120
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
  float* P = nullptr;
  float* Q = nullptr;
  float* part = nullptr;
  float* h1 = nullptr;
  long long* a_rows = nullptr;  // FC1 row table (segment path), max_batch entries
  long long* c_rows = nullptr;  // FC2 output-row table (segment path), max_batch entries
  int* win_seg_d = nullptr;     // window tables of the current segment call
  int* win_off_d = nullptr;
  int* win_row_d = nullptr;
  float* P2 = nullptr;           // patch trunk buffers (alt-cone path), lazily allocated
  float* Q2 = nullptr;
  uint8_t* patch_codes = nullptr;
  int win_cap = 0;
  size_t bytes = 0;
  std::vector<void*> allocs;
  int precision = EXPECTO_PRECISION_BF16X6;
  bool profiling = false;
  std::vector<hipEvent_t> ev_pool;
  std::vector<std::pair<int, int>> pending;  // (layer, event index of start)
  size_t ev_next = 0;
  double ms[kNumLayers] = {};
  long long calls[kNumLayers] = {};
  double macs[kNumLayers] = {};  // executed multiply-adds per layer while profiling (host-side count)
};

namespace {
int dalloc(expecto_beluga* h, float** p, size_t nfloat) {
  void* ptr = nullptr;
  hipError_t e = hipMalloc(&ptr, nfloat * sizeof(float));
  if (e != hipSuccess) {
    set_error(std::string("hipMalloc: ") + hipGetErrorString(e));
    return EXPECTO_ENOMEM;
  }
  h->allocs.push_back(ptr);
  h->bytes += nfloat * sizeof(float);
  *p = static_cast<float*>(ptr);
  return EXPECTO_OK;
}

int npad_of(int n) { return (n + GBN - 1) / GBN * GBN; }

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
  h->ev_next = 0;
  return EXPECTO_OK;
}

struct LayerTimer {
  expecto_beluga* h;
  int layer;
  int idx = -1;
  hipStream_t st;
  LayerTimer(expecto_beluga* hh, int l, hipStream_t s) : h(hh), layer(l), st(s) {
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

// Arithmetic of the MFMA GEMMs: exact fp32 (v_mfma_f32_32x32x2_f32) or the fp32-faithful
// 3-way bf16 split (six v_mfma_f32_32x32x16_bf16 products per k-step, gemm_kernel.h).
thread_local int g_precision = EXPECTO_PRECISION_BF16X6;

// activations stored as bf16 planes (bf16x6 path) or fp32 rows
int x3_act() { return g_precision == EXPECTO_PRECISION_BF16X6 ? 1 : 0; }
long long gemm_bm() { return g_precision == EXPECTO_PRECISION_BF16X6 ? X6P_BM : GBM; }

template <int LAYER, int EPI>
int launch_gemm(const GemmArgs& a, int splits, hipStream_t st) {
  const long long nblk = a.m_tiles * a.n_tiles * splits;
  EXPECTO_REQUIRE(nblk > 0 && nblk < (1LL << 31), "gemm grid out of range");
  EXPECTO_REQUIRE(a.kper % GBK == 0 && a.kper > 0, "gemm K not a multiple of 32");
  EXPECTO_REQUIRE(a.lda % 4 == 0 && a.ldb % 4 == 0, "gemm leading dims must be multiples of 4");
  EXPECTO_REQUIRE(a.taps == 1 || (a.taps == 8 && a.lda % GBK == 0), "conv GEMM needs Cin % 32 == 0");
  EXPECTO_REQUIRE(a.m_tiles * gemm_bm() >= a.M, "gemm M tiles do not cover M");
  if (g_precision == EXPECTO_PRECISION_BF16X6) {
    EXPECTO_REQUIRE(a.Bp != nullptr && a.lda % GBK == 0 && a.ldb % GBK == 0, "bf16x6 GEMM needs planes, K % 32");
    beluga_gemm_x6p<LAYER, EPI><<<dim3((unsigned)nblk), dim3(256), 0, st>>>(a);
  } else
    beluga_gemm<LAYER, EPI, kWM, kMinBlocks, GBK, kPipe><<<dim3((unsigned)nblk), dim3(64 * kWM), 0, st>>>(a);
  return check_launch("beluga_gemm");
}

int run_conv1(expecto_beluga* h, const float* x, const uint8_t* codes, long long code_stride, int n_src, int mode,
              long long row0, int nb, int len, int out_rows, hipStream_t st, float* dst = nullptr) {
  LayerTimer lt(h, 0, st);
  if (h->profiling) h->macs[0] += (double)nb * (len - 7) * 320 * 32;
  dim3 grid((len - 7 + C1_T - 1) / C1_T, nb);
  beluga_conv1<<<grid, dim3(320), 0, st>>>(x, codes, code_stride, n_src, mode, row0, h->w1, h->b1,
                                           dst ? dst : h->P, out_rows, len, x3_act());
  return check_launch("beluga_conv1");
}

// conv layer l (0 = conv2 .. 4 = conv6) over `groups` row groups of s_in rows each.
int run_conv(expecto_beluga* h, int l, const float* src, float* dst, long long groups, int s_in, int t_valid,
             int s_out, bool pool, hipStream_t st) {
  const ConvGeo& g = kConv[l];
  GemmArgs a{};
  a.A = src;
  a.lda = g.cin;
  a.M = groups * s_in;
  a.B = h->wt[l];
  a.Bp = h->wp[l];
  a.ldb = 8LL * g.cin;
  a.kper = 8 * g.cin;
  a.taps = 8;
  a.n_tiles = npad_of(g.cout) / GBN;
  a.m_tiles = (a.M + gemm_bm() - 1) / gemm_bm();
  a.m_fastest = 0;
  a.bias = h->bt[l];
  a.C = dst;
  a.ldc = g.cout;
  a.n_store = g.cout;
  a.s_in = s_in;
  a.t_valid = t_valid;
  a.s_out = s_out;
  LayerTimer lt(h, l + 1, st);
  if (h->profiling) h->macs[l + 1] += (double)a.M * g.cout * a.kper;
  if (pool) {
    EXPECTO_REQUIRE(s_in % 4 == 0, "pool epilogue needs 4-aligned row groups");
    return l == 0 ? launch_gemm<2, EPI_RELU_POOL4>(a, 1, st) : launch_gemm<4, EPI_RELU_POOL4>(a, 1, st);
  }
  switch (l) {
    case 1: return launch_gemm<3, EPI_RELU>(a, 1, st);
    case 2: return launch_gemm<4, EPI_RELU>(a, 1, st);
    case 3: return launch_gemm<5, EPI_RELU>(a, 1, st);
    default: return launch_gemm<6, EPI_RELU>(a, 1, st);
  }
}

// FC1 (split-K) + reduce + FC2/sigmoid for nb windows whose conv6 rows are at act
// (+ a_rows[m] when given, else m*67840).
int run_fc(expecto_beluga* h, const float* act, const long long* a_rows, int nb, float* y, hipStream_t st,
           const long long* c_rows = nullptr) {
  int rc;
  const long long m_tiles = (nb + gemm_bm() - 1) / gemm_bm();
  const int n_tiles1 = npad_of(kFc1Out) / GBN;
  int splits = kFcSplits[0];
  for (int s : kFcSplits) {
    splits = s;
    if (m_tiles * n_tiles1 * s >= 1000) break;
  }
  {
    GemmArgs a{};
    a.A = act;
    a.a_rows = a_rows;
    a.lda = (long long)kFc1In;
    a.M = nb;
    a.B = h->fc1w;
    a.Bp = h->fc1p;
    a.ldb = kFc1In;
    a.kper = kFc1In / splits;
    a.taps = 1;
    a.n_tiles = n_tiles1;
    a.m_tiles = m_tiles;
    a.m_fastest = 1;
    a.C = h->part;
    a.ldc = kHidLd;
    a.n_store = kHidLd;
    a.split_stride = (long long)nb * kHidLd;
    LayerTimer lt(h, 6, st);
    if (h->profiling) h->macs[6] += (double)nb * kFc1Out * kFc1In;
    if ((rc = launch_gemm<7, EPI_PARTIAL>(a, splits, st))) return rc;
  }
  {
    LayerTimer lt(h, 7, st);
    const long long count = (long long)nb * kHidLd;
    fc1_reduce<<<dim3((unsigned)((count + 255) / 256)), dim3(256), 0, st>>>(h->part, splits, count, count, h->fc1b,
                                                                            h->h1, x3_act());
    if ((rc = check_launch("fc1_reduce"))) return rc;
  }
  {
    GemmArgs a{};
    a.A = h->h1;
    a.lda = kHidLd;
    a.M = nb;
    a.B = h->fc2w;
    a.Bp = h->fc2p;
    a.ldb = kHidLd;
    a.kper = kHidLd;
    a.taps = 1;
    a.n_tiles = npad_of(kNFeat) / GBN;
    a.m_tiles = m_tiles;
    a.m_fastest = 1;
    a.bias = h->fc2b;
    a.c_rows = c_rows;
    a.C = y;
    a.ldc = kNFeat;
    a.n_store = kNFeat;
    a.s_in = 1;
    a.t_valid = 1;
    a.s_out = 1;
    LayerTimer lt(h, 8, st);
    if (h->profiling) h->macs[8] += (double)nb * kNFeat * kFc1Out;
    if ((rc = launch_gemm<8, EPI_SIGMOID>(a, 1, st))) return rc;
  }
  return EXPECTO_OK;
}

// One chunk of nb independent windows; conv1 input from x (one-hot) or codes.
int forward_chunk(expecto_beluga* h, const float* x, const uint8_t* codes, long long code_stride, int n_src,
                  int mode, long long row0, int nb, float* y, hipStream_t st) {
  int rc;
  g_precision = h->precision;
  if ((rc = run_conv1(h, x, codes, code_stride, n_src, mode, row0, nb, kLen, kS1, st))) return rc;
  float* src = h->P;
  float* dst = h->Q;
  for (int l = 0; l < 5; ++l) {
    const ConvGeo& g = kConv[l];
    if ((rc = run_conv(h, l, src, dst, nb, g.s_in, g.t_valid, g.s_out, g.pool != 0, st))) return rc;
    std::swap(src, dst);
  }
  return run_fc(h, src, nullptr, nb, y, st);  // src = act5 (buffer Q), 106 x 640 rows per window
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
  const size_t p_conv1 = (size_t)g.S1 * 320, p_conv3 = (size_t)g.T3 * 480, p_pool2 = (size_t)n_ph * g.S5 * 480,
               p_conv6 = (size_t)n_ph * g.T6 * 640;
  const size_t q_pool1 = (size_t)g.P1 * 320, q_conv4 = (size_t)g.T4 * 480, q_conv5 = (size_t)n_ph * g.T5 * 640;
  g.p_rows_floats = std::max(std::max(p_conv1, p_conv3), std::max(p_pool2, p_conv6));
  g.q_rows_floats = std::max(q_pool1, std::max(q_conv4, q_conv5));
  return g;
}

int forward_segments(expecto_beluga* h, const uint8_t* codes, int n_seg, int L, long long code_stride, int mode,
                     const int* win_seg, const int* win_off, const int* win_row, int n_win, float* y,
                     hipStream_t st) {
  EXPECTO_REQUIRE(L >= kLen && L % 4 == 0, "segment length must be >= 2000 and a multiple of 4");
  g_precision = h->precision;
  // phases present (fwd and, for BOTH, the mirrored rc offsets)
  int present[4] = {0, 0, 0, 0};
  for (int w = 0; w < n_win; ++w) {
    EXPECTO_REQUIRE(win_seg[w] >= 0 && win_seg[w] < n_seg, "window segment out of range");
    EXPECTO_REQUIRE(w == 0 || win_seg[w] >= win_seg[w - 1], "windows must be sorted by segment");
    const int o = win_off[w];
    EXPECTO_REQUIRE(o >= 0 && o % 4 == 0 && o + kLen <= L, "window offset must be 4-aligned inside the segment");
    present[(o >> 2) & 3] = 1;
    if (mode == EXPECTO_STRAND_BOTH) present[((L - kLen - o) >> 2) & 3] = 1;
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
    if (h->win_seg_d) EXPECTO_HIP_CHECK(hipFree(h->win_seg_d));
    if (h->win_off_d) EXPECTO_HIP_CHECK(hipFree(h->win_off_d));
    if (h->win_row_d) EXPECTO_HIP_CHECK(hipFree(h->win_row_d));
    h->win_seg_d = h->win_off_d = h->win_row_d = nullptr;
    h->win_cap = 0;
    EXPECTO_HIP_CHECK(hipMalloc(&h->win_seg_d, n_win * sizeof(int)));
    EXPECTO_HIP_CHECK(hipMalloc(&h->win_off_d, n_win * sizeof(int)));
    EXPECTO_HIP_CHECK(hipMalloc(&h->win_row_d, n_win * sizeof(int)));
    h->win_cap = n_win;
  }
  if (win_row) {
    for (int w = 0; w < n_win; ++w) EXPECTO_REQUIRE(win_row[w] >= 0 && win_row[w] < n_win, "window row out of range");
    EXPECTO_HIP_CHECK(hipMemcpyAsync(h->win_row_d, win_row, n_win * sizeof(int), hipMemcpyHostToDevice, st));
  }
  EXPECTO_HIP_CHECK(hipMemcpyAsync(h->win_seg_d, win_seg, n_win * sizeof(int), hipMemcpyHostToDevice, st));
  EXPECTO_HIP_CHECK(hipMemcpyAsync(h->win_off_d, win_off, n_win * sizeof(int), hipMemcpyHostToDevice, st));
  // the tables are caller-owned pageable host memory: finish the copies before returning
  EXPECTO_HIP_CHECK(hipStreamSynchronize(st));
  const int strands = mode == EXPECTO_STRAND_BOTH ? 2 : 1;
  int rc;
  for (int sd = 0; sd < strands; ++sd) {
    const bool is_rc = (mode == EXPECTO_STRAND_RC) || sd == 1;
    for (int s0 = 0; s0 < n_seg;) {
      // grow the chunk while the segment buffers and the FC workspace (<= max_batch windows) fit
      int s1 = s0 + 1;
      while (s1 < n_seg && s1 - s0 < seg_cap && first[s1 + 1] - first[s0] <= h->max_batch) ++s1;
      const int w0 = first[s0], nw = first[s1] - first[s0];
      EXPECTO_REQUIRE(nw <= h->max_batch, "more windows in one segment than max_batch");
      const int ns = s1 - s0;
      // conv1 from codes: virtual rows = segments; rc mode mirrors inside the kernel
      if ((rc = run_conv1(h, nullptr, codes + (long long)s0 * code_stride, code_stride, ns,
                          is_rc ? EXPECTO_STRAND_RC : EXPECTO_STRAND_FWD, 0, ns, L, g.S1, st)))
        return rc;
      // conv2 + pool1 (P -> Q), conv3 (Q -> P), conv4 unpooled (P -> Q)
      if ((rc = run_conv(h, 0, h->P, h->Q, ns, g.S1, g.P1, g.P1, true, st))) return rc;
      if ((rc = run_conv(h, 1, h->Q, h->P, ns, g.P1, g.T3, g.T3, false, st))) return rc;
      if ((rc = run_conv(h, 2, h->P, h->Q, ns, g.T3, g.T4, g.T4, false, st))) return rc;
      {  // pool2 phases (Q -> P)
        LayerTimer lt(h, 3, st);
        dim3 grid(g.S5, ns * n_ph);
        pool4_phases<<<grid, dim3(480), 0, st>>>(h->Q, ns, g.T4, g.T4, 480, n_ph,
                                               make_int4(ph[0], ph[1], ph[2], ph[3]), g.S5, h->P, x3_act());
        if ((rc = check_launch("pool4_phases"))) return rc;
      }
      // conv5 (P -> Q), conv6 (Q -> P) over (segment, phase) blocks
      if ((rc = run_conv(h, 3, h->P, h->Q, (long long)ns * n_ph, g.S5, g.T5, g.T5, false, st))) return rc;
      if ((rc = run_conv(h, 4, h->Q, h->P, (long long)ns * n_ph, g.T5, g.T6, g.T6, false, st))) return rc;
      if (nw > 0) {
        seg_a_rows<<<dim3((nw + 255) / 256), dim3(256), 0, st>>>(
            h->win_seg_d, h->win_off_d, win_row ? h->win_row_d : nullptr, w0, nw, s0, is_rc ? 1 : 0, L, n_ph,
            make_int4(ph_idx[0], ph_idx[1], ph_idx[2], ph_idx[3]), g.T6, (long long)sd * n_win, h->a_rows,
            h->c_rows);
        if ((rc = check_launch("seg_a_rows"))) return rc;
        if ((rc = run_fc(h, h->P, h->a_rows, nw, y, st, h->c_rows))) return rc;
      }
      s0 = s1;
    }
  }
  return EXPECTO_OK;
}
// Trunk (conv1..conv6) of nseg segments of length L with pool2 phase 0 only (segment
// starts 16-aligned relative to the windows they stand in for); conv6 rows end in `pbuf`.
int run_trunk_phase0(expecto_beluga* h, const uint8_t* codes, long long stride, int nseg, int L, float* pbuf,
                     float* qbuf, SegGeo& g, hipStream_t st) {
  int rc;
  g = seg_geo(L, 1);
  if ((rc = run_conv1(h, nullptr, codes, stride, nseg, EXPECTO_STRAND_FWD, 0, nseg, L, g.S1, st, pbuf))) return rc;
  if ((rc = run_conv(h, 0, pbuf, qbuf, nseg, g.S1, g.P1, g.P1, true, st))) return rc;
  if ((rc = run_conv(h, 1, qbuf, pbuf, nseg, g.P1, g.T3, g.T3, false, st))) return rc;
  if ((rc = run_conv(h, 2, pbuf, qbuf, nseg, g.T3, g.T4, g.T4, false, st))) return rc;
  {
    LayerTimer lt(h, 3, st);
    pool4_phases<<<dim3(g.S5, nseg), dim3(480), 0, st>>>(qbuf, nseg, g.T4, g.T4, 480, 1, make_int4(0, 0, 0, 0),
                                                         g.S5, pbuf, x3_act());
    if ((rc = check_launch("pool4_phases"))) return rc;
  }
  if ((rc = run_conv(h, 3, pbuf, qbuf, nseg, g.S5, g.T5, g.T5, false, st))) return rc;
  return run_conv(h, 4, qbuf, pbuf, nseg, g.T5, g.T6, g.T6, false, st);
}

int forward_pairs(expecto_beluga* h, const uint8_t* ref, const uint8_t* alt, int n, long long stride,
                  const int* var_pos, int mode, float* y_ref, float* y_alt, long long strand_stride, hipStream_t st) {
  g_precision = h->precision;
  const int strands = mode == EXPECTO_STRAND_BOTH ? 2 : 1;
  if (!h->P2) {
    const SegGeo g = seg_geo(kPatchLen, 1);
    size_t pf = (size_t)h->max_batch * g.p_rows_floats + 16 * 640, qf = (size_t)h->max_batch * g.q_rows_floats + 16 * 640;
    int rc;
    if ((rc = dalloc(h, &h->P2, act_alloc(pf))) || (rc = dalloc(h, &h->Q2, act_alloc(qf)))) return rc;
    float* pc = nullptr;
    if ((rc = dalloc(h, &pc, ((size_t)h->max_batch * kPatchLen + 3) / 4))) return rc;
    h->patch_codes = reinterpret_cast<uint8_t*>(pc);
  }
  const int nv_max = std::max(1, h->max_batch / strands);
  int rc;
  for (int v0 = 0; v0 < n; v0 += nv_max) {
    const int nv = std::min(nv_max, n - v0), R = strands * nv;
    // ref windows: full per-window trunk, conv6 rows stay in Q
    if ((rc = run_conv1(h, nullptr, ref + (long long)v0 * stride, stride, nv, mode, 0, R, kLen, kS1, st))) return rc;
    float* src = h->P;
    float* dst = h->Q;
    for (int l = 0; l < 5; ++l) {
      const ConvGeo& g = kConv[l];
      if ((rc = run_conv(h, l, src, dst, R, g.s_in, g.t_valid, g.s_out, g.pool != 0, st))) return rc;
      std::swap(src, dst);
    }
    float* act6 = src;
    pair_rows<<<dim3((R + 255) / 256), dim3(256), 0, st>>>(h->c_rows, R, nv, v0, strand_stride);
    if ((rc = check_launch("pair_rows"))) return rc;
    if ((rc = run_fc(h, act6, nullptr, R, y_ref, st, h->c_rows))) return rc;
    // alt windows: 600-bp patch trunk, patch rows spliced into the ref conv6 rows
    pair_patch_codes<<<dim3((kPatchLen + 255) / 256, R), dim3(256), 0, st>>>(alt + 0, stride, nv, v0, var_pos,
                                                                            h->patch_codes);
    if ((rc = check_launch("pair_patch_codes"))) return rc;
    SegGeo pg;
    if ((rc = run_trunk_phase0(h, h->patch_codes, kPatchLen, R, kPatchLen, h->P2, h->Q2, pg, st))) return rc;
    EXPECTO_REQUIRE(pg.T6 == kPatchRows, "patch geometry");
    pair_patch_apply<<<dim3(kPatchRows, R), dim3(256), 0, st>>>(h->P2, act6, nv, v0, var_pos,
                                                                x3_act() ? 240 : 160);
    if ((rc = check_launch("pair_patch_apply"))) return rc;
    if ((rc = run_fc(h, act6, nullptr, R, y_alt, st, h->c_rows))) return rc;
  }
  return EXPECTO_OK;
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
  int rc = 0;
  auto fail = [&](int code) {
    expecto_beluga_destroy(h);
    return code;
  };
  if ((rc = dalloc(h, &h->w1, 320 * 32)) || (rc = dalloc(h, &h->b1, 320))) return fail(rc);
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
  const size_t partf = (size_t)kFcSplits[5] * max_batch * kHidLd;
  if ((rc = dalloc(h, &h->P, act_alloc(pf))) || (rc = dalloc(h, &h->Q, act_alloc(qf))) ||
      (rc = dalloc(h, &h->part, partf)) || (rc = dalloc(h, &h->h1, act_alloc((size_t)max_batch * kHidLd))))
    return fail(rc);
  {
    float* rows = nullptr;
    if ((rc = dalloc(h, &rows, (size_t)max_batch * 4))) return fail(rc);
    h->a_rows = reinterpret_cast<long long*>(rows);
    h->c_rows = h->a_rows + max_batch;
  }
  EXPECTO_HIP_CHECK(hipMemsetAsync(h->P, 0, act_alloc(pf) * sizeof(float), st));
  EXPECTO_HIP_CHECK(hipMemsetAsync(h->Q, 0, act_alloc(qf) * sizeof(float), st));
  EXPECTO_HIP_CHECK(hipStreamSynchronize(st));
  *out = h;
  return EXPECTO_OK;
}

void expecto_beluga_destroy(expecto_beluga_t h) {
  if (!h) return;
  if (h->win_seg_d) (void)hipFree(h->win_seg_d);
  if (h->win_off_d) (void)hipFree(h->win_off_d);
  if (h->win_row_d) (void)hipFree(h->win_row_d);
  for (void* p : h->allocs) (void)hipFree(p);
  for (hipEvent_t e : h->ev_pool) (void)hipEventDestroy(e);
  delete h;
}

size_t expecto_beluga_device_bytes(expecto_beluga_t h) { return h ? h->bytes : 0; }

int expecto_beluga_forward_onehot(expecto_beluga_t h, const float* x, int n, float* y, void* stream) {
  EXPECTO_REQUIRE(h != nullptr, "null handle");
  EXPECTO_REQUIRE(n >= 0, "negative batch");
  if (n == 0) return EXPECTO_OK;
  EXPECTO_REQUIRE(x != nullptr && y != nullptr, "null input/output");
  EXPECTO_HIP_CHECK(hipSetDevice(h->device));
  hipStream_t st = as_stream(stream);
  for (long long r0 = 0; r0 < n; r0 += h->max_batch) {
    const int nb = (int)std::min<long long>(h->max_batch, n - r0);
    int rc = forward_chunk(h, x, nullptr, 0, 0, 0, r0, nb, y + r0 * kNFeat, st);
    if (rc) return rc;
  }
  return EXPECTO_OK;
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
  for (long long r0 = 0; r0 < rows; r0 += h->max_batch) {
    const int nb = (int)std::min<long long>(h->max_batch, rows - r0);
    int rc = forward_chunk(h, nullptr, codes, code_stride, n, strand_mode, r0, nb, y + r0 * kNFeat, st);
    if (rc) return rc;
  }
  return EXPECTO_OK;
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
  return forward_segments(h, codes, n_seg, seg_len, code_stride, strand_mode, win_seg, win_off, win_row, n_win, y,
                          as_stream(stream));
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
  return forward_pairs(h, ref_codes, alt_codes, n, code_stride, var_pos, strand_mode, y_ref, y_alt, strand_stride,
                       as_stream(stream));
}

int expecto_beluga_set_precision(expecto_beluga_t h, int precision) {
  EXPECTO_REQUIRE(h != nullptr, "null handle");
  EXPECTO_REQUIRE(precision == EXPECTO_PRECISION_FP32 || precision == EXPECTO_PRECISION_BF16X6, "bad precision");
  h->precision = precision;
  return EXPECTO_OK;
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
    std::fill(h->ms, h->ms + kNumLayers, 0.0);
    std::fill(h->calls, h->calls + kNumLayers, 0LL);
    std::fill(h->macs, h->macs + kNumLayers, 0.0);
  }
  return EXPECTO_OK;
}

int expecto_beluga_layer_times(expecto_beluga_t h, double* ms, long long* calls, double* macs, int max_layers) {
  EXPECTO_REQUIRE(h != nullptr, "null handle");
  int rc = resolve_events(h);
  if (rc) return rc;
  const int n = std::min(max_layers, kNumLayers);
  for (int i = 0; i < n; ++i) {
    if (ms) ms[i] = h->ms[i];
    if (calls) calls[i] = h->calls[i];
    if (macs) macs[i] = h->macs[i];
  }
  return kNumLayers;
}

}  // extern "C"
