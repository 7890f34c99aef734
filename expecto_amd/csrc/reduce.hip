// HBM-bound kernels around the Beluga forward (gfx950):
//  * variant window generation from a device-resident genome (chromatin.py:175-209),
//  * diff = alt - ref (chromatin.py:281), fwd/rc averaging (predict.py:186-190),
//  * TSS spatial-transform reduction (compute_expecto_features.py:88-124),
//  * variant spatial reduction (predict.py:87-136).
#include <hip/hip_runtime.h>

#include <string>

#include "common.h"

namespace expecto {

thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

constexpr int kLen = 2000;

// One window per blockIdx.y (variant) x blockIdx.z (allele*n_shift + shift); 2000 codes
// per window; 4 codes per thread (uint32 stores).
__global__ void variant_windows_kernel(const uint8_t* __restrict__ genome, long long genome_len,
                                       const long long* __restrict__ var_off, const uint8_t* __restrict__ ref_code,
                                       const uint8_t* __restrict__ alt_code, int n, const int* __restrict__ shifts,
                                       int n_shift, uint8_t* __restrict__ codes) {
  const int v = blockIdx.y;
  const int j = blockIdx.z % n_shift;
  const int allele = blockIdx.z / n_shift;
  const int i4 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i4 >= kLen) return;
  const int shift = shifts[j];
  // crop index i <-> genome offset off_v + shift - 999 + i; variant at i = 999 - shift.
  const long long base = var_off[v] + shift - 999;
  const int mut = 999 - shift;
  const uint8_t allele_code = allele ? alt_code[v] : ref_code[v];
  unsigned packed = 0;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int i = i4 + e;
    const long long g = base + i;
    unsigned c = (g >= 0 && g < genome_len) ? genome[g] : 4u;
    if (i == mut) c = allele_code;
    packed |= c << (8 * e);
  }
  *reinterpret_cast<unsigned*>(codes + ((long long)(allele * n_shift + j) * n + v) * kLen + i4) = packed;
}

// Indel / MNP windows (chromatin.py:202-209 then the centre crop of :164) for items whose
// 2100-base fetch window lies inside its contig, with 0 <= mutpos, mutpos + lref <= 2100 and a
// spliced length >= 2000 (the host keeps the rest, chromatin.py's Python-slicing corner cases).
// Spliced sequence S = G[s0, s0+mutpos) + allele + G[s0+mutpos+lref, s0+2100); output code i =
// S[crop + i], crop = floor((len(S) - 2000) / 2).  Item t: start0[t] = s0, the allele's codes at
// allele_codes[allele_off[t] .. + lalt[t]).  4 codes per thread (uint32 stores).
__global__ void indel_windows_kernel(const uint8_t* __restrict__ genome, long long genome_len,
                                     const long long* __restrict__ start0, const int* __restrict__ mutpos,
                                     const int* __restrict__ lref, const int* __restrict__ lalt,
                                     const int* __restrict__ crop, const int* __restrict__ allele_off,
                                     const uint8_t* __restrict__ allele_codes, uint8_t* __restrict__ codes) {
  const long long t = blockIdx.y;
  const int i4 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i4 >= kLen) return;
  const long long s0 = start0[t];
  const int mp = mutpos[t], lr = lref[t], la = lalt[t], c0 = crop[t], ao = allele_off[t];
  unsigned packed = 0;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int k = c0 + i4 + e;
    unsigned c;
    if (k >= mp && k < mp + la) {
      c = allele_codes[ao + k - mp];
    } else {
      const long long g = s0 + (k < mp ? k : k - la + lr);
      c = (g >= 0 && g < genome_len) ? genome[g] : 4u;
    }
    packed |= c << (8 * e);
  }
  *reinterpret_cast<unsigned*>(codes + t * kLen + i4) = packed;
}

// TSS tiling (compute_expecto_features.py:107-111): window of gene g at shift s covers the
// 1-based positions tss + s*strand - 999 .. tss + s*strand + 1000 -> 0-based offset
// tss_off[g] + s*strand - 999 + i.  Output codes[(g*n_shift + j)*2000 + i].
__global__ void tss_windows_kernel(const uint8_t* __restrict__ genome, long long genome_len,
                                   const long long* __restrict__ tss_off, const int8_t* __restrict__ strand,
                                   const int* __restrict__ shifts, int n_shift, uint8_t* __restrict__ codes) {
  const long long g = blockIdx.y;
  const int j = blockIdx.z;
  const int i4 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i4 >= kLen) return;
  const long long base = tss_off[g] + (long long)shifts[j] * strand[g] - 999;
  unsigned packed = 0;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const long long q = base + i4 + e;
    const unsigned c = (q >= 0 && q < genome_len) ? genome[q] : 4u;
    packed |= c << (8 * e);
  }
  *reinterpret_cast<unsigned*>(codes + (g * n_shift + j) * kLen + i4) = packed;
}

// grid: (ceil(seg_len/1024), n); 4 codes per thread.
__global__ void gather_segments_kernel(const uint8_t* __restrict__ genome, long long genome_len,
                                       const long long* __restrict__ start, int seg_len,
                                       const int* __restrict__ splice_pos, const uint8_t* __restrict__ splice_code,
                                       uint8_t* __restrict__ codes) {
  const long long i = blockIdx.y;
  const int j4 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (j4 >= seg_len) return;
  const long long base = start[i];
  const int sp = splice_code ? splice_pos[i] : -1;
  unsigned packed = 0;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const long long q = base + j4 + e;
    unsigned c = (q >= 0 && q < genome_len) ? genome[q] : 4u;
    if (j4 + e == sp) c = splice_code[i];
    packed |= c << (8 * e);
  }
  *reinterpret_cast<unsigned*>(codes + i * seg_len + j4) = packed;
}

__global__ void diff_kernel(const float4* __restrict__ a, const float4* __restrict__ b, long long n4,
                            float4* __restrict__ out) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    const float4 x = a[i], y = b[i];
    out[i] = make_float4(x.x - y.x, x.y - y.y, x.z - y.z, x.w - y.w);
  }
}

__global__ void diff_scalar(const float* __restrict__ a, const float* __restrict__ b, long long start, long long n,
                            float* __restrict__ out) {
  for (long long i = start + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    out[i] = a[i] - b[i];
}

__global__ void fwd_rc_avg_kernel(const float* __restrict__ x, int rows, int cols, float* __restrict__ out) {
  const long long total = (long long)rows * cols;
  const long long half = total;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x)
    out[i] = (x[i] + x[i + half]) / 2.0f;
}

// Generalised shift reduction (geuvadis_sed_for_top_eqtls.py:95-121,
// geuvadis_predict_consensus.py:110-128): F64AVG averages fwd/rc in float64
// ((double)a + (double)b) / 2 like numpy on float64 prediction arrays; LEGACY writes the
// "backwards compatibility" layout 10 x [0, f_0 .. f_{nfeat-1}] (a zero column ahead of each
// decay block: 10 * (nfeat + 1) = 20030 features).  Shifts are summed sequentially in order.
// Shifts whose input loads a reduction thread issues together before it runs their products
// (all four shift/spatial reductions below): the sums still go shift by shift in order, so the
// results are bitwise those of the one-load-then-products loop.
constexpr int kRedChunk = 8;

template <bool F64AVG, bool LEGACY>
__global__ void shift_reduce_kernel(const float* __restrict__ fwd, const float* __restrict__ rc,
                                    const double* __restrict__ weights, int n_shift, int nfeat,
                                    double* __restrict__ out) {
#pragma clang fp contract(off)   // products rounded before the sum, as numpy
  extern __shared__ double wsx[];  // [10][n_shift]
  for (int i = threadIdx.x; i < 10 * n_shift; i += blockDim.x) wsx[i] = weights[i];
  __syncthreads();
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  const long long g = blockIdx.y;
  constexpr int kStride = LEGACY ? 1 : 0;
  double* o = out + g * 10LL * (nfeat + kStride);
  if (LEGACY && f < 10) o[(long long)f * (nfeat + 1)] = 0.0;
  if (f >= nfeat) return;
  double acc[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) acc[k] = 0.0;
  const float* pf = fwd + g * n_shift * nfeat + f;
  const float* pr = rc + g * n_shift * nfeat + f;
  // the grid is only n_seq x nfeat threads (~3 waves per SIMD on the 96-variant step), so a
  // loop waiting on every load was latency-bound: a chunk's 2 x kRedChunk loads go out first
  for (int s0 = 0; s0 < n_shift; s0 += kRedChunk) {
    float a[kRedChunk], b[kRedChunk];
#pragma unroll
    for (int u = 0; u < kRedChunk; ++u) {
      if (s0 + u < n_shift) {
        a[u] = pf[(long long)(s0 + u) * nfeat];
        b[u] = pr[(long long)(s0 + u) * nfeat];
      }
    }
#pragma unroll
    for (int u = 0; u < kRedChunk; ++u) {
      if (s0 + u < n_shift) {
        const double pd = F64AVG ? ((double)a[u] + (double)b[u]) / 2.0 : (double)(0.5f * (a[u] + b[u]));
#pragma unroll
        for (int k = 0; k < 10; ++k) acc[k] += wsx[k * n_shift + s0 + u] * pd;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 10; ++k) o[(long long)k * (nfeat + kStride) + kStride + f] = acc[k];
}

// grid: (ceil(nfeat/256), n_genes); thread = feature f; loops over the shifts in order.
__global__ void tss_reduce_kernel(const float* __restrict__ fwd, const float* __restrict__ rc,
                                  const double* __restrict__ weights, int n_shift, int nfeat,
                                  double* __restrict__ out) {
#pragma clang fp contract(off)   // products rounded before the sum, as numpy
  extern __shared__ double wsh[];  // [10][n_shift]
  for (int i = threadIdx.x; i < 10 * n_shift; i += blockDim.x) wsh[i] = weights[i];
  __syncthreads();
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  const long long g = blockIdx.y;
  if (f >= nfeat) return;
  double acc[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) acc[k] = 0.0;
  const float* pf = fwd + g * n_shift * nfeat + f;
  const float* pr = rc + g * n_shift * nfeat + f;
  for (int s = 0; s < n_shift; ++s) {
    const float p = 0.5f * (pf[(long long)s * nfeat] + pr[(long long)s * nfeat]);  // f32 like numpy
    const double pd = (double)p;
#pragma unroll
    for (int k = 0; k < 10; ++k) acc[k] += wsh[k * n_shift + s] * pd;
  }
  double* o = out + g * 10LL * nfeat + f;
#pragma unroll
  for (int k = 0; k < 10; ++k) o[(long long)k * nfeat] = acc[k];
}

typedef double f64x2 __attribute__((ext_vector_type(2)));
// Streaming 16-byte store: outputs are written once and never re-read by the kernel.
__device__ __forceinline__ void store_nt2(double* p, double a, double b) {
  f64x2 v = {a, b};
  __builtin_nontemporal_store(v, reinterpret_cast<f64x2*>(p));
}

// The same with 2 features per thread (nfeat even, 8-byte aligned inputs, 16-byte aligned
// output): float2 loads and double2 stores, so each wave moves 512 B per load instruction and
// 1 KB per store, and half as many workgroups redo the per-gene weight staging.  Per output the
// same shift-sequential products and sums: bitwise equal to tss_reduce_kernel.
__global__ __launch_bounds__(1024) void tss_reduce2_kernel(const float* __restrict__ fwd, const float* __restrict__ rc,
                                   const double* __restrict__ weights, int n_shift, int nfeat,
                                   double* __restrict__ out) {
#pragma clang fp contract(off)   // products rounded before the sum, as numpy
  extern __shared__ double wsh[];  // [10][n_shift]
  const int f = 2 * (blockIdx.x * blockDim.x + threadIdx.x);
  const long long g = blockIdx.y;
  const bool act = f < nfeat;
  const long long h2 = nfeat / 2;
  const float2* pf = reinterpret_cast<const float2*>(fwd + g * n_shift * nfeat + f);
  const float2* pr = reinterpret_cast<const float2*>(rc + g * n_shift * nfeat + f);
  // round 3: the first chunk's loads go out before the weight staging and its barrier
  float2 x[kRedChunk], y[kRedChunk];
#pragma unroll
  for (int u = 0; u < kRedChunk; ++u) {
    if (act && u < n_shift) {
      x[u] = pf[u * h2];
      y[u] = pr[u * h2];
    }
  }
  for (int i = threadIdx.x; i < 10 * n_shift; i += blockDim.x) wsh[i] = weights[i];
  __syncthreads();
  if (!act) return;
  double a0[10], a1[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) a0[k] = a1[k] = 0.0;
  for (int s0 = 0; s0 < n_shift; s0 += kRedChunk) {   // a chunk's loads first, sums in shift order
    if (s0 > 0) {
#pragma unroll
      for (int u = 0; u < kRedChunk; ++u) {
        if (s0 + u < n_shift) {
          x[u] = pf[(s0 + u) * h2];
          y[u] = pr[(s0 + u) * h2];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < kRedChunk; ++u) {
      if (s0 + u < n_shift) {
        const double p0 = (double)(0.5f * (x[u].x + y[u].x)), p1 = (double)(0.5f * (x[u].y + y[u].y));  // f32 like numpy
#pragma unroll
        for (int k = 0; k < 10; ++k) {
          const double w = wsh[k * n_shift + s0 + u];
          a0[k] += w * p0;
          a1[k] += w * p1;
        }
      }
    }
  }
  double* o = out + g * 10LL * nfeat + f;
#pragma unroll
  for (int k = 0; k < 10; ++k) store_nt2(o + (long long)k * nfeat, a0[k], a1[k]);
}

// grid: (ceil(nfeat/256), n); weights W_j[k] computed per variant in f64.
__global__ void variant_reduce_kernel(const float* __restrict__ eff, const long long* __restrict__ dist,
                                      const uint8_t* __restrict__ strand_plus, const int* __restrict__ shifts,
                                      int n_shift, int n, int nfeat, const double* __restrict__ lut,
                                      int lut_len, double* __restrict__ out) {
#pragma clang fp contract(off)   // products rounded before the sum, as numpy
  extern __shared__ double wsh[];   // [n_shift][10]
  const long long v = blockIdx.y;
  const double decay[5] = {0.01, 0.02, 0.05, 0.1, 0.2};
  for (int j = threadIdx.x; j < n_shift; j += blockDim.x) {
    const long long sgn = strand_plus[v] ? 1 : -1;
    const long long d = dist[v] * sgn + (long long)shifts[j] * sgn;
    const double fl = floor(fabs((double)d) / 200.0);
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      // host table exp(-c_k * fl) (numpy's exp, as predict.py:88-107) when given, else the device exp
      // (a table too short for this distance: the device exp, never a read past its end)
      const double e = lut && fl < (double)lut_len ? lut[k * lut_len + (long long)fl] : exp(-decay[k] * fl);
      wsh[j * 10 + k] = d <= 0 ? e : 0.0;
      wsh[j * 10 + 5 + k] = d >= 0 ? e : 0.0;
    }
  }
  __syncthreads();
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= nfeat) return;
  double acc[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) acc[k] = 0.0;
  for (int j = 0; j < n_shift; ++j) {
    const double e = (double)eff[((long long)j * n + v) * nfeat + f];
#pragma unroll
    for (int k = 0; k < 10; ++k) acc[k] += e * wsh[j * 10 + k];
  }
  double* o = out + v * 10LL * nfeat + f;
#pragma unroll
  for (int k = 0; k < 10; ++k) o[(long long)k * nfeat] = acc[k];
}

// 2 features per thread (as tss_reduce2_kernel): 4 instead of 8 workgroups per variant compute
// the 9 x 10 weights, float2 loads and double2 stores; bitwise equal to variant_reduce_kernel.
// The weight prologue of one variant (shared by all its features).
__device__ __forceinline__ void variant_weights_lds(const long long* __restrict__ dist,
                                                    const uint8_t* __restrict__ strand_plus,
                                                    const int* __restrict__ shifts, int n_shift, long long v,
                                                    const double* __restrict__ lut, int lut_len, double* wsh) {
  const double decay[5] = {0.01, 0.02, 0.05, 0.1, 0.2};
  for (int j = threadIdx.x; j < n_shift; j += blockDim.x) {
    const long long sgn = strand_plus[v] ? 1 : -1;
    const long long d = dist[v] * sgn + (long long)shifts[j] * sgn;
    const double fl = floor(fabs((double)d) / 200.0);
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      // host table exp(-c_k * fl) (numpy's exp, as predict.py:88-107) when given, else the device exp
      // (a table too short for this distance: the device exp, never a read past its end)
      const double e = lut && fl < (double)lut_len ? lut[k * lut_len + (long long)fl] : exp(-decay[k] * fl);
      wsh[j * 10 + k] = d <= 0 ? e : 0.0;
      wsh[j * 10 + 5 + k] = d >= 0 ? e : 0.0;
    }
  }
}

__global__ void variant_reduce2_kernel(const float* __restrict__ eff, const long long* __restrict__ dist,
                                       const uint8_t* __restrict__ strand_plus, const int* __restrict__ shifts,
                                       int n_shift, int n, int nfeat, const double* __restrict__ lut,
                                       int lut_len, double* __restrict__ out) {
#pragma clang fp contract(off)   // products rounded before the sum, as numpy
  extern __shared__ double wsh[];   // [n_shift][10]
  const long long v = blockIdx.y;
  variant_weights_lds(dist, strand_plus, shifts, n_shift, v, lut, lut_len, wsh);
  __syncthreads();
  const int f = 2 * (blockIdx.x * blockDim.x + threadIdx.x);
  if (f >= nfeat) return;
  double a0[10], a1[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) a0[k] = a1[k] = 0.0;
  for (int j = 0; j < n_shift; ++j) {
    const float2 e2 = *reinterpret_cast<const float2*>(eff + ((long long)j * n + v) * nfeat + f);
    const double e0 = (double)e2.x, e1 = (double)e2.y;
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      a0[k] += e0 * wsh[j * 10 + k];
      a1[k] += e1 * wsh[j * 10 + k];
    }
  }
  double* o = out + v * 10LL * nfeat + f;
#pragma unroll
  for (int k = 0; k < 10; ++k) store_nt2(o + (long long)k * nfeat, a0[k], a1[k]);
}

// The same sums with line-aligned stores.  An output row is 2002 f64 = 16,016 B, not a whole
// number of 128-B lines, so the per-thread stores above start every 1-KB wave store inside a
// line: 2 of its 9 lines are partial, each a read-modify-write at the memory, and the stores run
// at 0.55-0.60 of 8 TB/s where a fill of the same bytes runs at 0.83-0.85
// (tools/reduce_probe).  Here a 256-pair workgroup keeps its 10 x 2 sums in registers and puts
// each decay row's 4-KB piece through a double-buffered LDS slot, from which its wave stores
// start on 128-B lines: only the piece's first and last line are partial.  Same products and
// sums per output: bitwise equal (probe: 0.63-0.67 vs 0.61-0.64 of 8 TB/s for the kernel above).
constexpr int kRowsPairs = 256;
__global__ __launch_bounds__(kRowsPairs) void variant_reduce_rows_kernel(
    const float* __restrict__ eff, const long long* __restrict__ dist, const uint8_t* __restrict__ strand_plus,
    const int* __restrict__ shifts, int n_shift, int n, int nfeat, const double* __restrict__ lut, int lut_len,
    double* __restrict__ out) {
#pragma clang fp contract(off)   // products rounded before the sum, as numpy
  // the row slots static, the weights in the dynamic region (weights behind a 16-B-aligned
  // dynamic base were read as merged 16-B loads: 66 instead of 56 VGPRs, 7 waves per SIMD)
  __shared__ __attribute__((aligned(16))) double rows_lds[2 * 2 * kRowsPairs];   // [2][256] f64 pairs
  extern __shared__ double wsh[];                                                 // [n_shift][10]
  const long long v = blockIdx.y;
  const int t = threadIdx.x, pb = blockIdx.x * kRowsPairs;
  const int np = min(kRowsPairs, nfeat / 2 - pb);
  variant_weights_lds(dist, strand_plus, shifts, n_shift, v, lut, lut_len, wsh);
  __syncthreads();
  double a0[10], a1[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) a0[k] = a1[k] = 0.0;
  if (t < np) {
    const int f = 2 * (pb + t);
    for (int j = 0; j < n_shift; ++j) {
      const float2 e2 = *reinterpret_cast<const float2*>(eff + ((long long)j * n + v) * nfeat + f);
      const double e0 = (double)e2.x, e1 = (double)e2.y;
#pragma unroll
      for (int k = 0; k < 10; ++k) {
        a0[k] += e0 * wsh[j * 10 + k];
        a1[k] += e1 * wsh[j * 10 + k];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    // slot k & 1: the barrier of row k+1 orders every thread's reads of row k-1 before its reuse
    double* const sb = rows_lds + (k & 1) * 2 * kRowsPairs;
    if (t < np) *reinterpret_cast<f64x2*>(sb + 2 * t) = f64x2{a0[k], a1[k]};
    __syncthreads();
    double* const row = out + (v * 10 + k) * (long long)nfeat + 2 * pb;
    const int lead = (int)(((unsigned long long)(size_t)row & 127) >> 4);   // 16-B slots before its line
    for (int s = t; s < lead + np; s += kRowsPairs) {
      const int piece = s - lead;
      if (piece >= 0) {
        const f64x2 x = *reinterpret_cast<const f64x2*>(sb + 2 * piece);
        store_nt2(row + 2 * piece, x.x, x.y);
      }
    }
  }
}

}  // namespace expecto

using namespace expecto;

// ---- gblinear scoring (predict.py:150-166, xgboost 0.7 GBLinear::Pred) ---------------------
// out[m] = init + sum_j float32(X[m][cols[j]]) * w[j], accumulated in float32 in column order
// with separate rounding of every product and sum (no FMA) -- the reference's CPU loop.  One
// thread per row (64 rows per block); each 64-column slab of the 64 rows is staged through LDS
// with row-contiguous (coalesced) loads.
__global__ __launch_bounds__(64) void gblinear_kernel(const double* __restrict__ X, long long n, long long ld,
                                                      const int* __restrict__ cols, int ncols,
                                                      const float* __restrict__ w, float init,
                                                      float* __restrict__ out) {
#pragma clang fp contract(off)   // products and sums rounded separately (HIP's __fmul_rn is a plain *)
  __shared__ float tile[64][65];
  __shared__ float ws[64];
  const long long r0 = (long long)blockIdx.x * 64;
  const int t = threadIdx.x;
  float psum = init;
  for (int j0 = 0; j0 < ncols; j0 += 64) {
    const int j = j0 + t;
    const int c = j < ncols ? cols[j] : 0;
    ws[t] = j < ncols ? w[j] : 0.f;
    for (int rr = 0; rr < 64; ++rr) {
      const long long m = r0 + rr;
      tile[rr][t] = (m < n && j < ncols) ? (float)X[m * ld + c] : 0.f;
    }
    __syncthreads();
    const int jn = min(64, ncols - j0);
    for (int jj = 0; jj < jn; ++jj) psum = psum + tile[t][jj] * ws[jj];
    __syncthreads();
  }
  if (r0 + t < n) out[r0 + t] = psum;
}

extern "C" {

const char* expecto_last_error(void) { return g_last_error.c_str(); }
const char* expecto_version(void) { return "expecto_hip 0.1.0 gfx950"; }

int expecto_variant_windows(const uint8_t* genome, long long genome_len, const long long* var_off,
                            const uint8_t* ref_code, const uint8_t* alt_code, int n, const int* shifts, int n_shift,
                            uint8_t* codes, void* stream) {
  EXPECTO_REQUIRE(n >= 0 && n_shift > 0 && n_shift <= 65535 / 2, "bad variant/shift count");
  if (n == 0) return EXPECTO_OK;
  EXPECTO_REQUIRE(n <= 65535, "at most 65535 variants per call");
  EXPECTO_REQUIRE(genome && var_off && ref_code && alt_code && shifts && codes, "null argument");
  dim3 grid((kLen / 4 + 255) / 256, n, 2 * n_shift);
  variant_windows_kernel<<<grid, dim3(256), 0, as_stream(stream)>>>(genome, genome_len, var_off, ref_code, alt_code, n,
                                                                    shifts, n_shift, codes);
  return check_launch("variant_windows");
}

int expecto_indel_windows(const uint8_t* genome, long long genome_len, const long long* start0, const int* mutpos,
                          const int* lref, const int* lalt, const int* crop, const int* allele_off,
                          const uint8_t* allele_codes, int n, uint8_t* codes, void* stream) {
  EXPECTO_REQUIRE(n >= 0 && n <= 65535, "0..65535 indel windows per call");
  if (n == 0) return EXPECTO_OK;
  EXPECTO_REQUIRE(genome && start0 && mutpos && lref && lalt && crop && allele_off && allele_codes && codes,
                  "null argument");
  dim3 grid((kLen / 4 + 255) / 256, n);
  indel_windows_kernel<<<grid, dim3(256), 0, as_stream(stream)>>>(genome, genome_len, start0, mutpos, lref, lalt, crop,
                                                                  allele_off, allele_codes, codes);
  return check_launch("indel_windows");
}

int expecto_tss_windows(const uint8_t* genome, long long genome_len, const long long* tss_off, const int8_t* strand,
                        int n_genes, const int* shifts, int n_shift, uint8_t* codes, void* stream) {
  EXPECTO_REQUIRE(n_genes >= 0 && n_shift > 0 && n_shift <= 65535, "bad gene/shift count");
  if (n_genes == 0) return EXPECTO_OK;
  EXPECTO_REQUIRE(n_genes <= 65535, "at most 65535 genes per call");
  EXPECTO_REQUIRE(genome && tss_off && strand && shifts && codes, "null argument");
  dim3 grid((kLen / 4 + 255) / 256, n_genes, n_shift);
  tss_windows_kernel<<<grid, dim3(256), 0, as_stream(stream)>>>(genome, genome_len, tss_off, strand, shifts, n_shift,
                                                                codes);
  return check_launch("tss_windows");
}

int expecto_gather_segments(const uint8_t* genome, long long genome_len, const long long* start, int n, int seg_len,
                            const int* splice_pos, const uint8_t* splice_code, uint8_t* codes, void* stream) {
  EXPECTO_REQUIRE(n >= 0 && seg_len > 0 && seg_len % 4 == 0, "bad segment shape (seg_len % 4 == 0)");
  if (n == 0) return EXPECTO_OK;
  EXPECTO_REQUIRE(n <= 65535, "at most 65535 segments per call");
  EXPECTO_REQUIRE(genome && start && codes && (!splice_code || splice_pos), "null argument");
  dim3 grid((seg_len / 4 + 255) / 256, n);
  gather_segments_kernel<<<grid, dim3(256), 0, as_stream(stream)>>>(genome, genome_len, start, seg_len, splice_pos,
                                                                    splice_code, codes);
  return check_launch("gather_segments");
}

int expecto_diff(const float* alt, const float* ref, long long count, float* out, void* stream) {
  EXPECTO_REQUIRE(count >= 0, "negative count");
  if (count == 0) return EXPECTO_OK;
  EXPECTO_REQUIRE(alt && ref && out, "null argument");
  hipStream_t st = as_stream(stream);
  if (((uintptr_t)alt | (uintptr_t)ref | (uintptr_t)out) % 16 != 0) {
    const long long blocks = std::min<long long>((count + 255) / 256, 8192);
    diff_scalar<<<dim3((unsigned)blocks), dim3(256), 0, st>>>(alt, ref, 0, count, out);
    return check_launch("diff");
  }
  const long long n4 = count / 4;
  if (n4 > 0) {
    const long long blocks = std::min<long long>((n4 + 255) / 256, 8192);
    diff_kernel<<<dim3((unsigned)blocks), dim3(256), 0, st>>>(
        reinterpret_cast<const float4*>(alt), reinterpret_cast<const float4*>(ref), n4, reinterpret_cast<float4*>(out));
  }
  if (count % 4) diff_scalar<<<1, 64, 0, st>>>(alt, ref, n4 * 4, count, out);
  return check_launch("diff");
}

int expecto_fwd_rc_average(const float* x, int rows, int cols, float* out, void* stream) {
  EXPECTO_REQUIRE(rows >= 0 && cols >= 0, "negative shape");
  if (rows == 0 || cols == 0) return EXPECTO_OK;
  EXPECTO_REQUIRE(x && out, "null argument");
  const long long total = (long long)rows * cols;
  const long long blocks = std::min<long long>((total + 255) / 256, 8192);
  fwd_rc_avg_kernel<<<dim3((unsigned)blocks), dim3(256), 0, as_stream(stream)>>>(x, rows, cols, out);
  return check_launch("fwd_rc_average");
}

// The reductions stage their [n_shift][10] f64 weights in dynamic LDS: at most 64 KiB per
// workgroup without an opt-in attribute, so 819 shifts (the reference sweeps 9 to 201).
constexpr int kMaxShifts = 65536 / (10 * (int)sizeof(double));

int expecto_tss_reduce(const float* fwd, const float* rc, const double* weights, int n_genes, int n_shift, int nfeat,
                       double* out, void* stream) {
  EXPECTO_REQUIRE(n_genes >= 0 && n_shift > 0 && n_shift <= kMaxShifts && nfeat > 0, "bad shape (n_shift <= 819)");
  if (n_genes == 0) return EXPECTO_OK;
  EXPECTO_REQUIRE(n_genes <= 65535, "at most 65535 genes per call");
  EXPECTO_REQUIRE(fwd && rc && weights && out, "null argument");
  const bool v2 = nfeat % 2 == 0 && ((reinterpret_cast<uintptr_t>(fwd) | reinterpret_cast<uintptr_t>(rc)) & 7) == 0 &&
                  (reinterpret_cast<uintptr_t>(out) & 15) == 0;
  if (v2) {
    // 1024-thread workgroups: one per gene streams whole 8-KB rows (2002 features) and stages the
    // weights once per gene (tools/reduce_probe: 0.68 vs 0.66 of 8 TB/s for 256 threads; a
    // loads-and-stores-only kernel of the same pattern reaches 0.68-0.69)
    dim3 grid((nfeat / 2 + 1023) / 1024, n_genes);
    tss_reduce2_kernel<<<grid, dim3(1024), 10 * n_shift * sizeof(double), as_stream(stream)>>>(fwd, rc, weights,
                                                                                              n_shift, nfeat, out);
  } else {
    dim3 grid((nfeat + 255) / 256, n_genes);
    tss_reduce_kernel<<<grid, dim3(256), 10 * n_shift * sizeof(double), as_stream(stream)>>>(fwd, rc, weights, n_shift,
                                                                                            nfeat, out);
  }
  return check_launch("tss_reduce");
}

int expecto_variant_reduce_lut(const float* effects, const long long* dist, const uint8_t* strand_plus,
                               const int* shifts, int n_shift, int n, int nfeat, const double* exp_lut, int lut_len,
                               double* out, void* stream) {
  EXPECTO_REQUIRE(n >= 0 && n_shift > 0 && n_shift <= kMaxShifts && nfeat > 0, "bad shape (n_shift <= 819)");
  if (n == 0) return EXPECTO_OK;
  EXPECTO_REQUIRE(n <= 65535, "at most 65535 variants per call");
  EXPECTO_REQUIRE(effects && dist && strand_plus && shifts && out, "null argument");
  EXPECTO_REQUIRE(!exp_lut || lut_len > 0, "empty exp table");
  const size_t shm = 10 * (size_t)n_shift * sizeof(double);
  const bool v2 =
      nfeat % 2 == 0 && (reinterpret_cast<uintptr_t>(effects) & 7) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0;
  if (v2 && shm + 2 * 2 * kRowsPairs * sizeof(double) <= 65536) {   // <= 716 shifts (the reference sweeps 9)
    dim3 grid((nfeat / 2 + kRowsPairs - 1) / kRowsPairs, n);
    variant_reduce_rows_kernel<<<grid, dim3(kRowsPairs), shm, as_stream(stream)>>>(
        effects, dist, strand_plus, shifts, n_shift, n, nfeat, exp_lut, lut_len, out);
  } else if (v2) {
    dim3 grid((nfeat / 2 + 255) / 256, n);
    variant_reduce2_kernel<<<grid, dim3(256), shm, as_stream(stream)>>>(effects, dist, strand_plus, shifts, n_shift, n,
                                                                      nfeat, exp_lut, lut_len, out);
  } else {
    dim3 grid((nfeat + 255) / 256, n);
    variant_reduce_kernel<<<grid, dim3(256), shm, as_stream(stream)>>>(effects, dist, strand_plus, shifts, n_shift, n,
                                                                     nfeat, exp_lut, lut_len, out);
  }
  return check_launch("variant_reduce");
}

int expecto_variant_reduce(const float* effects, const long long* dist, const uint8_t* strand_plus, const int* shifts,
                           int n_shift, int n, int nfeat, double* out, void* stream) {
  return expecto_variant_reduce_lut(effects, dist, strand_plus, shifts, n_shift, n, nfeat, nullptr, 0, out, stream);
}

int expecto_gblinear_predict(const double* X, long long n, long long ld, const int* cols, int ncols, const float* w,
                             float init, float* out, void* stream) {
  EXPECTO_REQUIRE(n >= 0 && ncols >= 0 && ld >= 0, "negative shape");
  if (n == 0) return EXPECTO_OK;
  EXPECTO_REQUIRE(X && out && (ncols == 0 || (cols && w)), "null argument");
  EXPECTO_REQUIRE((n + 63) / 64 < (1LL << 31), "too many rows");
  gblinear_kernel<<<dim3((unsigned)((n + 63) / 64)), dim3(64), 0, as_stream(stream)>>>(X, n, ld, cols, ncols, w, init,
                                                                                      out);
  return check_launch("gblinear_predict");
}

int expecto_shift_reduce(const float* fwd, const float* rc, const double* weights, int n_genes, int n_shift, int nfeat,
                         int flags, double* out, void* stream) {
  EXPECTO_REQUIRE(n_genes >= 0 && n_shift > 0 && n_shift <= kMaxShifts && nfeat >= 10, "bad shape (n_shift <= 819)");
  EXPECTO_REQUIRE((flags & ~3) == 0, "bad flags");
  if (n_genes == 0) return EXPECTO_OK;
  EXPECTO_REQUIRE(n_genes <= 65535, "at most 65535 sequences per call");
  EXPECTO_REQUIRE(fwd && rc && weights && out, "null argument");
  dim3 grid((nfeat + 255) / 256, n_genes);
  const size_t shm = 10 * n_shift * sizeof(double);
  hipStream_t st = as_stream(stream);
  switch (flags) {
    case 0: shift_reduce_kernel<false, false><<<grid, dim3(256), shm, st>>>(fwd, rc, weights, n_shift, nfeat, out); break;
    case 1: shift_reduce_kernel<true, false><<<grid, dim3(256), shm, st>>>(fwd, rc, weights, n_shift, nfeat, out); break;
    case 2: shift_reduce_kernel<false, true><<<grid, dim3(256), shm, st>>>(fwd, rc, weights, n_shift, nfeat, out); break;
    default: shift_reduce_kernel<true, true><<<grid, dim3(256), shm, st>>>(fwd, rc, weights, n_shift, nfeat, out); break;
  }
  return check_launch("shift_reduce");
}

}  // extern "C"
