// Probe of the HBM-bound reductions (expecto_amd/csrc/reduce.hip) on the bench's shapes
// (bench.hbm_reductions): the library kernels against restructured candidates and against
// memory-only kernels with the SAME access pattern and bytes (the "ceiling" rows: loads and
// stores only, no float64 math), so a kernel's gap splits into pattern vs arithmetic.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/reduce_probe.hip -o tools/reduce_probe
// Run:   tools/reduce_probe [rounds=5]
// Interleaved rounds in one process; every candidate is compared bit for bit with the library
// kernel it replaces.
#include "../expecto_amd/csrc/reduce.hip"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <vector>

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));         \
      exit(1);                                                                                  \
    }                                                                                           \
  } while (0)

namespace probe {
using expecto::f64x2;
using expecto::store_nt2;
using expecto::variant_weights_lds;

// ---- memory-only rows -------------------------------------------------------------------------
__global__ void fill_nt(double* __restrict__ out, long long n2) {   // n2 = number of f64 pairs
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n2) store_nt2(out + 2 * i, 0.0, 0.0);
}

// TSS pattern: the same grid, loads (200 shifts x fwd/rc float2 per thread, chunks of 8) and
// stores (10 x 16 B per thread) as tss_reduce2_kernel, one f32 add per load instead of the math
template <int CH>
__global__ void tss_pattern(const float* __restrict__ fwd, const float* __restrict__ rc, int n_shift, int nfeat,
                            double* __restrict__ out) {
  const int f = 2 * (blockIdx.x * blockDim.x + threadIdx.x);
  const long long g = blockIdx.y;
  if (f >= nfeat) return;
  const long long h2 = nfeat / 2;
  const float2* pf = reinterpret_cast<const float2*>(fwd + g * n_shift * nfeat + f);
  const float2* pr = reinterpret_cast<const float2*>(rc + g * n_shift * nfeat + f);
  float sx = 0.f, sy = 0.f;
  for (int s0 = 0; s0 < n_shift; s0 += CH) {
    float2 x[CH], y[CH];
#pragma unroll
    for (int u = 0; u < CH; ++u)
      if (s0 + u < n_shift) {
        x[u] = pf[(s0 + u) * h2];
        y[u] = pr[(s0 + u) * h2];
      }
#pragma unroll
    for (int u = 0; u < CH; ++u)
      if (s0 + u < n_shift) {
        sx += x[u].x + y[u].x;
        sy += x[u].y + y[u].y;
      }
  }
  double* o = out + g * 10LL * nfeat + f;
#pragma unroll
  for (int k = 0; k < 10; ++k) store_nt2(o + (long long)k * nfeat, sx + k, sy + k);
}

// variant pattern: variant_reduce2_kernel's grid, 9 float2 loads and 10 x 16 B stores per thread
__global__ void variant_pattern(const float* __restrict__ eff, int n_shift, int n, int nfeat, double* __restrict__ out) {
  const long long v = blockIdx.y;
  const int f = 2 * (blockIdx.x * blockDim.x + threadIdx.x);
  if (f >= nfeat) return;
  float sx = 0.f, sy = 0.f;
  for (int j = 0; j < n_shift; ++j) {
    const float2 e2 = *reinterpret_cast<const float2*>(eff + ((long long)j * n + v) * nfeat + f);
    sx += e2.x;
    sy += e2.y;
  }
  double* o = out + v * 10LL * nfeat + f;
#pragma unroll
  for (int k = 0; k < 10; ++k) store_nt2(o + (long long)k * nfeat, sx + k, sy + k);
}

// ---- candidates ---------------------------------------------------------------------------
// TSS, software-pipelined: chunk c+1's loads are issued before chunk c's products (two register
// chunks), so a wave always has loads in flight; per output the same shift-ordered sums
template <int CH>
__global__ void tss_pipe(const float* __restrict__ fwd, const float* __restrict__ rc, const double* __restrict__ weights,
                         int n_shift, int nfeat, double* __restrict__ out) {
#pragma clang fp contract(off)
  extern __shared__ double wsh[];
  const int f = 2 * (blockIdx.x * blockDim.x + threadIdx.x);
  const long long g = blockIdx.y;
  const bool act = f < nfeat;
  const long long h2 = nfeat / 2;
  const float2* pf = reinterpret_cast<const float2*>(fwd + g * n_shift * nfeat + f);
  const float2* pr = reinterpret_cast<const float2*>(rc + g * n_shift * nfeat + f);
  float2 xa[CH], ya[CH], xb[CH], yb[CH];
  auto load = [&](int s0, float2 (&x)[CH], float2 (&y)[CH]) {
#pragma unroll
    for (int u = 0; u < CH; ++u)
      if (act && s0 + u < n_shift) {
        x[u] = pf[(s0 + u) * h2];
        y[u] = pr[(s0 + u) * h2];
      }
  };
  load(0, xa, ya);
  for (int i = threadIdx.x; i < 10 * n_shift; i += blockDim.x) wsh[i] = weights[i];
  __syncthreads();
  if (!act) return;
  double a0[10], a1[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) a0[k] = a1[k] = 0.0;
  auto sum = [&](int s0, const float2 (&x)[CH], const float2 (&y)[CH]) {
#pragma unroll
    for (int u = 0; u < CH; ++u)
      if (s0 + u < n_shift) {
        const double p0 = (double)(0.5f * (x[u].x + y[u].x)), p1 = (double)(0.5f * (x[u].y + y[u].y));
#pragma unroll
        for (int k = 0; k < 10; ++k) {
          const double w = wsh[k * n_shift + s0 + u];
          a0[k] += w * p0;
          a1[k] += w * p1;
        }
      }
  };
  for (int s0 = 0; s0 < n_shift; s0 += 2 * CH) {
    load(s0 + CH, xb, yb);
    sum(s0, xa, ya);
    if (s0 + CH >= n_shift) break;
    load(s0 + 2 * CH, xa, ya);
    sum(s0 + CH, xb, yb);
  }
  double* o = out + g * 10LL * nfeat + f;
#pragma unroll
  for (int k = 0; k < 10; ++k) store_nt2(o + (long long)k * nfeat, a0[k], a1[k]);
}

// variant, every load issued before the weight prologue (n_shift <= NS)
template <int NS>
__global__ void variant_hoist(const float* __restrict__ eff, const long long* __restrict__ dist,
                              const uint8_t* __restrict__ strand_plus, const int* __restrict__ shifts, int n_shift,
                              int n, int nfeat, const double* __restrict__ lut, int lut_len, double* __restrict__ out) {
#pragma clang fp contract(off)
  extern __shared__ double wsh[];
  const long long v = blockIdx.y;
  const int f = 2 * (blockIdx.x * blockDim.x + threadIdx.x);
  const bool act = f < nfeat;
  float2 e[NS];
#pragma unroll
  for (int j = 0; j < NS; ++j)
    if (act && j < n_shift) e[j] = *reinterpret_cast<const float2*>(eff + ((long long)j * n + v) * nfeat + f);
  variant_weights_lds(dist, strand_plus, shifts, n_shift, v, lut, lut_len, wsh);
  __syncthreads();
  if (!act) return;
  double a0[10], a1[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) a0[k] = a1[k] = 0.0;
#pragma unroll
  for (int j = 0; j < NS; ++j)
    if (j < n_shift) {
      const double e0 = (double)e[j].x, e1 = (double)e[j].y;
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

// variant, two variants per 512-thread workgroup (one weight table each, halves of the block)
__global__ void variant_two(const float* __restrict__ eff, const long long* __restrict__ dist,
                            const uint8_t* __restrict__ strand_plus, const int* __restrict__ shifts, int n_shift, int n,
                            int nfeat, const double* __restrict__ lut, int lut_len, double* __restrict__ out) {
#pragma clang fp contract(off)
  extern __shared__ double wsh2[];
  const int half = threadIdx.x >> 8, t = threadIdx.x & 255;
  const long long v = 2LL * blockIdx.y + half;
  if (v >= n) return;
  double* wsh = wsh2 + half * 10 * n_shift;
  const double decay[5] = {0.01, 0.02, 0.05, 0.1, 0.2};
  for (int j = t; j < n_shift; j += 256) {
    const long long sgn = strand_plus[v] ? 1 : -1;
    const long long d = dist[v] * sgn + (long long)shifts[j] * sgn;
    const double fl = floor(fabs((double)d) / 200.0);
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const double e = lut && fl < (double)lut_len ? lut[k * lut_len + (long long)fl] : exp(-decay[k] * fl);
      wsh[j * 10 + k] = d <= 0 ? e : 0.0;
      wsh[j * 10 + 5 + k] = d >= 0 ? e : 0.0;
    }
  }
  __syncthreads();
  const int f = 2 * (blockIdx.x * 256 + t);
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

// the library kernels' bodies with a different workgroup size BS (grid x = ceil(pairs / BS)):
// BS 1024 = one workgroup streams whole 8-KB rows (TSS) / writes whole 16-KB output rows (variant)
template <int BS>
__global__ __launch_bounds__(BS) void tss_bs(const float* __restrict__ fwd, const float* __restrict__ rc,
                                             const double* __restrict__ weights, int n_shift, int nfeat,
                                             double* __restrict__ out) {
#pragma clang fp contract(off)
  extern __shared__ double wsh[];
  const int f = 2 * (blockIdx.x * BS + threadIdx.x);
  const long long g = blockIdx.y;
  const bool act = f < nfeat;
  const long long h2 = nfeat / 2;
  const float2* pf = reinterpret_cast<const float2*>(fwd + g * n_shift * nfeat + f);
  const float2* pr = reinterpret_cast<const float2*>(rc + g * n_shift * nfeat + f);
  constexpr int CH = 8;
  float2 x[CH], y[CH];
#pragma unroll
  for (int u = 0; u < CH; ++u)
    if (act && u < n_shift) {
      x[u] = pf[u * h2];
      y[u] = pr[u * h2];
    }
  for (int i = threadIdx.x; i < 10 * n_shift; i += BS) wsh[i] = weights[i];
  __syncthreads();
  if (!act) return;
  double a0[10], a1[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) a0[k] = a1[k] = 0.0;
  for (int s0 = 0; s0 < n_shift; s0 += CH) {
    if (s0 > 0) {
#pragma unroll
      for (int u = 0; u < CH; ++u)
        if (s0 + u < n_shift) {
          x[u] = pf[(s0 + u) * h2];
          y[u] = pr[(s0 + u) * h2];
        }
    }
#pragma unroll
    for (int u = 0; u < CH; ++u)
      if (s0 + u < n_shift) {
        const double p0 = (double)(0.5f * (x[u].x + y[u].x)), p1 = (double)(0.5f * (x[u].y + y[u].y));
#pragma unroll
        for (int k = 0; k < 10; ++k) {
          const double w = wsh[k * n_shift + s0 + u];
          a0[k] += w * p0;
          a1[k] += w * p1;
        }
      }
  }
  double* o = out + g * 10LL * nfeat + f;
#pragma unroll
  for (int k = 0; k < 10; ++k) store_nt2(o + (long long)k * nfeat, a0[k], a1[k]);
}

template <int BS>
__global__ __launch_bounds__(BS) void variant_bs(const float* __restrict__ eff, const long long* __restrict__ dist,
                                                 const uint8_t* __restrict__ strand_plus, const int* __restrict__ shifts,
                                                 int n_shift, int n, int nfeat, const double* __restrict__ lut,
                                                 int lut_len, double* __restrict__ out) {
#pragma clang fp contract(off)
  extern __shared__ double wsh[];
  const long long v = blockIdx.y;
  variant_weights_lds(dist, strand_plus, shifts, n_shift, v, lut, lut_len, wsh);
  __syncthreads();
  const int f = 2 * (blockIdx.x * BS + threadIdx.x);
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


// variant pattern with the effects variant-major ([n][S][F]: a variant's 9 rows contiguous)
template <bool READ, bool WRITE>
__global__ void variant_pattern_vmajor(const float* __restrict__ eff, int n_shift, int n, int nfeat,
                                       double* __restrict__ out) {
  const long long v = blockIdx.y;
  const int f = 2 * (blockIdx.x * blockDim.x + threadIdx.x);
  if (f >= nfeat) return;
  float sx = 0.f, sy = 0.f;
  if (READ)
    for (int j = 0; j < n_shift; ++j) {
      const float2 e2 = *reinterpret_cast<const float2*>(eff + (v * n_shift + j) * nfeat + f);
      sx += e2.x;
      sy += e2.y;
    }
  double* o = out + v * 10LL * nfeat + f;
  if (WRITE) {
#pragma unroll
    for (int k = 0; k < 10; ++k) store_nt2(o + (long long)k * nfeat, sx + k, sy + k);
  } else if (sx == -1.f) {
    o[0] = sy;
  }
}

// the shift-major pattern with reads only / writes only
template <bool READ, bool WRITE>
__global__ void variant_pattern_rw(const float* __restrict__ eff, int n_shift, int n, int nfeat, double* __restrict__ out) {
  const long long v = blockIdx.y;
  const int f = 2 * (blockIdx.x * blockDim.x + threadIdx.x);
  if (f >= nfeat) return;
  float sx = 0.f, sy = 0.f;
  if (READ)
    for (int j = 0; j < n_shift; ++j) {
      const float2 e2 = *reinterpret_cast<const float2*>(eff + ((long long)j * n + v) * nfeat + f);
      sx += e2.x;
      sy += e2.y;
    }
  double* o = out + v * 10LL * nfeat + f;
  if (WRITE) {
#pragma unroll
    for (int k = 0; k < 10; ++k) store_nt2(o + (long long)k * nfeat, sx + k, sy + k);
  } else if (sx == -1.f) {
    o[0] = sy;
  }
}

// write-only geometries over one 160,160-B region per workgroup of 1024 threads (the output of
// one variant): WAVE_LINEAR = each wave writes 10 consecutive 1-KB pieces (wave w: bytes
// [10 KB w, 10 KB (w+1))); else store c of every thread goes to row c (16 KB apart), as now
template <bool WAVE_LINEAR>
__global__ __launch_bounds__(1024) void write_geom(double* __restrict__ out, int nfeat) {
  const long long v = blockIdx.x;
  const int t = threadIdx.x, w = t >> 6, l = t & 63;
  double* o = out + v * 10LL * nfeat;
  const long long npair = 5LL * nfeat;   // 16-B pieces per region
#pragma unroll
  for (int c = 0; c < 10; ++c) {
    const long long piece = WAVE_LINEAR ? (long long)w * 640 + c * 64 + l : (long long)c * (nfeat / 2) + t;
    if (WAVE_LINEAR ? piece < npair : t < nfeat / 2) store_nt2(o + 2 * piece, (double)c, (double)t);
  }
}

// fill variants: SCATTER = workgroup i writes 4-KB piece (i % 40) * (pieces / 40) + i / 40 (the
// grid's concurrent pieces ~80 MB apart); GRID10 = each thread 10 stores, grid-stride apart
// (10 compact streams)
template <int MODE>
__global__ void fill_geom(double* __restrict__ out, long long n2) {
  const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (MODE == 0) {   // scattered 4-KB pieces
    const long long pieces = n2 / 256, i = blockIdx.x;
    const long long pc = (i % 40) * (pieces / 40) + i / 40;
    if (pc < pieces) store_nt2(out + 2 * (pc * 256 + threadIdx.x), 0.0, 0.0);
  } else {           // 10 grid-stride streams
    const long long per = n2 / 10;
#pragma unroll
    for (int c = 0; c < 10; ++c)
      if (tid < per) store_nt2(out + 2 * (c * per + tid), 0.0, 0.0);
  }
}

// the variant kernel's store geometry (4 x 256 threads per region, 1001 16-B pieces per row, 10
// rows) with a row stride of S pieces (S = 1001: the real [n][10][2002] f64 layout)
__global__ void write_rows_stride(double* __restrict__ out, int S) {
  const long long v = blockIdx.y;
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= 1001) return;
#pragma unroll
  for (int c = 0; c < 10; ++c) store_nt2(out + 2 * ((v * 10 + c) * (long long)S + p), (double)c, (double)p);
}

// variant through LDS with line-aligned stores: a 512-thread workgroup computes one half of a
// variant's feature pairs (pairs [h*P0, ...), P0 = ceil(pairs / 2)) for the 10 decay rows into LDS,
// then writes each half row (16-B aligned, 8,008 B: not a whole number of 128-B lines, and rows
// 16,016 B apart) as 16-B stores whose wave-instructions cover whole aligned lines: only the
// half row's first and last lines are partial (the per-thread layout leaves 2 partial lines in
// every 1-KB wave store, each a read-modify-write at the memory).  Same products and sums.
template <bool MATH>
__global__ __launch_bounds__(512) void variant_lds(const float* __restrict__ eff, const long long* __restrict__ dist,
                                                   const uint8_t* __restrict__ strand_plus,
                                                   const int* __restrict__ shifts, int n_shift, int n, int nfeat,
                                                   const double* __restrict__ lut, int lut_len,
                                                   double* __restrict__ out) {
#pragma clang fp contract(off)
  __shared__ __attribute__((aligned(16))) double stage[10 * 2 * 512];   // [k][pair] x 2 doubles = 80 KB
  __shared__ double wsh[16 * 10];
  const long long v = blockIdx.y;
  const int h = blockIdx.x, t = threadIdx.x;
  const int pairs = nfeat / 2, p0 = (pairs + 1) / 2;
  const int pb = h * p0, np = h ? pairs - p0 : p0;
  if (MATH) variant_weights_lds(dist, strand_plus, shifts, n_shift, v, lut, lut_len, wsh);
  __syncthreads();
  if (t < np) {
    const int f = 2 * (pb + t);
    double a0[10], a1[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) a0[k] = a1[k] = 0.0;
    for (int j = 0; j < n_shift; ++j) {
      const float2 e2 = *reinterpret_cast<const float2*>(eff + ((long long)j * n + v) * nfeat + f);
      const double e0 = (double)e2.x, e1 = (double)e2.y;
#pragma unroll
      for (int k = 0; k < 10; ++k) {
        if (MATH) {
          a0[k] += e0 * wsh[j * 10 + k];
          a1[k] += e1 * wsh[j * 10 + k];
        } else {
          a0[k] += e0;
          a1[k] += e1;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 10; ++k) *reinterpret_cast<f64x2*>(stage + 2 * (k * 512 + t)) = f64x2{a0[k], a1[k]};
  }
  __syncthreads();
#pragma unroll 2
  for (int k = 0; k < 10; ++k) {
    double* row = out + (v * 10 + k) * (long long)nfeat + 2 * pb;       // this half row
    const long long a = (long long)(size_t)row;
    const long long a0 = a & ~127LL;                                     // its first line
    const int lead = (int)((a - a0) >> 4);                               // 16-B slots before it (0..7)
    for (int s = t; s < lead + np; s += 512) {
      const int piece = s - lead;
      if (piece >= 0) {
        const f64x2 x = *reinterpret_cast<const f64x2*>(stage + 2 * (k * 512 + piece));
        store_nt2(row + 2 * piece, x.x, x.y);
      }
    }
  }
}

// variant with per-row LDS staging: a 256-thread workgroup (256 feature pairs) keeps its 10 x 2
// sums in registers, and for each decay row k puts its 4-KB piece of the row through an 8-KB
// double-buffered LDS slot and writes it with wave stores that start on 128-B lines (only the
// piece's first and last line partial, instead of 2 of every wave store's 9 lines)
template <int PB = 256>
__global__ __launch_bounds__(PB) void variant_rowstage(const float* __restrict__ eff, const long long* __restrict__ dist,
                                                        const uint8_t* __restrict__ strand_plus,
                                                        const int* __restrict__ shifts, int n_shift, int n, int nfeat,
                                                        const double* __restrict__ lut, int lut_len,
                                                        double* __restrict__ out) {
#pragma clang fp contract(off)
  __shared__ __attribute__((aligned(16))) double stage[2][2 * PB];
  extern __shared__ double wsh[];
  const long long v = blockIdx.y;
  const int t = threadIdx.x, pb = blockIdx.x * PB;
  const int pairs = nfeat / 2, np = min(PB, pairs - pb);
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
    double* sb = stage[k & 1];
    if (t < np) *reinterpret_cast<f64x2*>(sb + 2 * t) = f64x2{a0[k], a1[k]};
    __syncthreads();
    double* row = out + (v * 10 + k) * (long long)nfeat + 2 * pb;
    const int lead = (int)(((long long)(size_t)row & 127) >> 4);
    for (int s = t; s < lead + np; s += PB) {
      const int piece = s - lead;
      if (piece >= 0) {
        const f64x2 x = *reinterpret_cast<const f64x2*>(sb + 2 * piece);
        store_nt2(row + 2 * piece, x.x, x.y);
      }
    }
  }
}

// variant, one 1024-thread workgroup per variant (thread = feature pair): the 10 sums per thread
// stay in registers; row k goes through a triple-buffered 16-KB LDS slot and is written by a
// sweep over the 128-B lines between row k's first line and row k+1's first line, the line that
// straddles rows k-1 and k taking row k-1's tail from its slot: a variant's 160,160 contiguous
// output bytes are written in whole lines except the two at its ends.  One barrier per row.
__global__ __launch_bounds__(1024) void variant_vrow(const float* __restrict__ eff, const long long* __restrict__ dist,
                                                     const uint8_t* __restrict__ strand_plus,
                                                     const int* __restrict__ shifts, int n_shift, int n, int nfeat,
                                                     const double* __restrict__ lut, int lut_len,
                                                     double* __restrict__ out) {
#pragma clang fp contract(off)
  __shared__ __attribute__((aligned(16))) double stage[3][2 * 1024];
  extern __shared__ double wsh[];
  const long long v = blockIdx.x;
  const int t = threadIdx.x, pairs = nfeat / 2;
  variant_weights_lds(dist, strand_plus, shifts, n_shift, v, lut, lut_len, wsh);
  __syncthreads();
  double a0[10], a1[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) a0[k] = a1[k] = 0.0;
  if (t < pairs) {
    const int f = 2 * t;
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
  double* const vbase = out + v * 10LL * nfeat;            // 16-B aligned; rows of `pairs` pieces
  const long long lead0 = ((long long)(size_t)vbase & 127) >> 4;   // pieces before the first line
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    if (t < pairs) *reinterpret_cast<f64x2*>(stage[k % 3] + 2 * t) = f64x2{a0[k], a1[k]};
    __syncthreads();
    // this sweep: variant pieces [q0, q1) with q the piece index from the variant's start;
    // line-aligned except q0 = 0 (k = 0) and q1 = 10 * pairs (k = 9)
    const long long rk = (long long)k * pairs;
    const long long q0 = k == 0 ? 0 : ((rk + lead0) & ~7LL) - lead0;
    const long long q1 = k == 9 ? 10LL * pairs : ((rk + pairs + lead0) & ~7LL) - lead0;
    for (long long q = q0 + t; q < q1; q += 1024) {
      const long long r = q - rk;                            // < 0: row k-1's tail
      const double* src = r < 0 ? stage[(k + 2) % 3] + 2 * (r + pairs) : stage[k % 3] + 2 * r;
      const f64x2 x = *reinterpret_cast<const f64x2*>(src);
      store_nt2(vbase + 2 * q, x.x, x.y);
    }
  }
}

// sed reduction (shift_reduce_kernel<true, true>) with the 10 decay rows split over KS threads:
// KS x the waves of the 96 x 2002-thread grid (3 waves per SIMD), each loading every shift (the
// repeats hit L2) and summing its 10 / KS rows in the same shift order: bitwise equal
template <int KS>
__global__ void shift_reduce_ks(const float* __restrict__ fwd, const float* __restrict__ rc,
                                const double* __restrict__ weights, int n_shift, int nfeat, double* __restrict__ out) {
#pragma clang fp contract(off)
  extern __shared__ double wsx[];
  for (int i = threadIdx.x; i < 10 * n_shift; i += blockDim.x) wsx[i] = weights[i];
  __syncthreads();
  constexpr int KN = 10 / KS;
  const int ks = blockIdx.z;
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  const long long g = blockIdx.y;
  double* o = out + g * 10LL * (nfeat + 1);
  if (f < KN && ks == 0) {
    for (int k = 0; k < 10; ++k) if (k % KN == f) o[(long long)k * (nfeat + 1)] = 0.0;
  }
  if (f >= nfeat) return;
  double acc[KN];
#pragma unroll
  for (int k = 0; k < KN; ++k) acc[k] = 0.0;
  const float* pf = fwd + g * n_shift * nfeat + f;
  const float* pr = rc + g * n_shift * nfeat + f;
  constexpr int CH = 8;
  for (int s0 = 0; s0 < n_shift; s0 += CH) {
    float a[CH], b[CH];
#pragma unroll
    for (int u = 0; u < CH; ++u)
      if (s0 + u < n_shift) {
        a[u] = pf[(long long)(s0 + u) * nfeat];
        b[u] = pr[(long long)(s0 + u) * nfeat];
      }
#pragma unroll
    for (int u = 0; u < CH; ++u)
      if (s0 + u < n_shift) {
        const double pd = ((double)a[u] + (double)b[u]) / 2.0;
#pragma unroll
        for (int k = 0; k < KN; ++k) acc[k] += wsx[(ks * KN + k) * n_shift + s0 + u] * pd;
      }
  }
#pragma unroll
  for (int k = 0; k < KN; ++k) o[(long long)(ks * KN + k) * (nfeat + 1) + 1 + f] = acc[k];
}

// TSS read pattern with a row stride of `ld` floats (ld = nfeat: the real [G][200][2002] layout,
// rows 8,008 B apart, starting inside 128-B lines; ld = 2048: every row line-aligned)
__global__ void tss_pattern_ld(const float* __restrict__ fwd, const float* __restrict__ rc, int n_shift, int nfeat,
                               int ld, double* __restrict__ out) {
  const int f = 2 * (blockIdx.x * blockDim.x + threadIdx.x);
  const long long g = blockIdx.y;
  if (f >= nfeat) return;
  const long long h2 = ld / 2;
  const float2* pf = reinterpret_cast<const float2*>(fwd + g * n_shift * (long long)ld + f);
  const float2* pr = reinterpret_cast<const float2*>(rc + g * n_shift * (long long)ld + f);
  float sx = 0.f, sy = 0.f;
  constexpr int CH = 8;
  for (int s0 = 0; s0 < n_shift; s0 += CH) {
    float2 x[CH], y[CH];
#pragma unroll
    for (int u = 0; u < CH; ++u)
      if (s0 + u < n_shift) {
        x[u] = pf[(s0 + u) * h2];
        y[u] = pr[(s0 + u) * h2];
      }
#pragma unroll
    for (int u = 0; u < CH; ++u)
      if (s0 + u < n_shift) {
        sx += x[u].x + y[u].x;
        sy += x[u].y + y[u].y;
      }
  }
  double* o = out + g * 10LL * nfeat + f;
#pragma unroll
  for (int k = 0; k < 10; ++k) store_nt2(o + (long long)k * nfeat, sx + k, sy + k);
}
}  // namespace probe

__global__ void hash_fill(float* d, long long n, unsigned seed) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned x = (unsigned)i * 2654435761u ^ seed * 40503u;
  x ^= x >> 15; x *= 2246822519u; x ^= x >> 13; x *= 3266489917u; x ^= x >> 16;
  d[i] = (float)(x >> 8) * (1.0f / 16777216.0f);
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 5;
  const int G = 1000, S = 200, F = 2002, NV = 20000, S9 = 9, NSED = 96;
  float *fwd, *rc, *eff;
  double *w, *out_a, *out_b, *vout_a, *vout_b, *lut;
  CK(hipMalloc(&fwd, (size_t)G * S * F * 4));
  CK(hipMalloc(&rc, (size_t)G * S * F * 4));
  CK(hipMalloc(&eff, (size_t)S9 * NV * F * 4));
  CK(hipMalloc(&w, 10 * S * 8));
  CK(hipMalloc(&out_a, (size_t)G * 10 * F * 8));
  CK(hipMalloc(&out_b, (size_t)G * 10 * F * 8));
  CK(hipMalloc(&vout_a, (size_t)NV * 10 * F * 8));
  CK(hipMalloc(&vout_b, (size_t)NV * 10 * F * 8));
  hash_fill<<<(unsigned)(((long long)G * S * F + 255) / 256), 256>>>(fwd, (long long)G * S * F, 1);
  hash_fill<<<(unsigned)(((long long)G * S * F + 255) / 256), 256>>>(rc, (long long)G * S * F, 2);
  hash_fill<<<(unsigned)(((long long)S9 * NV * F + 255) / 256), 256>>>(eff, (long long)S9 * NV * F, 3);
  {
    std::vector<double> hw(10 * S);
    for (int k = 0; k < 10; ++k)
      for (int s = 0; s < S; ++s) hw[k * S + s] = std::exp(-0.01 * (k % 5 + 1) * std::abs(s - 100)) * ((s < 100) == (k < 5));
    CK(hipMemcpy(w, hw.data(), hw.size() * 8, hipMemcpyHostToDevice));
  }
  long long* dist;
  uint8_t* plus;
  int* shifts;
  CK(hipMalloc(&dist, NV * 8));
  CK(hipMalloc(&plus, NV));
  CK(hipMalloc(&shifts, S9 * 4));
  const int lut_len = 205;
  CK(hipMalloc(&lut, 5 * lut_len * 8));
  {
    std::vector<long long> hd(NV);
    std::vector<uint8_t> hp(NV);
    unsigned x = 12345;
    for (int i = 0; i < NV; ++i) {
      x = x * 1664525u + 1013904223u;
      hd[i] = (long long)(x % 40000) - 20000;
      hp[i] = (x >> 20) & 1;
    }
    const int hs[9] = {0, -200, 200, -400, 400, -600, 600, -800, 800};
    std::vector<double> hl(5 * lut_len);
    for (int k = 0; k < 5; ++k)
      for (int i = 0; i < lut_len; ++i) hl[k * lut_len + i] = std::exp(-(0.01 * (k == 0) + 0.02 * (k == 1) + 0.05 * (k == 2) + 0.1 * (k == 3) + 0.2 * (k == 4)) * i);
    CK(hipMemcpy(dist, hd.data(), NV * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(plus, hp.data(), NV, hipMemcpyHostToDevice));
    CK(hipMemcpy(shifts, hs, 36, hipMemcpyHostToDevice));
    CK(hipMemcpy(lut, hl.data(), hl.size() * 8, hipMemcpyHostToDevice));
  }
  CK(hipDeviceSynchronize());
  const double tss_bytes = 2.0 * G * S * F * 4 + (double)G * 10 * F * 8;
  const double var_bytes = (double)S9 * NV * F * 4 + (double)NV * 10 * F * 8;
  const double sed_bytes = 2.0 * NSED * S * F * 4 + (double)NSED * 10 * (F + 1) * 8;
  const dim3 tgrid((F / 2 + 255) / 256, G), vgrid((F / 2 + 255) / 256, NV);
  struct V { const char* name; double bytes; double* out; double* ref; size_t n; std::function<void()> f; };
  std::vector<V> vs = {
      {"fill_f64_nt (write ceiling)", (double)NV * 10 * F * 8, vout_b, nullptr, 0,
       [&] { probe::fill_nt<<<(unsigned)(((long long)NV * 10 * F / 2 + 255) / 256), 256>>>(vout_b, (long long)NV * 10 * F / 2); }},
      {"tss library", tss_bytes, out_a, nullptr, 0,
       [&] { expecto_tss_reduce(fwd, rc, w, G, S, F, out_a, nullptr); }},
      {"tss pattern ch8 (no math)", tss_bytes, out_b, nullptr, 0,
       [&] { probe::tss_pattern<8><<<tgrid, 256>>>(fwd, rc, S, F, out_b); }},
      {"tss pattern ch16 (no math)", tss_bytes, out_b, nullptr, 0,
       [&] { probe::tss_pattern<16><<<tgrid, 256>>>(fwd, rc, S, F, out_b); }},
      {"tss pattern ld 2002 (real)", tss_bytes, out_b, nullptr, 0,
       [&] { probe::tss_pattern_ld<<<dim3((F / 2 + 1023) / 1024, G), 1024>>>(fwd, rc, S, F, F, out_b); }},
      {"tss pattern ld 2048 (lines)", tss_bytes * 977.0 / 1000.0, out_b, nullptr, 0,
       [&] { probe::tss_pattern_ld<<<dim3((F / 2 + 1023) / 1024, 977), 1024>>>(fwd, rc, S, F, 2048, out_b); }},
      {"tss pipe ch8", tss_bytes, out_b, out_a, (size_t)G * 10 * F,
       [&] { probe::tss_pipe<8><<<tgrid, 256, 10 * S * 8>>>(fwd, rc, w, S, F, out_b); }},
      {"tss pipe ch4", tss_bytes, out_b, out_a, (size_t)G * 10 * F,
       [&] { probe::tss_pipe<4><<<tgrid, 256, 10 * S * 8>>>(fwd, rc, w, S, F, out_b); }},
      {"variant library", var_bytes, vout_a, nullptr, 0,
       [&] { expecto_variant_reduce_lut(eff, dist, plus, shifts, S9, NV, F, lut, lut_len, vout_a, nullptr); }},
      {"variant pattern (no math)", var_bytes, vout_b, nullptr, 0,
       [&] { probe::variant_pattern<<<vgrid, 256>>>(eff, S9, NV, F, vout_b); }},
      {"variant hoist9", var_bytes, vout_b, vout_a, (size_t)NV * 10 * F,
       [&] { probe::variant_hoist<9><<<vgrid, 256, S9 * 10 * 8>>>(eff, dist, plus, shifts, S9, NV, F, lut, lut_len, vout_b); }},
      {"variant two per block", var_bytes, vout_b, vout_a, (size_t)NV * 10 * F,
       [&] {
         probe::variant_two<<<dim3((F / 2 + 255) / 256, NV / 2), 512, 2 * S9 * 10 * 8>>>(eff, dist, plus, shifts, S9, NV, F,
                                                                                           lut, lut_len, vout_b);
       }},
      {"tss bs512", tss_bytes, out_b, out_a, (size_t)G * 10 * F,
       [&] { probe::tss_bs<512><<<dim3((F / 2 + 511) / 512, G), 512, 10 * S * 8>>>(fwd, rc, w, S, F, out_b); }},
      {"tss bs1024", tss_bytes, out_b, out_a, (size_t)G * 10 * F,
       [&] { probe::tss_bs<1024><<<dim3(1, G), 1024, 10 * S * 8>>>(fwd, rc, w, S, F, out_b); }},
      {"tss library (late in the round)", tss_bytes, out_b, nullptr, 0,
       [&] { expecto_tss_reduce(fwd, rc, w, G, S, F, out_b, nullptr); }},
      {"tss bs128", tss_bytes, out_b, out_a, (size_t)G * 10 * F,
       [&] { probe::tss_bs<128><<<dim3((F / 2 + 127) / 128, G), 128, 10 * S * 8>>>(fwd, rc, w, S, F, out_b); }},
      {"variant per-thread stores (r02)", var_bytes, vout_b, vout_a, (size_t)NV * 10 * F,
       [&] { probe::variant_bs<256><<<dim3((F / 2 + 255) / 256, NV), 256, S9 * 10 * 8>>>(eff, dist, plus, shifts, S9, NV, F, lut, lut_len, vout_b); }},
      {"variant bs512", var_bytes, vout_b, vout_a, (size_t)NV * 10 * F,
       [&] { probe::variant_bs<512><<<dim3((F / 2 + 511) / 512, NV), 512, S9 * 10 * 8>>>(eff, dist, plus, shifts, S9, NV, F, lut, lut_len, vout_b); }},
      {"variant bs1024", var_bytes, vout_b, vout_a, (size_t)NV * 10 * F,
       [&] { probe::variant_bs<1024><<<dim3(1, NV), 1024, S9 * 10 * 8>>>(eff, dist, plus, shifts, S9, NV, F, lut, lut_len, vout_b); }},
      {"variant bs128", var_bytes, vout_b, vout_a, (size_t)NV * 10 * F,
       [&] { probe::variant_bs<128><<<dim3((F / 2 + 127) / 128, NV), 128, S9 * 10 * 8>>>(eff, dist, plus, shifts, S9, NV, F, lut, lut_len, vout_b); }},
      {"variant pattern vmajor", var_bytes, vout_b, nullptr, 0,
       [&] { probe::variant_pattern_vmajor<true, true><<<vgrid, 256>>>(eff, S9, NV, F, vout_b); }},
      {"variant pattern reads only", (double)S9 * NV * F * 4, vout_b, nullptr, 0,
       [&] { probe::variant_pattern_rw<true, false><<<vgrid, 256>>>(eff, S9, NV, F, vout_b); }},
      {"variant pattern vmajor reads only", (double)S9 * NV * F * 4, vout_b, nullptr, 0,
       [&] { probe::variant_pattern_vmajor<true, false><<<vgrid, 256>>>(eff, S9, NV, F, vout_b); }},
      {"variant pattern writes only", (double)NV * 10 * F * 8, vout_b, nullptr, 0,
       [&] { probe::variant_pattern_rw<false, true><<<vgrid, 256>>>(eff, S9, NV, F, vout_b); }},
      {"write geom rows (16 KB apart)", (double)NV * 10 * F * 8, vout_b, nullptr, 0,
       [&] { probe::write_geom<false><<<NV, 1024>>>(vout_b, F); }},
      {"write geom wave-linear", (double)NV * 10 * F * 8, vout_b, nullptr, 0,
       [&] { probe::write_geom<true><<<NV, 1024>>>(vout_b, F); }},
      {"fill scattered 4-KB pieces", (double)NV * 10 * F * 8, vout_b, nullptr, 0,
       [&] { probe::fill_geom<0><<<(unsigned)((long long)NV * 10 * F / 2 / 256), 256>>>(vout_b, (long long)NV * 10 * F / 2); }},
      {"fill 10 grid-stride streams", (double)NV * 10 * F * 8, vout_b, nullptr, 0,
       [&] { probe::fill_geom<1><<<(unsigned)(((long long)NV * F / 2 + 255) / 256), 256>>>(vout_b, (long long)NV * 10 * F / 2); }},
      {"rows stride 1001 (real)", (double)NV * 10 * F * 8, vout_b, nullptr, 0,
       [&] { probe::write_rows_stride<<<dim3(4, NV), 256>>>(vout_b, 1001); }},
      {"rows stride 1024 (16 KB)", (double)(NV * 1001LL / 1024) * 10 * F * 8, vout_b, nullptr, 0,
       [&] { probe::write_rows_stride<<<dim3(4, NV * 1001 / 1024), 256>>>(vout_b, 1024); }},
      {"rows stride 1040", (double)(NV * 1001LL / 1040) * 10 * F * 8, vout_b, nullptr, 0,
       [&] { probe::write_rows_stride<<<dim3(4, NV * 1001 / 1040), 256>>>(vout_b, 1040); }},
      {"rows stride 1152", (double)(NV * 1001LL / 1152) * 10 * F * 8, vout_b, nullptr, 0,
       [&] { probe::write_rows_stride<<<dim3(4, NV * 1001 / 1152), 256>>>(vout_b, 1152); }},
      {"rows stride 1536", (double)(NV * 1001LL / 1536) * 10 * F * 8, vout_b, nullptr, 0,
       [&] { probe::write_rows_stride<<<dim3(4, NV * 1001 / 1536), 256>>>(vout_b, 1536); }},
      {"variant rowstage", var_bytes, vout_b, vout_a, (size_t)NV * 10 * F,
       [&] { probe::variant_rowstage<256><<<dim3(4, NV), 256, S9 * 10 * 8>>>(eff, dist, plus, shifts, S9, NV, F, lut, lut_len, vout_b); }},
      {"variant rowstage 512", var_bytes, vout_b, vout_a, (size_t)NV * 10 * F,
       [&] { probe::variant_rowstage<512><<<dim3(2, NV), 512, S9 * 10 * 8>>>(eff, dist, plus, shifts, S9, NV, F, lut, lut_len, vout_b); }},
      {"variant rowstage 128", var_bytes, vout_b, vout_a, (size_t)NV * 10 * F,
       [&] { probe::variant_rowstage<128><<<dim3(8, NV), 128, S9 * 10 * 8>>>(eff, dist, plus, shifts, S9, NV, F, lut, lut_len, vout_b); }},
      {"variant vrow", var_bytes, vout_b, vout_a, (size_t)NV * 10 * F,
       [&] { probe::variant_vrow<<<NV, 1024, S9 * 10 * 8>>>(eff, dist, plus, shifts, S9, NV, F, lut, lut_len, vout_b); }},
      {"variant lds aligned", var_bytes, vout_b, vout_a, (size_t)NV * 10 * F,
       [&] { probe::variant_lds<true><<<dim3(2, NV), 512>>>(eff, dist, plus, shifts, S9, NV, F, lut, lut_len, vout_b); }},
      {"variant lds aligned (no math)", var_bytes, vout_b, nullptr, 0,
       [&] { probe::variant_lds<false><<<dim3(2, NV), 512>>>(eff, dist, plus, shifts, S9, NV, F, lut, lut_len, vout_b); }},
      {"sed library (96)", sed_bytes, out_a, nullptr, 0,
       [&] { expecto_shift_reduce(fwd, rc, w, NSED, S, F, 3, out_a, nullptr); }},
      {"sed k-split 2", sed_bytes, out_b, out_a, (size_t)NSED * 10 * (F + 1),
       [&] { probe::shift_reduce_ks<2><<<dim3((F + 255) / 256, NSED, 2), 256, 10 * S * 8>>>(fwd, rc, w, S, F, out_b); }},
      {"sed k-split 5", sed_bytes, out_b, out_a, (size_t)NSED * 10 * (F + 1),
       [&] { probe::shift_reduce_ks<5><<<dim3((F + 255) / 256, NSED, 5), 256, 10 * S * 8>>>(fwd, rc, w, S, F, out_b); }},
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<float>> t(vs.size());
  for (int r = 0; r < rounds; ++r)
    for (size_t i = 0; i < vs.size(); ++i) {
      vs[i].f();
      CK(hipDeviceSynchronize());
      if (r == 0 && vs[i].ref) {
        std::vector<double> a(vs[i].n), b(vs[i].n);
        CK(hipMemcpy(a.data(), vs[i].ref, vs[i].n * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), vs[i].out, vs[i].n * 8, hipMemcpyDeviceToHost));
        printf("%-30s bitwise equal to the library kernel: %s\n", vs[i].name,
               memcmp(a.data(), b.data(), vs[i].n * 8) == 0 ? "yes" : "NO");
      }
      CK(hipEventRecord(e0));
      for (int k = 0; k < 5; ++k) vs[i].f();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[i].push_back(ms / 5);
    }
  for (size_t i = 0; i < vs.size(); ++i) {
    std::sort(t[i].begin(), t[i].end());
    const float md = t[i][t[i].size() / 2];
    printf("%-30s median %7.3f ms  %6.0f GB/s  %.3f of 8 TB/s  (min %.3f ms)\n", vs[i].name, md,
           vs[i].bytes / (md * 1e-3) / 1e9, vs[i].bytes / (md * 1e-3) / 8e12, t[i][0]);
  }
  return 0;
}
