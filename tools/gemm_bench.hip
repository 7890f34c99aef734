// A/B micro-benchmark of beluga_gemm variants on the conv2 / conv4 / fc1 shapes (gfx950):
// the library's kernels (expecto_amd/csrc/gemm_kernel.h) against the probe-only ones
// (tools/gemm_probes.h) and their timing probes (TM bits, wrong results).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/gemm_bench.hip -o tools/gemm_bench
// Run:   tools/gemm_bench [windows=1000] [rounds=5]
// Interleaved rounds in one process (cdna_hip_programming.md rule 24); outputs of every
// variant are compared bitwise with variant 0 (same per-element K order => identical).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <functional>
#include <random>
#include <string>
#include <vector>

#include "gemm_probes.h"   // the library's kernel header + the probe-only kernels

using namespace expecto;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

struct Variant {
  std::string name;
  int bm;
  std::function<void(const GemmArgs&, unsigned)> launch;
};

template <int L, int EPI, int WM, int MINB>
Variant mk6(const char* name) {
  return {name, 32 * WM, [](const GemmArgs& a, unsigned nblk) {
            beluga_gemm_x6<L, EPI, WM, MINB><<<nblk, 64 * WM>>>(a);
          }};
}

template <int L, int EPI, int TM = 0>
Variant mk6q(const char* name) {
  return {name, X6P_BM, [](const GemmArgs& a, unsigned nblk) { beluga_gemm_x6q<L, EPI, TM><<<nblk, 256>>>(a); }};
}

template <int L, int EPI, int TM = 0, int NS = 3>
Variant mkh3q(const char* name) {
  return {name, X6P_BM, [](const GemmArgs& a, unsigned nblk) { beluga_gemm_h3q<L, EPI, TM, NS><<<nblk, 256>>>(a); }};
}

template <int L, int EPI, int TM = 0, int NSB = 3>
Variant mkc3(const char* name) {
  return {name, X6P_BM, [](const GemmArgs& a, unsigned nblk) { beluga_conv_h3q<L, EPI, TM, NSB><<<nblk, 256>>>(a); }};
}

template <int L, int EPI, int TM = 0>
Variant mkr3(const char* name) {
  return {name, 384, [](const GemmArgs& a, unsigned nblk) { beluga_conv_h3r<L, EPI, TM><<<nblk, 256>>>(a); }};
}

template <int L, int EPI, int TM = 0, int NSB = 3>
Variant mkp3(const char* name) {
  return {name, X6P_BM, [](const GemmArgs& a, unsigned nblk) { beluga_conv_h3p<L, EPI, TM, NSB><<<nblk, 512>>>(a); }};
}

// persistent producer / consumer (grid = 256 workgroups, one per CU, looping over tiles)
template <int L, int EPI, int TM = 0>
Variant mkpp(const char* name) {
  return {name, X6P_BM, [](const GemmArgs& a, unsigned nblk) {
            beluga_conv_h3pp<L, EPI, TM><<<std::min(nblk, 256u), 512>>>(a);
          }};
}

template <int L, int EPI, int TM = 0, int NSB = 4>
Variant mkp32(const char* name) {
  return {name, X6P_BM, [](const GemmArgs& a, unsigned nblk) { beluga_conv_h3p32<L, EPI, TM, NSB><<<nblk, 512>>>(a); }};
}

template <int L, int EPI, int MB, int STG, int TM = 0>
Variant mks3(const char* name) {
  return {name, 64 * MB, [](const GemmArgs& a, unsigned nblk) { beluga_conv_h3s<L, EPI, TM, MB, STG><<<nblk, 512>>>(a); }};
}

template <int L, int EPI, int WM, int MINB, int BK, int PIPE = 0>
Variant mk(const char* name) {
  return {name, 32 * WM, [](const GemmArgs& a, unsigned nblk) {
            beluga_gemm<L, EPI, WM, MINB, BK, PIPE><<<nblk, 64 * WM>>>(a);
          }};
}

static void fill(float* d, size_t n, float lo, float hi, unsigned seed) {
  std::vector<float> h(n);
  std::mt19937 g(seed);
  std::uniform_real_distribution<float> u(lo, hi);
  for (auto& x : h) x = u(g);
  CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
}

__global__ void relu_inplace(float* d, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) d[i] = fmaxf(d[i], 0.f);
}

__global__ void hash_fill(float* d, long long n, float lo, float hi, unsigned seed) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned x = (unsigned)i * 2654435761u ^ seed * 40503u;
  x ^= x >> 15; x *= 2246822519u; x ^= x >> 13; x *= 3266489917u; x ^= x >> 16;
  d[i] = lo + (hi - lo) * (float)(x >> 8) * (1.0f / 16777216.0f);
}

// FC1 shape (M = windows, N = 2003 -> 2080, K = 67840, split-K slabs, partial epilogue):
// the f16x3 planes GEMM and its timing probes (TM 2: no LDS-DMA in the loop).
template <int TM>
void fc1_launch(const GemmArgs& a, unsigned nblk) { beluga_gemm_h3q<7, EPI_PARTIAL, TM, 3><<<nblk, 256>>>(a); }
template <int TM, int NS = 3>
void fc1p_launch(const GemmArgs& a, unsigned nblk) { beluga_fc_h3p<7, EPI_PARTIAL, TM, NS><<<nblk, 512>>>(a); }
template <int TM>
void fc1w_launch(const GemmArgs& a, unsigned nblk) { beluga_fc_h3w<7, EPI_PARTIAL, TM><<<nblk, 512>>>(a); }
template <int TM, int NS = 3, int NB = 10, int NW = 4>
void fc1r_launch(const GemmArgs& a, unsigned nblk) { beluga_fc_h3<7, EPI_PARTIAL, TM, NS, NB, NW><<<nblk, 64 * NW>>>(a); }

int fc1_bench(int nb, int rounds, int splits, bool toe) {
  const int K = 67840, npad = 2080, ldc = 2016;
  // toe: A rows gathered like the segment path's FC1 (a_rows): windows in groups of 100 whose
  // conv6 rows start 25 rows apart (one pool2 phase of one 200-shift segment), so the A rows
  // overlap 4.24-fold and their unique bytes are ~4x fewer than nb x K
  const int grp = 100, grows = 25 * (grp - 1) + 106 + 8;
  const long long xrows = toe ? (long long)(nb + grp - 1) / grp * grows * 640 / K + 2 : nb;
  float *X, *W, *C;
  CK(hipMalloc(&X, (size_t)xrows * K * 4));
  CK(hipMalloc(&W, (size_t)npad * K * 4));
  CK(hipMalloc(&C, (size_t)splits * nb * ldc * 4));
  hash_fill<<<(unsigned)(((long long)xrows * K + 255) / 256), 256>>>(X, (long long)xrows * K, 0.f, 1.f, 1);
  hash_fill<<<(unsigned)(((long long)npad * K + 255) / 256), 256>>>(W, (long long)npad * K, -0.05f, 0.05f, 2);
  int* zs;
  CK(hipMalloc(&zs, std::max<long long>(xrows, npad) * 4));
  CK(hipMemset(zs, 0, std::max<long long>(xrows, npad) * 4));
  _Float16 *Xh, *Bh;
  CK(hipMalloc(&Xh, (size_t)xrows * K * 4));
  CK(hipMalloc(&Bh, (size_t)npad * K * 4));
  split_planes_h2<<<(unsigned)(((long long)xrows * K / 4 + 255) / 256), 256>>>(X, xrows, K, zs, Xh);
  split_planes_h2<<<(unsigned)(((long long)npad * K / 4 + 255) / 256), 256>>>(W, npad, K, zs, Bh);
  long long* arows = nullptr;
  if (toe) {
    std::vector<long long> ar(nb);
    for (int m = 0; m < nb; ++m) ar[m] = ((long long)(m / grp) * grows + 25LL * (m % grp)) * 640;
    CK(hipMalloc(&arows, nb * 8));
    CK(hipMemcpy(arows, ar.data(), nb * 8, hipMemcpyHostToDevice));
  }
  CK(hipDeviceSynchronize());
  GemmArgs a{};
  a.A = (const float*)Xh; a.lda = K; a.M = nb; a.B = W; a.Bp = Bh; a.ldb = K; a.kper = K / splits; a.taps = 1;
  a.n_tiles = npad / GBN; a.m_tiles = (nb + X6P_BM - 1) / X6P_BM; a.m_fastest = 1; a.linear_order = 1;
  a.C = C; a.ldc = ldc; a.n_store = ldc; a.split_stride = (long long)nb * ldc; a.a_rows = arows;
  struct V { const char* name; void (*f)(const GemmArgs&, unsigned); };
  // block orders: m = M tiles fastest in dispatch order, x = N tiles fastest per XCD (XCD-aware
  // remap; the library's order for large M).  Probes (wrong results): hotA / hotB / hotAB = that
  // operand's LDS-DMA always from K stage 0 (L2-hot), noload = no LDS-DMA in the loop.
  // g<k>: grouped order (m_fastest 3) with k M tiles per group
  V vs[] = {{"fcp_m", fc1p_launch<0>}, {"fcp_x", fc1p_launch<0>},
            {"fcp_g3", fc1p_launch<0>}, {"fcp_g4", fc1p_launch<0>}, {"fcp_g5", fc1p_launch<0>},
            {"fcp_g6", fc1p_launch<0>}, {"fcp_g8", fc1p_launch<0>},
            {"fcp_g5_hotB", fc1p_launch<32>},
            {"fcp_x_hotA", fc1p_launch<16>}, {"fcp_x_hotB", fc1p_launch<32>},
            {"fcp_x_hotAB", fc1p_launch<8>}, {"fcp_x_noload", fc1p_launch<2>},
            {"fcw_x", fc1w_launch<0>}, {"fcw_m", fc1w_launch<0>}, {"fcw_g4", fc1w_launch<0>},
            {"fcw_x_hotB", fc1w_launch<32>}, {"fcw_x_noload", fc1w_launch<2>},
            };
  constexpr int NV = sizeof(vs) / sizeof(vs[0]);
  const size_t csz = (size_t)splits * nb * ldc;
  std::vector<float> ref(csz), out(csz);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<float>> t(NV);
  for (int r = 0; r < rounds; ++r)
    for (int v = 0; v < NV; ++v) {
      CK(hipMemset(C, 0, csz * 4));
      a.m_fastest = vs[v].name[4] == 'm' ? 1 : vs[v].name[4] == 'g' ? 3 : 0;
      a.m_group = vs[v].name[4] == 'g' ? vs[v].name[5] - '0' : 0;
      a.linear_order = vs[v].name[4] == 'm';
      a.n_tiles = vs[v].name[2] == 'w' ? 6 : npad / GBN;   // fcw: 336-column tiles
      const unsigned nblk = (unsigned)(a.m_tiles * a.n_tiles * splits);
      vs[v].f(a, nblk);
      if (r == 0 && strstr(vs[v].name, "hot") == nullptr && strstr(vs[v].name, "no") == nullptr) {
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(v == 0 ? ref.data() : out.data(), C, csz * 4, hipMemcpyDeviceToHost));
        if (v > 0) {
          size_t bad = 0;
          for (size_t i = 0; i < csz; ++i) bad += memcmp(&ref[i], &out[i], 4) != 0;
          printf("variant %s vs %s: %zu of %zu partials differ bitwise\n", vs[v].name, vs[0].name, bad, csz);
        }
      }
      CK(hipEventRecord(e0));
      vs[v].f(a, nblk);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[v].push_back(ms);
    }
  const double flops = 2.0 * nb * 2003.0 * K;
  printf("shape fc1 windows %d splits %d %s (M=%d K=%d N=2003)\n", nb, splits, toe ? "toeplitz-rows" : "dense-rows",
         nb, K);
  for (int v = 0; v < NV; ++v) {
    std::sort(t[v].begin(), t[v].end());
    printf("  %-14s median %8.3f ms  %7.1f TFLOP/s fp32-equivalent\n", vs[v].name, t[v][t[v].size() / 2],
           flops / (t[v][t[v].size() / 2] * 1e-3) / 1e12);
  }
  return 0;
}

int main(int argc, char** argv) {
  const int nb = argc > 1 ? atoi(argv[1]) : 1000;
  const int rounds = argc > 2 ? atoi(argv[2]) : 5;
  const char* which = argc > 3 ? argv[3] : "conv2";
  if (!strcmp(which, "fc1") || !strcmp(which, "fc1t"))
    return fc1_bench(nb, rounds, argc > 4 ? atoi(argv[4]) : 8, which[3] == 't');
  struct Shape { const char* name; int cin, cout, s_in, t_valid, s_out, pool; double macs; };
  Shape shapes[] = {{"conv2", 320, 320, 2000, 496, 500, 1, 1986.0 * 320 * 2560},
                    {"conv3", 320, 480, 500, 489, 500, 0, 489.0 * 480 * 2560},
                    {"conv4", 480, 480, 500, 120, 125, 1, 482.0 * 480 * 3840},
                    {"conv5", 480, 640, 120, 113, 113, 0, 113.0 * 640 * 3840},
                    {"conv6", 640, 640, 113, 106, 106, 0, 106.0 * 640 * 5120}};
  Shape sh = shapes[0];
  for (auto& x : shapes) if (!strcmp(x.name, which)) sh = x;
  const long long M = (long long)nb * sh.s_in;
  const size_t xa = (size_t)(M + 64) * sh.cin;
  const int K = 8 * sh.cin;
  const int npad = (sh.cout + GBN - 1) / GBN * GBN;
  float *X, *W, *bias, *C0, *C1;
  CK(hipMalloc(&X, xa * 4));
  CK(hipMalloc(&W, (size_t)npad * K * 4));
  CK(hipMalloc(&bias, npad * 4));
  const size_t csz = (size_t)nb * sh.s_out * sh.cout;
  CK(hipMalloc(&C0, csz * 4));
  CK(hipMalloc(&C1, csz * 6));   // x6q writes bf16 planes (6 B per element)
  // RELU_X=1: activations like a ReLU layer's output (half of them zero), as the conv layers see
  const bool relu_x = getenv("RELU_X") != nullptr;
  fill(X, xa, relu_x ? -1.f : 0.f, 1.f, 1);
  if (relu_x) relu_inplace<<<(unsigned)((xa + 255) / 256), 256>>>(X, (long long)xa);
  fill(W, (size_t)npad * K, -0.05f, 0.05f, 2);
  fill(bias, npad, -0.1f, 0.1f, 3);

  std::vector<Variant> vs;
  __bf16* Bp;
  CK(hipMalloc(&Bp, (size_t)npad * K * 6));
  split_planes<<<(unsigned)(((long long)npad * K / 4 + 255) / 256), 256>>>(W, npad, K, Bp);
  __bf16* Xp;
  CK(hipMalloc(&Xp, xa * 6));
  split_planes<<<(unsigned)((xa / 4 + 255) / 256), 256>>>(X, (long long)(M + 64), sh.cin, Xp);
  // f16x3 operands: unit scales (timing; weights' lo planes go subnormal, numerics are not the point)
  int* zs;
  const long long zrows = std::max<long long>(npad, M + 64);
  CK(hipMalloc(&zs, zrows * 4));
  CK(hipMemset(zs, 0, zrows * 4));
  float* ones;
  CK(hipMalloc(&ones, npad * 4));
  {
    std::vector<float> o(npad, 1.f);
    CK(hipMemcpy(ones, o.data(), npad * 4, hipMemcpyHostToDevice));
  }
  _Float16 *Bh, *Xh;
  CK(hipMalloc(&Bh, (size_t)npad * K * 4));
  CK(hipMalloc(&Xh, xa * 4));
  split_planes_h2<<<(unsigned)(((long long)npad * K / 4 + 255) / 256), 256>>>(W, npad, K, zs, Bh);
  split_planes_h2<<<(unsigned)((xa / 4 + 255) / 256), 256>>>(X, (long long)(M + 64), sh.cin, zs, Xh);
  int* ovf;
  CK(hipMalloc(&ovf, 4));
  CK(hipMemset(ovf, 0, 4));
  CK(hipDeviceSynchronize());
  // variant 0 is the reference for the bitwise comparison: x6 and x6d must agree exactly
  if (sh.pool) {
    vs.push_back(mk6<2, EPI_RELU_POOL4, 4, 1>("x6_wm4_b1"));
    vs.push_back(mk6q<2, EPI_RELU_POOL4>("x6q"));
    vs.push_back(mkc3<2, EPI_RELU_POOL4>("h3c"));
    vs.push_back(mkr3<2, EPI_RELU_POOL4>("h3r"));
    vs.push_back(mks3<2, EPI_RELU_POOL4, 4, 0>("h3s4"));
    vs.push_back(mkp3<2, EPI_RELU_POOL4>("h3p"));
    vs.push_back(mkp3<2, EPI_RELU_POOL4, 256, 4>("h3p4_pf"));

    vs.push_back(mkp3<2, EPI_RELU_POOL4, 256 | 8192, 4>("h3p4_pf_oldepi"));
    vs.push_back(mkr3<2, EPI_RELU_POOL4, 8192>("h3r_oldepi"));
    vs.push_back(mkpp<2, EPI_RELU_POOL4>("h3pp"));
    vs.push_back(mkpp<2, EPI_RELU_POOL4, 2048>("h3pp_noepi"));
    vs.push_back(mkpp<2, EPI_RELU_POOL4, 4096>("h3pp_stagger"));
    vs.push_back(mkp3<2, EPI_RELU_POOL4, 0, 4>("h3p4"));
    vs.push_back(mkp3<2, EPI_RELU_POOL4, 256 | 2048, 4>("h3p4_pf_noepi"));
    vs.push_back(mkp3<2, EPI_RELU_POOL4, 2>("h3p_noglds"));
    vs.push_back(mkp3<2, EPI_RELU_POOL4, 8>("h3p_hotAB"));
    vs.push_back(mks3<2, EPI_RELU_POOL4, 6, 0>("h3s6"));
    vs.push_back(mkr3<2, EPI_RELU_POOL4, 2>("h3r_noglds"));
    vs.push_back(mkr3<2, EPI_RELU_POOL4, 4>("h3r_nobar"));
    vs.push_back(mkr3<2, EPI_RELU_POOL4, 6>("h3r_noglds_nobar"));
    vs.push_back(mkc3<2, EPI_RELU_POOL4, 2>("h3c_noglds"));
  } else {
    vs.push_back(mk6<3, EPI_RELU, 4, 1>("x6_wm4_b1"));
    vs.push_back(mk6q<3, EPI_RELU>("x6q"));
    vs.push_back(mkc3<3, EPI_RELU>("h3c"));
    vs.push_back(mkr3<3, EPI_RELU>("h3r"));
    vs.push_back(mks3<3, EPI_RELU, 4, 0>("h3s4"));
    vs.push_back(mkp3<3, EPI_RELU>("h3p"));
    vs.push_back(mkp3<3, EPI_RELU, 256, 4>("h3p4_pf"));
    vs.push_back(mkp3<3, EPI_RELU, 256 | 8192, 4>("h3p4_pf_oldepi"));
    vs.push_back(mkr3<3, EPI_RELU, 8192>("h3r_oldepi"));
    vs.push_back(mkpp<3, EPI_RELU>("h3pp"));
    vs.push_back(mkpp<3, EPI_RELU, 2048>("h3pp_noepi"));
    vs.push_back(mkpp<3, EPI_RELU, 4096>("h3pp_stagger"));
    vs.push_back(mkp3<3, EPI_RELU, 0, 4>("h3p4"));
    vs.push_back(mkp3<3, EPI_RELU, 256 | 2048, 4>("h3p4_pf_noepi"));
    vs.push_back(mks3<3, EPI_RELU, 6, 0>("h3s6"));
  }
  auto args_for = [&](int bm, float* C) {
    GemmArgs a{};
    a.A = X; a.lda = sh.cin; a.M = M; a.B = W; a.ldb = K; a.kper = K; a.taps = 8;
    a.n_tiles = npad / GBN; a.m_tiles = (M + bm - 1) / bm; a.m_fastest = 0; a.bias = bias;
    a.Bp = Bp;
    a.C = C; a.ldc = sh.cout; a.n_store = sh.cout; a.s_in = sh.s_in; a.t_valid = sh.t_valid; a.s_out = sh.s_out;
    return a;
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<float>> times(vs.size());
  std::vector<float> ref(csz), out(csz), ref_h3;
  const char* only = getenv("VARIANT");   // run just this variant (profiling)
  if (only) {
    std::vector<Variant> keep;
    for (auto& v : vs)
      if ((std::string(",") + only + ",").find("," + v.name + ",") != std::string::npos || v.name == vs[0].name)
        keep.push_back(v);   // VARIANT: comma-separated names
    vs = keep;
    times.assign(vs.size(), {});
  }
  for (int r = 0; r < rounds; ++r) {
    for (size_t v = 0; v < vs.size(); ++v) {
      float* C = v == 0 ? C0 : C1;
      CK(hipMemset(C, 0, v == 0 ? csz * 4 : csz * 6));
      GemmArgs a = args_for(vs[v].bm, C);
      if (vs[v].name.rfind("x6q", 0) == 0) a.A = (const float*)Xp;
      if (vs[v].name.rfind("h3", 0) == 0) {
        a.A = (const float*)Xh;
        a.Bp = Bh;
        a.col_scale = ones;
        a.out_scale = 1.f;
        a.ovf = ovf;
      }
      unsigned nblk = (unsigned)(a.m_tiles * a.n_tiles);
      vs[v].launch(a, nblk);  // warm
      CK(hipEventRecord(e0));
      vs[v].launch(a, nblk);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      times[v].push_back(ms);
      if (r == 0) {
        if (vs[v].name.rfind("h3", 0) == 0) {   // decode fp16 planes
          std::vector<_Float16> pl(csz * 2);
          CK(hipMemcpy(pl.data(), C, csz * 4, hipMemcpyDeviceToHost));
          for (size_t i = 0; i < csz; ++i) {
            const size_t row = i / sh.cout, n = i % sh.cout;
            const size_t k = ((row * (sh.cout / 32) + n / 32) * 2) * 32 + n % 32;
            out[i] = (float)pl[k] + (float)pl[k + 32];
          }
        } else if (vs[v].name.rfind("x6q", 0) == 0) {   // decode planes
          std::vector<uint16_t> pl(csz * 3);
          CK(hipMemcpy(pl.data(), C, csz * 6, hipMemcpyDeviceToHost));
          auto f = [](uint16_t b) { uint32_t u = (uint32_t)b << 16; float x; memcpy(&x, &u, 4); return x; };
          for (size_t i = 0; i < csz; ++i) {
            const size_t row = i / sh.cout, n = i % sh.cout;
            const size_t k = ((row * (sh.cout / 32) + n / 32) * 3) * 32 + n % 32;
            out[i] = f(pl[k]) + (f(pl[k + 32]) + f(pl[k + 64]));
          }
        } else {
          CK(hipMemcpy(v == 0 ? ref.data() : out.data(), C, csz * 4, hipMemcpyDeviceToHost));
        }
        if (vs[v].name == "h3c") ref_h3 = out;
        if (vs[v].name.rfind("h3", 0) == 0 && vs[v].name != "h3c" && !ref_h3.empty() &&
            vs[v].name.find("noglds") == std::string::npos && vs[v].name.find("noepi") == std::string::npos &&
            vs[v].name.find("nosplit") == std::string::npos && vs[v].name.find("nostore") == std::string::npos) {
          size_t bad = 0;
          for (size_t i = 0; i < csz; ++i) bad += memcmp(&ref_h3[i], &out[i], 4) != 0;
          printf("variant %s vs h3c: %zu elements differ bitwise\n", vs[v].name.c_str(), bad);
        }
        if (v > 0) {
          double mx = 0, md = 0;
          size_t bad = 0;
          for (size_t i = 0; i < csz; ++i) {
            mx = std::max(mx, (double)fabsf(ref[i]));
            md = std::max(md, (double)fabsf(ref[i] - out[i]));
            bad += ref[i] != out[i];
          }
          printf("variant %s vs %s: %zu elements differ, max|diff|/max|ref| = %.3g\n", vs[v].name.c_str(),
                 vs[0].name.c_str(), bad, md / mx);
        }
      }
    }
  }
  const double flops = 2.0 * sh.macs * nb;
  printf("shape %s windows %d (M=%lld K=%d N=%d)\n", sh.name, nb, M, K, sh.cout);
  for (size_t v = 0; v < vs.size(); ++v) {
    auto t = times[v];
    std::sort(t.begin(), t.end());
    printf("  %-10s median %8.3f ms  min %8.3f ms  %7.1f TFLOP/s (median)\n", vs[v].name.c_str(), t[t.size() / 2],
           t[0], flops / (t[t.size() / 2] * 1e-3) / 1e12);
  }
  return 0;
}
