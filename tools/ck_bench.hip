// A/B timing of the f16x3 conv3 / conv4 kernels (gfx950): the direct producer / consumer kernel
// (beluga_conv_h3p<.., 256, 4>) against the pair Karatsuba kernel (beluga_conv_h3k) and its timing
// probes (PROBE bits, wrong results).  Random ReLU-like activation planes, unit scales.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/ck_bench.hip -o tools/ck_bench
// Run:   tools/ck_bench [windows=2000] [rounds=5] [conv3|conv4|conv5|conv6]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "ck_karatsuba.h"

using namespace expecto;

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e = (x);                                                                         \
    if (e != hipSuccess) {                                                                      \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));          \
      exit(1);                                                                                  \
    }                                                                                           \
  } while (0)

__device__ __forceinline__ float hash01(unsigned long long i, unsigned seed) {
  unsigned long long x = i * 0x9E3779B97F4A7C15ull + seed;
  x ^= x >> 31;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 29;
  return (float)(x & 0xFFFFFF) / 16777216.f;
}

// planes [rows][C/32][2][32] of values in [lo, hi) (relu: max(v, 0)), scaled by 2^sc
__global__ void fill_planes(_Float16* P, long long rows, int C, unsigned seed, float lo, float hi, int relu, float sc) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * C) return;
  const long long r = i / C;
  const int c = (int)(i - r * C);
  float v = lo + (hi - lo) * hash01(i, seed);
  if (relu) v = fmaxf(v, 0.f);
  v *= sc;
  _Float16 h, l;
  split_h2p(v, h, l);
  _Float16* d = P + (r * (C / 32) + c / 32) * 64 + (c & 31);
  d[0] = h;
  d[32] = l;
}

struct Variant {
  std::string name;
  long long rows_per_tile;
  std::function<void(const GemmArgs&, unsigned)> launch;
};

template <int L, int PROBE>
Variant mkk(const char* name) {
  return {name, 2 * CK_PAIRS, [](const GemmArgs& a, unsigned nblk) { beluga_conv_h3k<L, EPI_RELU, PROBE><<<nblk, 512>>>(a); }};
}

template <int L, int TM = 256>
Variant mkp(const char* name) {
  return {name, 256, [](const GemmArgs& a, unsigned nblk) { beluga_conv_h3p<L, EPI_RELU, TM, 4><<<nblk, 512>>>(a); }};
}

template <int L>
Variant mkr(const char* name) {
  return {name, 384, [](const GemmArgs& a, unsigned nblk) { beluga_conv_h3r<L, EPI_RELU, 0><<<nblk, 256>>>(a); }};
}

// stamp build: per-wave cycle sums (gemm_kernel.h H3P_STAMP), summarised as shares of the loop
static void stamp_report(const unsigned long long* d, long long nblk, int nk) {
  double cl = 0, cb = 0, ce = 0, pl = 0, pb = 0, pv = 0;
  for (long long b = 0; b < nblk; ++b)
    for (int w = 0; w < 8; ++w) {
      const unsigned long long* e = d + (b * 8 + w) * 4;
      if (w < 4) { cl += e[0]; cb += e[1]; ce += e[3]; }
      else { pl += e[0]; pb += e[1]; pv += e[2]; }
    }
  const double nw = 4.0 * nblk;
  printf("stamp: %d stages per tile; consumer loop %.0f cycles/tile (%.0f per stage; 120 MFMAs = 1920 at 16 each), "
         "barrier wait %.3f of the loop, epilogue %.0f cycles (%.3f of loop)\n",
         nk, cl / nw, cl / nw / nk, cb / cl, ce / nw, ce / cl);
  printf("stamp: producer loop %.0f cycles/tile, vmcnt wait %.3f, barrier wait %.3f of its loop\n", pl / nw, pv / pl, pb / pl);
}

int main(int argc, char** argv) {
  const int nb = argc > 1 ? atoi(argv[1]) : 2000;
  const int rounds = argc > 2 ? atoi(argv[2]) : 5;
  const char* layer = argc > 3 ? argv[3] : "conv3";
  const bool c4 = !strcmp(layer, "conv4"), c5 = !strcmp(layer, "conv5"), c6 = !strcmp(layer, "conv6");
  // conv5 / conv6: the per-window shapes (Q4 120 rows -> 113; conv5 113 rows -> 106)
  const int cin = c6 ? 640 : (c4 || c5) ? 480 : 320, cout = (c5 || c6) ? 640 : 480;
  const int s_in = c6 ? 113 : c5 ? 120 : c4 ? 492 : 496, t_valid = c6 ? 106 : c5 ? 113 : c4 ? 482 : 489;
  const int s_out = c6 ? 106 : c5 ? 113 : c4 ? 482 : 492;
  const long long M = (long long)nb * s_in;
  const int npad = (cout + GBN - 1) / GBN * GBN;
  _Float16 *X, *Bd, *Bk;
  float *bias, *cs, *C;
  int* ovf;
  CK(hipMalloc(&X, (size_t)(M + 64) * cin * 4));
  CK(hipMalloc(&Bd, (size_t)npad * 8 * cin * 4));
  CK(hipMalloc(&Bk, (size_t)npad * 13 * cin * 4));
  CK(hipMalloc(&bias, npad * 4));
  CK(hipMalloc(&cs, npad * 4));
  CK(hipMalloc(&C, (size_t)nb * s_out * cout * 4));
  CK(hipMalloc(&ovf, 4));
  const long long nx = (M + 64) * cin, nd = (long long)npad * 8 * cin, nk = (long long)npad * 13 * cin;
  fill_planes<<<(unsigned)((nx + 255) / 256), 256>>>(X, M + 64, cin, 1, -1.f, 1.f, 1, 1024.f);
  fill_planes<<<(unsigned)((nd + 255) / 256), 256>>>(Bd, npad, 8 * cin, 2, -0.05f, 0.05f, 0, 1024.f);
  fill_planes<<<(unsigned)((nk + 255) / 256), 256>>>(Bk, npad, 13 * cin, 3, -0.05f, 0.05f, 0, 1024.f);
  {
    std::vector<float> b(npad, 0.01f), one(npad, 1.f / (1024.f * 1024.f));
    CK(hipMemcpy(bias, b.data(), npad * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(cs, one.data(), npad * 4, hipMemcpyHostToDevice));
  }
  CK(hipMemset(ovf, 0, 4));
  CK(hipDeviceSynchronize());
  std::vector<Variant> vs;
  if (c5) {
    vs.push_back(mkp<5>("direct_h3p"));
    vs.push_back(mkp<5, 256 | H3P_STAMP>("direct_stamp"));
    vs.push_back(mkp<5, 256 | 2048>("direct_noepi"));
    vs.push_back(mkp<5, 256 | 64>("direct_ea"));
    vs.push_back(mkp<5, 256 | 64 | H3P_STAMP>("direct_stamp_ea"));
    vs.push_back(mkp<5, 256 | 512>("direct_nostore"));
    vs.push_back(mkp<5, 256 | 2>("direct_noload"));
    vs.push_back(mkp<5, 256 | H3P_STAMP | 8>("direct_stamp_hotAB"));
    vs.push_back(mkp<5, 256 | H3P_STAMP | 2>("direct_stamp_noload"));
    vs.push_back(mkr<5>("h3r_384"));
    vs.push_back(mkp<5, 256 | 8>("direct_hotAB"));
  } else if (c6) {
    vs.push_back(mkp<6>("direct_h3p"));
    vs.push_back(mkp<6, 256 | H3P_STAMP>("direct_stamp"));
    vs.push_back(mkp<6, 256 | 2048>("direct_noepi"));
    vs.push_back(mkp<6, 256 | 64>("direct_ea"));
    vs.push_back(mkp<6, 256 | 64 | H3P_STAMP>("direct_stamp_ea"));
    vs.push_back(mkp<6, 256 | 512>("direct_nostore"));
    vs.push_back(mkp<6, 256 | 2>("direct_noload"));
    vs.push_back(mkp<6, 256 | H3P_STAMP | 8>("direct_stamp_hotAB"));
    vs.push_back(mkp<6, 256 | H3P_STAMP | 2>("direct_stamp_noload"));
    vs.push_back(mkr<6>("h3r_384"));
    vs.push_back(mkp<6, 256 | 8>("direct_hotAB"));
  } else if (c4) {
    vs.push_back(mkp<4>("direct_h3p"));
    vs.push_back(mkp<4, 256 | H3P_STAMP>("direct_stamp"));
    vs.push_back(mkp<4, 256 | 2048>("direct_noepi"));
    vs.push_back(mkp<4, 256 | 64>("direct_ea"));
    vs.push_back(mkp<4, 256 | 64 | H3P_STAMP>("direct_stamp_ea"));
    vs.push_back(mkp<4, 256 | 512>("direct_nostore"));
    vs.push_back(mkp<4, 256 | 2>("direct_noload"));
    vs.push_back(mkp<4, 256 | H3P_STAMP | 8>("direct_stamp_hotAB"));
    vs.push_back(mkp<4, 256 | H3P_STAMP | 2>("direct_stamp_noload"));
    vs.push_back(mkr<4>("h3r_384"));
    vs.push_back(mkp<4, 256 | 8>("direct_hotAB"));
    vs.push_back(mkp<4, 256 | 16>("direct_hotA"));
    vs.push_back(mkp<4, 256 | 32>("direct_hotB"));
    vs.push_back(mkk<4, 0>("karatsuba"));
    vs.push_back(mkk<4, 1>("k_no_s"));
    vs.push_back(mkk<4, 2>("k_no_barrier"));
    vs.push_back(mkk<4, 4>("k_no_loads"));
    vs.push_back(mkk<4, 7>("k_mfma_only"));
    vs.push_back(mkk<4, 8>("k_s_loads_only"));
    vs.push_back(mkk<4, 16>("k_s_valu_only"));
  } else {
    vs.push_back(mkp<3>("direct_h3p"));
    vs.push_back(mkp<3, 256 | H3P_STAMP>("direct_stamp"));
    vs.push_back(mkp<3, 256 | 2048>("direct_noepi"));
    vs.push_back(mkp<3, 256 | 64>("direct_ea"));
    vs.push_back(mkp<3, 256 | 64 | H3P_STAMP>("direct_stamp_ea"));
    vs.push_back(mkp<3, 256 | 512>("direct_nostore"));
    vs.push_back(mkp<3, 256 | 2>("direct_noload"));
    vs.push_back(mkp<3, 256 | H3P_STAMP | 8>("direct_stamp_hotAB"));
    vs.push_back(mkp<3, 256 | H3P_STAMP | 2>("direct_stamp_noload"));
    vs.push_back(mkr<3>("h3r_384"));
    vs.push_back(mkp<3, 256 | 8>("direct_hotAB"));
    vs.push_back(mkp<3, 256 | 16>("direct_hotA"));
    vs.push_back(mkp<3, 256 | 32>("direct_hotB"));
    vs.push_back(mkk<3, 0>("karatsuba"));
    vs.push_back(mkk<3, 1>("k_no_s"));
    vs.push_back(mkk<3, 2>("k_no_barrier"));
    vs.push_back(mkk<3, 4>("k_no_loads"));
    vs.push_back(mkk<3, 7>("k_mfma_only"));
    vs.push_back(mkk<3, 8>("k_s_loads_only"));
    vs.push_back(mkk<3, 16>("k_s_valu_only"));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // ONLY=<name>: that variant alone (counter passes under rocprofv3 --pmc)
  if (const char* only = getenv("ONLY")) {
    std::vector<Variant> keep;
    for (auto& v : vs)
      if (v.name == only) keep.push_back(v);
    vs = keep;
  }
  std::vector<double> best(vs.size(), 1e30), sum(vs.size(), 0.0);
  for (int r = 0; r < rounds; ++r)
    for (size_t v = 0; v < vs.size(); ++v) {
      const bool kar = vs[v].name.rfind("k", 0) == 0;   // karatsuba, k_*
      GemmArgs a{};
      a.A = reinterpret_cast<const float*>(X);
      a.lda = cin;
      a.M = M;
      a.Bp = kar ? (const void*)Bk : (const void*)Bd;
      a.ldb = (kar ? 13 : 8) * cin;
      a.kper = (int)a.ldb;
      a.taps = 8;
      a.n_tiles = npad / GBN;
      a.m_tiles = kar ? (M / 2 + CK_PAIRS - 1) / CK_PAIRS : (M + vs[v].rows_per_tile - 1) / vs[v].rows_per_tile;
      a.bias = bias;
      a.col_scale = cs;
      a.out_scale = 1.f;
      a.ovf = ovf;
      a.C = C;
      a.ldc = cout;
      a.n_store = cout;
      a.s_in = s_in;
      a.t_valid = t_valid;
      a.s_out = s_out;
      const unsigned nblk = (unsigned)(a.m_tiles * a.n_tiles);
      const bool stamp = vs[v].name.rfind("direct_stamp", 0) == 0;
      if (stamp) {
        CK(hipMalloc(&a.stamps, (size_t)nblk * 8 * 4 * 8));
        CK(hipMemset(a.stamps, 0, (size_t)nblk * 8 * 4 * 8));
      }
      vs[v].launch(a, nblk);   // warm
      CK(hipEventRecord(e0));
      for (int i = 0; i < 3; ++i) vs[v].launch(a, nblk);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= 3;
      if (stamp) {
        std::vector<unsigned long long> h((size_t)nblk * 8 * 4);
        CK(hipMemcpy(h.data(), a.stamps, h.size() * 8, hipMemcpyDeviceToHost));
        if (r == rounds - 1) {
          printf("%s ", vs[v].name.c_str());
          stamp_report(h.data(), nblk, (int)(cin / 32 * 8));
        }
        CK(hipFree(a.stamps));
      }
      best[v] = std::min(best[v], (double)ms);
      sum[v] += ms;
    }
  // same bits: the early-read variant against the direct kernel (one launch each, output compared)
  {
    int iref = -1, iea = -1;
    for (size_t v = 0; v < vs.size(); ++v) {
      if (vs[v].name == "direct_h3p") iref = (int)v;
      if (vs[v].name == "direct_ea") iea = (int)v;
    }
    if (iref >= 0 && iea >= 0) {
      const size_t cb = (size_t)nb * s_out * cout * 4;
      std::vector<char> h0(cb), h1(cb);
      for (int k = 0; k < 2; ++k) {
        GemmArgs a{};
        a.A = reinterpret_cast<const float*>(X);
        a.lda = cin;
        a.M = M;
        a.Bp = Bd;
        a.ldb = 8 * cin;
        a.kper = (int)a.ldb;
        a.taps = 8;
        a.n_tiles = npad / GBN;
        a.m_tiles = (M + 255) / 256;
        a.bias = bias;
        a.col_scale = cs;
        a.out_scale = 1.f;
        a.ovf = ovf;
        a.C = C;
        a.ldc = cout;
        a.n_store = cout;
        a.s_in = s_in;
        a.t_valid = t_valid;
        a.s_out = s_out;
        CK(hipMemset(C, 0, cb));
        vs[k ? iea : iref].launch(a, (unsigned)(a.m_tiles * a.n_tiles));
        CK(hipMemcpy(k ? h1.data() : h0.data(), C, cb, hipMemcpyDeviceToHost));
      }
      printf("direct_ea output bitwise equal to direct_h3p: %s\n", memcmp(h0.data(), h1.data(), cb) ? "NO" : "yes");
    }
  }
  const double alg = 2.0 * M * cout * 8.0 * cin;   // direct fp32-equivalent flops
  printf("%s, %d windows, M %lld rows\n", c4 ? "conv4 (unpooled)" : layer, nb, M);
  for (size_t v = 0; v < vs.size(); ++v)
    printf("%-14s mean %.3f ms  best %.3f ms  dense-equivalent %.1f TF/s  (%.3fx direct)\n", vs[v].name.c_str(),
           sum[v] / rounds, best[v], alg / (sum[v] / rounds * 1e-3) / 1e12, vs.empty() ? 0.0 : sum[0] / sum[v]);
  return 0;
}
