// Energy-per-MAC probe for DESIGN 8 item 5: sustained fp16 MFMA throughput of the 16x16x32 form
// the GEMM kernels issue vs the 32x32x16 form (half the operand elements per MAC), register
// operands only, every SIMD busy (4 waves per SIMD), ~1.5 s per launch so the board reaches its
// power-limited clock.  If the chip holds a higher clock on the 32x32x16 loop, the operand
// delivery is a measurable share of the power the headline is bound by.
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_power_probe.hip -o tools/mfma_power_probe
//   ./tools/mfma_power_probe [iters] [zero_frac]   -> one JSON line per (form, launch)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

// 8 independent 16x16x32 chains (8 x 16 cycles covers the MFMA dependency latency).
// ORD 0: A and B operands both change from one MFMA to the next (round 2's probe); ORD 1: the
// B operand stays for 4 consecutive MFMAs (A changes), the order a GEMM unit gets when its
// 3 split products are issued product-major over the 4 row blocks instead of row-block-major.
template <int ORD>
__global__ __launch_bounds__(256) void mfma16(const halfx8* __restrict__ in, int iters, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  halfx8 a[4], b[4];   // 4 operand pairs rotating over the chains: the datapath sees changing data
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    a[q] = in[q * 64 + lane];
    b[q] = in[(4 + q) * 64 + lane];
  }
  floatx4 acc[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) acc[c] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < 8; ++c)
      acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[c & 3], ORD == 0 ? b[(c + 1) & 3] : b[c >> 2], acc[c], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < 8; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// 4 independent 32x32x16 chains: the same MACs per iteration as mfma16 (4 x 32768 = 8 x 16384 flops)
__global__ __launch_bounds__(256) void mfma32(const halfx8* __restrict__ in, int iters, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  halfx8 a[4], b[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    a[q] = in[q * 64 + lane];
    b[q] = in[(4 + q) * 64 + lane];
  }
  floatx16 acc[4];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[c & 3], b[(c + 1) & 3], acc[c], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r) s += acc[c][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 3000000;
  // optional: fraction of operand elements set to zero (ReLU-like sparsity of real activations)
  const double zero_frac = argc > 2 ? atof(argv[2]) : 0.0;
  int ncu = 0;
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const int blocks = ncu * 4;   // 4 workgroups x 4 waves per CU = 4 waves per SIMD
  halfx8* in;
  float* out;
  CHECK(hipMalloc(&in, 512 * sizeof(halfx8)));
  CHECK(hipMalloc(&out, (size_t)blocks * 256 * sizeof(float)));
  static halfx8 h[512];
  unsigned r = 12345;
  for (int i = 0; i < 512; ++i)
    for (int e = 0; e < 8; ++e) {
      r = r * 1664525u + 1013904223u;
      h[i][e] = (_Float16)(((int)(r >> 9) % 2001 - 1000) * 1e-6f);   // random-looking, no overflow
      r = r * 1664525u + 1013904223u;
      if ((r >> 8) % 1000 < (unsigned)(zero_frac * 1000)) h[i][e] = (_Float16)0.f;
    }
  CHECK(hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const double flops = (double)blocks * 4 /*waves*/ * iters * 8.0 * 16384.0;
  for (int rep = 0; rep < 3; ++rep) {
    for (int form = 0; form < 3; ++form) {
      CHECK(hipEventRecord(e0, 0));
      if (form == 0)
        mfma16<0><<<blocks, 256>>>(in, iters, out);
      else if (form == 1)
        mfma32<<<blocks, 256>>>(in, iters, out);
      else
        mfma16<1><<<blocks, 256>>>(in, iters, out);
      CHECK(hipGetLastError());
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float ms = 0.f;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      const double tf = flops / (ms * 1e-3) / 1e12;
      printf("{\"form\": \"%s\", \"zero_frac\": %.2f, \"rep\": %d, \"ms\": %.2f, \"tflops\": %.1f, "
             "\"frac_of_2516.6\": %.4f, \"clock_ghz_if_busy\": %.3f}\n",
             form == 0 ? "16x16x32_f16" : form == 1 ? "32x32x16_f16" : "16x16x32_f16_stableB", zero_frac, rep, ms,
             tf, tf / 2516.5824,
             2.4 * tf / 2516.5824);
      fflush(stdout);
    }
  }
  CHECK(hipFree(in));
  CHECK(hipFree(out));
  return 0;
}
