// conv3 / conv4 as pair Karatsuba GEMMs (f16x3): built and measured in round 5 (bitwise across the
// library's paths, -18.75 % MFMAs, 4-5 % SLOWER than the direct beluga_conv_h3p: DESIGN.md §7), then
// moved out of the library (round 6) and kept here as a tools/ck_bench probe with its timing variants.
#pragma once
#include "../expecto_amd/csrc/gemm_kernel.h"

namespace expecto {

// ---- f16x3 conv GEMM as a 2 x 2 Toeplitz Karatsuba (conv3 / conv4) --------------------------
// The 8-tap correlation y[t] = sum_j w_j x[t+j] (Beluga.py:29-32, one output channel, all input
// channels) over pair blocks X_q = (x[2q], x[2q+1]): the output pair (y[2p], y[2p+1]) is
// sum_{i=0..4} T_i X_{p+i} with the Toeplitz T_i = [[w_2i, w_2i+1], [w_2i-1, w_2i]] (w_-1 = w_8 = 0),
// and a Toeplitz 2 x 2 times a vector takes 3 products, [[a, b], [c, a]] (u, v) =
// (a (u+v) + (b-a) v, a (u+v) + (c-a) u):
//   y[2p]   = S[p] + V[p]        S[p] = sum_{i<4} w_2i s[p+i],              s[q] = x[2q] + x[2q+1]
//   y[2p+1] = S[p] + U[p]        V[p] = sum_{i<4} (w_2i+1 - w_2i) x[2(p+i)+1]
//                                U[p] = sum_{i<5} (w_2i-1 - w_2i) x[2(p+i)]
// 13 (chunk, tap) K blocks per output pair instead of 16: -18.75 % of the MFMAs.  Operands stay in
// the layers' activation layout (no producer changes): U and V read the even / odd rows of the
// stored planes by LDS-DMA, and the producer waves form s (hi + lo of both rows, one fp32 add,
// plain split) into the slab.  Register budget as the direct kernel: the shared S is accumulated
// first, over every chunk, into acc_e and copied into acc_o; then U goes into acc_o and V into
// acc_e.  Tile 128 pairs (256 output rows) x 160 columns: 4 consumer waves of 32 pairs x 160
// (acc_e + acc_o = 160 accumulators), 4 producer waves (LDS-DMA, the s slabs).  Pairs are rows
// (2p, 2p+1) of the flattened M index: s_in must be even (pairs never straddle two windows), and
// two launches give the same bits for the same window only with the same row parity
// (forward_segments: conv_karatsuba_ok).  B = the Karatsuba weight planes in step order: S
// (chunk, tap 0..3), U (chunk, tap 0..4), V (chunk, tap 0..3), ldb = 13 * Cin.
constexpr int CK_PAIRS = 128;                          // output pairs per tile
constexpr int CK_AROWS = 144;                          // slab rows: 128 + 4 needed, 9 groups of 16
constexpr int CK_APLANE = CK_AROWS * 64;               // 9,216 B
constexpr int CK_ASLAB = 2 * CK_APLANE;                // 18,432 B
constexpr int CK_NSB = 4;
constexpr int CK_LDS = 2 * CK_ASLAB + CK_NSB * H3C_BSTAGE;   // 118,784 B
constexpr int CK_SITEMS = (CK_PAIRS + 4) * 4;          // s slab: 132 rows x 4 16-B pieces (per plane)
static_assert(4 * H3E_WAVE <= CK_LDS, "epilogue staging exceeds the kernel's LDS");

// Epilogues of the pair layout: acc_e[mb][nb][j] is output row 2 * (16 mb + 4 fq + j) of the wave,
// acc_o the row after it.  Same values, splits and stores as epilogue_relu_h2_lds /
// epilogue_pool_h2_lds (the LDS staging rows are the output rows).
template <bool BATCH = true>
__device__ __forceinline__ void epilogue_relu_h2_pairs(const GemmArgs& p, const floatx4v (&acc_e)[2][10],
                                                       const floatx4v (&acc_o)[2][10], long long mw, int n0,
                                                       int lane, char* lds) {
  const int fr = lane & 15, fq = lane >> 4;
  const long long w0 = mw / p.s_in;
  const int t0 = (int)(mw - w0 * p.s_in);
  float csov[10], bov[10];
  epi_factors<BATCH>(p, n0, fr, csov, bov);
  float vmax = 0.f;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
#pragma unroll
    for (int nb = 0; nb < 10; ++nb) {
      const float cso = csov[nb], bo = bov[nb];
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const float x = fmaxf(fmaf(e ? acc_o[half][nb][j] : acc_e[half][nb][j], cso, bo), 0.f);
          vmax = fmaxf(vmax, x);
          _Float16 hi, lo;
          split_h2p(x, hi, lo);
          char* d = lds + (8 * fq + 2 * j + e) * H3E_ROW + (nb >> 1) * 128 + ((nb & 1) * 16 + fr) * 2;
          *(_Float16*)d = hi;
          *(_Float16*)(d + 64) = lo;
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const long long ldb = p.ldc >> 5;
#pragma unroll 4
    for (int i = 0; i < 20; ++i) {
      const int k = i * 64 + lane, row = k / 40, ch = k - row * 40;
      const long long m = mw + half * 32 + row;
      if (m < p.M) {
        long long w;
        int tpos;
        row_wt(w0, t0, half * 32 + row, p.s_in, w, tpos);
        if (tpos < p.t_valid && n0 + (ch >> 3) * 32 < p.n_store) {
          const long long orow = w * p.s_out + tpos;
          char* g = (char*)p.C + (orow * ldb + (n0 >> 5)) * 128 + ch * 16;
          *(floatx4v*)g = *(const floatx4v*)(lds + row * H3E_ROW + ch * 16);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if (!(vmax < 65504.f)) *p.ovf = 1;   // overflow: the call is recomputed (bf16x6)
}

template <bool CANON, bool BATCH = true>
__device__ __forceinline__ void epilogue_pool_h2_pairs(const GemmArgs& p, const floatx4v (&acc_e)[2][10],
                                                       const floatx4v (&acc_o)[2][10], long long mw, int n0,
                                                       int lane, char* lds) {
  const int fr = lane & 15, fq = lane >> 4;
  float csov[10], bov[10];
  epi_factors<BATCH>(p, n0, fr, csov, bov);
  float vmax = 0.f;
#pragma unroll
  for (int nb = 0; nb < 10; ++nb) {
    const float cso = csov[nb], bo = bov[nb];
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {   // pool group = output rows 4g..4g+3 = pairs 2g, 2g+1
        const float mx = fmaxf(fmaxf(acc_e[mb][nb][2 * jj], acc_o[mb][nb][2 * jj]),
                               fmaxf(acc_e[mb][nb][2 * jj + 1], acc_o[mb][nb][2 * jj + 1]));
        const float x = fmaxf(fmaf(mx, cso, bo), 0.f);
        vmax = fmaxf(vmax, x);
        _Float16 hi, lo;
        if constexpr (CANON)
          split_h2(x, hi, lo);
        else
          split_h2p(x, hi, lo);
        char* d = lds + (8 * mb + 2 * fq + jj) * H3E_ROW + (nb >> 1) * 128 + ((nb & 1) * 16 + fr) * 2;
        *(_Float16*)d = hi;
        *(_Float16*)(d + 64) = lo;
      }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const long long ldb = p.ldc >> 5;
  const long long w0 = mw / p.s_in;
  const int t0 = (int)(mw - w0 * p.s_in);
#pragma unroll 5
  for (int i = 0; i < (16 * 40) / 64; ++i) {
    const int k = i * 64 + lane, row = k / 40, ch = k - row * 40;
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

// Steps of the Karatsuba conv: phase 0 = S (4 taps per chunk, s slabs), 1 = U (5 taps, even rows),
// 2 = V (4 taps, odd rows); slab g = phase * nchunk + chunk.
__device__ __forceinline__ int ck_taps(int phase) { return phase == 1 ? 5 : 4; }

// PROBE (tools/ck_bench timing probes, wrong results; the library launches 0): 1 = no s slabs
// (producers skip the pair sums), 2 = no per-step barriers, 4 = no LDS-DMA / loads in the K loop,
// 8 = s loads without the sums, 16 = s sums without the loads.
template <int LAYER, int EPI, int PROBE = 0>
__global__ __launch_bounds__(512, 1) void beluga_conv_h3k(GemmArgs p) {
  __shared__ __attribute__((aligned(1024))) char smem[CK_LDS];
  constexpr int ROW_KB = 128;
  constexpr int NAP = 5;                              // DMA slab pieces per producer (18 over 4, repeats)
  const unsigned nblk = gridDim.x, bid = blockIdx.x;
  const unsigned xcd = bid & 7u, q = nblk >> 3, rr = nblk & 7u;
  const unsigned lin = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  const int nt = (int)(lin % (unsigned)p.n_tiles);
  const long long mt = (long long)(lin / (unsigned)p.n_tiles) % p.m_tiles;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const long long p0 = mt * CK_PAIRS;                 // first pair of the tile (rows 2 p0 ..)
  const int n0 = nt * GBN;
  const int kb_total = (int)(p.ldb / GBK);            // 13 * nchunk
  const long long lda_kb = p.lda / GBK;
  const int nchunk = (int)lda_kb;
  const int nslab = 3 * nchunk;
  auto swz = [](int r) { return conv_swz<0>(r); };
  char* const aslab = smem;
  char* const bring = smem + 2 * CK_ASLAB;
  const long long row_bytes = lda_kb * ROW_KB;

  if (wave >= 4) {
    // ---------------- producers: LDS-DMA (B ring, even / odd row slabs) and the s slabs ----------------
    const int pw = wave - 4;
    const char* Ab = (const char*)p.A + 2 * p0 * row_bytes;
    const long long last_row = p.M - 1 + 7;             // rows past it feed only rows past M
    unsigned aoff[2][NAP];                               // [0] even rows (U), [1] odd rows (V)
#pragma unroll
    for (int i = 0; i < NAP; ++i) {
      const int P = min(pw + 4 * i, 2 * (CK_AROWS / 16) - 1), gq = P >> 1, pl = P & 1;
      const int r = 16 * gq + (lane >> 2);
      const int c = (lane & 3) ^ swz(r);
#pragma unroll
      for (int par = 0; par < 2; ++par) {
        const long long m = min(2 * p0 + 2 * r + par, last_row);
        aoff[par][i] = (unsigned)((m - 2 * p0) * row_bytes + pl * 64 + 16 * c);
      }
    }
    // s slab items (row r, 16-B piece pc of each plane): 3 per lane, items >= CK_SITEMS idle
    unsigned soff_e[3], soff_o[3];
    int sdst[3];
    bool sact[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int it = i * 256 + pw * 64 + lane;
      sact[i] = it < CK_SITEMS;
      const int itc = min(it, CK_SITEMS - 1), r = itc >> 2, pc = itc & 3;
      const long long me = min(2 * p0 + 2 * r, last_row), mo = min(2 * p0 + 2 * r + 1, last_row);
      soff_e[i] = (unsigned)((me - 2 * p0) * row_bytes + 16 * pc);
      soff_o[i] = (unsigned)((mo - 2 * p0) * row_bytes + 16 * pc);
      sdst[i] = r * 64 + 16 * (pc ^ swz(r));
    }
    const char* Bb = (const char*)p.Bp + (long long)n0 * kb_total * ROW_KB;
    unsigned boff[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const int gq = pw + 4 * j;
      const int pl = gq / 10, r = 16 * (gq % 10) + (lane >> 2);
      const int c = (lane & 3) ^ swz(r);
      boff[j] = (unsigned)((long long)r * kb_total * ROW_KB + pl * 64 + 16 * c);
    }
    const __amdgpu_buffer_rsrc_t arsrc = __builtin_amdgcn_make_buffer_rsrc((void*)Ab, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t brsrc = __builtin_amdgcn_make_buffer_rsrc((void*)Bb, (short)0, 0x7fffffff, 0x00020000);
    auto issue_b = [&](int s, int slot) {
      char* base = bring + slot * H3C_BSTAGE;
#pragma unroll
      for (int j = 0; j < 5; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(brsrc, (lds_void*)(base + (pw + 4 * j) * 1024), 16, boff[j],
                                                 (unsigned)(s * ROW_KB), 0, 0);
    };
    auto issue_slab = [&](int g) {                     // even (U) / odd (V) rows of slab g's chunk
      const int par = g >= 2 * nchunk ? 1 : 0, chunk = g - (par ? 2 : 1) * nchunk;
      char* base = aslab + (g & 1) * CK_ASLAB;
#pragma unroll
      for (int i = 0; i < NAP; ++i) {
        const int P = min(pw + 4 * i, 2 * (CK_AROWS / 16) - 1);
        char* dst = base + (P & 1) * CK_APLANE + (P >> 1) * 1024;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(arsrc, (lds_void*)dst, 16, par ? aoff[1][i] : aoff[0][i],
                                                 (unsigned)(chunk * ROW_KB), 0, 0);
      }
    };
    u32x4 sv[3][4];                                      // hi_e, lo_e, hi_o, lo_o per item
    auto load_s = [&](int chunk) {
      if constexpr ((PROBE & 16) != 0) return;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const unsigned co = (unsigned)(chunk * ROW_KB);
        sv[i][0] = __builtin_amdgcn_raw_buffer_load_b128(arsrc, soff_e[i] + co, 0, 0);
        sv[i][1] = __builtin_amdgcn_raw_buffer_load_b128(arsrc, soff_e[i] + co + 64, 0, 0);
        sv[i][2] = __builtin_amdgcn_raw_buffer_load_b128(arsrc, soff_o[i] + co, 0, 0);
        sv[i][3] = __builtin_amdgcn_raw_buffer_load_b128(arsrc, soff_o[i] + co + 64, 0, 0);
      }
    };
    float smax = 0.f;
    auto write_s = [&](int g) {                        // s = (hi_e + lo_e) + (hi_o + lo_o), plain split
      char* base = aslab + (g & 1) * CK_ASLAB;
      if constexpr ((PROBE & 8) != 0) {
        smax = fmaxf(smax, (float)__builtin_bit_cast(halfx8, sv[0][0])[0] + (float)__builtin_bit_cast(halfx8, sv[2][3])[7]);
        return;
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const halfx8 he = __builtin_bit_cast(halfx8, sv[i][0]), le = __builtin_bit_cast(halfx8, sv[i][1]);
        const halfx8 ho = __builtin_bit_cast(halfx8, sv[i][2]), lo = __builtin_bit_cast(halfx8, sv[i][3]);
        halfx8 hs, ls;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float s = ((float)he[k] + (float)le[k]) + ((float)ho[k] + (float)lo[k]);
          smax = fmaxf(smax, s);
          hs[k] = (_Float16)s;
          ls[k] = (_Float16)(s - (float)hs[k]);
        }
        if (sact[i]) {
          *(halfx8*)(base + sdst[i]) = hs;
          *(halfx8*)(base + CK_APLANE + sdst[i]) = ls;
        }
      }
    };
    const int nk = kb_total;
    // prologue: slab 0 (s of chunk 0), B stages 0..2
    if constexpr (!(PROBE & 1)) load_s(0);
    issue_b(0, 0);
    issue_b(min(1, nk - 1), 1);
    issue_b(min(2, nk - 1), 2);
    asm volatile("s_waitcnt vmcnt(5)" ::: "memory");   // s loads, stages 0 and 1
    if constexpr (!(PROBE & 1)) write_s(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    int slot = 0, s = 0;
    for (int g = 0; g < nslab; ++g) {
      const int T = ck_taps(g / nchunk);
      const bool more = g + 1 < nslab && !(PROBE & 4);
      const bool next_s = more && g + 1 < nchunk && !(PROBE & 1);   // next slab is an s slab (phase S)
      for (int t = 0; t < T; ++t, ++s) {
        const int lslot = slot == 0 ? CK_NSB - 1 : slot - 1;   // stage s+3's slot (read at s-1)
        if constexpr (!(PROBE & 4)) issue_b(min(s + CK_NSB - 1, nk - 1), lslot);
        // the next slab's loads go out at tap 0 AFTER that stage's B pieces, so every wait below
        // still covers B(s+2) (consumers read stage s+1 before barrier s) and the slab loads land
        // by tap 2's wait (vmcnt(5) there = all but B(s+3))
        if (t == 0 && next_s) {
          load_s(g + 1);
          asm volatile("s_waitcnt vmcnt(17)" ::: "memory");
        } else if (t == 0 && more) {
          issue_slab(g + 1);
          asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
        } else if (t == 1 && next_s) {
          asm volatile("s_waitcnt vmcnt(17)" ::: "memory");
        } else if (t == 1 && more) {
          asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
        }
        if (t == 2 && next_s) {
          write_s(g + 1);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        if constexpr (!(PROBE & 2)) __builtin_amdgcn_s_barrier();
        slot = slot + 1 == CK_NSB ? 0 : slot + 1;
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!(smax < 65504.f)) *p.ovf = 1;                 // a pair sum out of fp16 range: recomputed (bf16x6)
    __builtin_amdgcn_s_barrier();                      // consumers' epilogue reuses the LDS
    return;
  }

  // ---------------- consumers: LDS reads and MFMAs ----------------
  floatx4v acc_e[2][10], acc_o[2][10];
#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int nb = 0; nb < 10; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc_e[mb][nb][r] = 0.f;
  const int fr = lane & 15, fq = lane >> 4;
  const int brow = fr * 64 + 16 * (fq ^ swz(fr));
  auto read_a = [&](const char* slab, int t, bf16x8 (&a)[2][3]) {
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
      const int r = wave * 32 + mb * 16 + fr + t;
      const int off = r * 64 + 16 * (fq ^ swz(r));
      a[mb][0] = *(const bf16x8*)(slab + off);
      a[mb][1] = *(const bf16x8*)(slab + off + CK_APLANE);
    }
  };
  auto read_b = [&](const char* base, int nb, bf16x8 (&b)[3]) {
    const char* br = base + brow + nb * 1024;
    b[0] = *(const bf16x8*)(br);
    b[1] = *(const bf16x8*)(br + X6P_B_PLANE);
  };
  auto pin = [&]() {
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      if ((i & 1) == 0) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
    }
  };
  const int nk = kb_total;
  __builtin_amdgcn_s_barrier();                       // slab 0, B stages 0 and 1 landed
  asm volatile("" ::: "memory");
  bf16x8 as[2][3];
  bf16x8 b0[3], b1[3];
  read_a(aslab, 0, as);
  read_b(bring, 0, b0);
  int slot = 0, s = 0, g = 0;
  auto run_phase = [&](floatx4v (&acc)[2][10], int T) {
    for (int c = 0; c < nchunk; ++c, ++g) {
      const char* slab = aslab + (g & 1) * CK_ASLAB;
      for (int t = 0; t < T; ++t, ++s) {
        const char* base = bring + slot * H3C_BSTAGE;
        const int nslot = slot + 1 == CK_NSB ? 0 : slot + 1;
#pragma unroll
        for (int nb = 0; nb < 10; ++nb) {
          if (nb + 1 < 10) read_b(base, nb + 1, (nb & 1) ? b0 : b1);
#pragma unroll
          for (int mb = 0; mb < 2; ++mb) acc[mb][nb] = planes_mfma<2>(acc[mb][nb], as[mb], (nb & 1) ? b1 : b0);
          pin();
        }
        if (t + 1 < T)
          read_a(slab, t + 1, as);                      // slab reads stay in flight across the barrier
        else if (g + 1 < nslab)
          read_a(aslab + ((g + 1) & 1) * CK_ASLAB, 0, as);   // next slab complete since tap 2's barrier
        if (s + 1 < nk) read_b(bring + nslot * H3C_BSTAGE, 0, b0);   // stage s+1 landed at barrier s-1
        if constexpr (!(PROBE & 2)) __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        slot = nslot;
      }
    }
  };
  run_phase(acc_e, 4);                                // S into acc_e
#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int nb = 0; nb < 10; ++nb) acc_o[mb][nb] = acc_e[mb][nb];
  run_phase(acc_o, 5);                                // + U
  run_phase(acc_e, 4);                                // + V
  __builtin_amdgcn_s_barrier();                       // producers drained their tail pieces
  const long long mw = 2 * (p0 + wave * 32);          // first output row of the wave
  if constexpr (EPI == EPI_RELU)
    epilogue_relu_h2_pairs(p, acc_e, acc_o, mw, n0, lane, smem + wave * H3E_WAVE);
  else
    epilogue_pool_h2_pairs<LAYER == 4>(p, acc_e, acc_o, mw, n0, lane, smem + wave * H3E_WAVE);
}

}  // namespace expecto
