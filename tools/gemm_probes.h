// Probe-only GEMM kernels of tools/gemm_bench (never launched by libexpecto_hip.so): the
// measured-and-rejected shapes DESIGN.md section 7 quotes, kept so their numbers can be re-taken
// against the library's kernels (expecto_amd/csrc/gemm_kernel.h) on the same box.
//   beluga_gemm_x6   register-staged bf16x6 (A re-split per Toeplitz tap; 197 vs 284 TF/s)
//   beluga_fc_h3     FC with each wave's A fragments loaded straight into registers
//   beluga_conv_h3s  8-wave (two per SIMD) conv tiles, optionally staggered partners
//   beluga_gemm_h3q  the planes GEMM at PL 2 (f16x3 without the chunk slab)
//   beluga_conv_h3q  the chunk-slab conv body at 256-row tiles, 4 waves
//   beluga_conv_h3pp persistent producer / consumer conv workgroups (round 3: hides the
//                    per-tile prologue, +1-3 % without epilogue, not the epilogue itself)
#pragma once
#include "../expecto_amd/csrc/gemm_kernel.h"

namespace expecto {

// ---- fp32-faithful split-bf16 variant ("bf16x6") -------------------------------------
// Every fp32 operand x is split exactly into three bf16 terms x = x0 + x1 + x2 (+ <2^-24|x|)
// while it is staged into LDS; each 16-deep k-step issues the six v_mfma_f32_32x32x16_bf16
// products of combined order <= 2 (x0y0, x0y1, x1y0, x0y2, x1y1, x2y0) into the same fp32
// accumulator.  Products of bf16 terms are exact in fp32, so the result is fp32-accurate
// (tools/split_precision_study.py: 0.06 of the parity bound on alt-ref diffs, vs 0.08 for
// oneDNN fp32) at 6 x 1/16 = 3/8 the MFMA cycles of v_mfma_f32_32x32x2_f32.

template <int LAYER, int EPI, int WM = 4, int MINB = 2>
__global__ __launch_bounds__(64 * WM, MINB * WM / 4) void beluga_gemm_x6(GemmArgs p) {
  constexpr int BM = 32 * WM;
  constexpr int NT = 64 * WM;
  constexpr int BK = GBK;                        // one 32-wide K block per stage
  constexpr int F4 = BK / 4;
  constexpr int RSTEP = NT / F4;
  constexpr int ALD = BM / RSTEP;
  constexpr int BLD = (GBN + RSTEP - 1) / RSTEP;
  constexpr int RS = 40;                         // LDS row stride in bf16 (80 B): b128 reads conflict-free
  constexpr int APL = BM * RS, BPL = GBN * RS;    // plane sizes (bf16 elements)
  __shared__ __attribute__((aligned(16))) __bf16 smem[3 * APL + 3 * BPL];
  __bf16* As = smem;
  __bf16* Bs = smem + 3 * APL;

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
  const long long m0 = mt * BM;
  const int n0 = nt * GBN;
  const int gs0 = ks * (p.kper / GBK);
  const float* ag[ALD];
#pragma unroll
  for (int i = 0; i < ALD; ++i) {
    long long m = m0 + lr + RSTEP * i;
    if (m > p.M - 1) m = p.M - 1;
    ag[i] = p.A + (p.a_rows ? p.a_rows[m] : m * p.lda) + lc;
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
  floatx4 ra[ALD], rb[BLD];
  auto gload = [&](int s) {
    const long long ao = a_off(gs0 + s);
#pragma unroll
    for (int i = 0; i < ALD; ++i) ra[i] = *(const floatx4*)(ag[i] + ao);
#pragma unroll
    for (int i = 0; i < BLD; ++i) rb[i] = *(const floatx4*)(bg[i] + s * BK);
  };
  auto sstore = [&]() {
#pragma unroll
    for (int i = 0; i < ALD; ++i) {
      bf16x4 h, m, l;
      split3(ra[i], h, m, l);
      __bf16* d = As + (lr + RSTEP * i) * RS + lc;
      *(bf16x4*)(d) = h;
      *(bf16x4*)(d + APL) = m;
      *(bf16x4*)(d + 2 * APL) = l;
    }
#pragma unroll
    for (int i = 0; i < BLD; ++i) {
      if ((GBN % RSTEP == 0) || (lr + RSTEP * i < GBN)) {
        bf16x4 h, m, l;
        split3(rb[i], h, m, l);
        __bf16* d = Bs + (lr + RSTEP * i) * RS + lc;
        *(bf16x4*)(d) = h;
        *(bf16x4*)(d + BPL) = m;
        *(bf16x4*)(d + 2 * BPL) = l;
      }
    }
  };

  const int wave = tid >> 6, lane = tid & 63, li = lane & 31, lh = lane >> 5;
  floatx16 acc[GTN];
#pragma unroll
  for (int t = 0; t < GTN; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  // 16-deep k-step kq: lane half h reads columns 16kq + 8h .. +7 of its row (A and B alike)
  const __bf16* aw = As + (wave * 32 + li) * RS + 8 * lh;
  const __bf16* bw = Bs + li * RS + 8 * lh;
  const int nk = p.kper / BK;

  gload(0);
  sstore();
  __syncthreads();
  for (int s = 0; s < nk; ++s) {
    const bool more = (s + 1) < nk;
    if (more) gload(s + 1);
#pragma unroll
    for (int kq = 0; kq < 2; ++kq) {
      const bf16x8 a0 = *(const bf16x8*)(aw + 16 * kq);
      const bf16x8 a1 = *(const bf16x8*)(aw + APL + 16 * kq);
      const bf16x8 a2 = *(const bf16x8*)(aw + 2 * APL + 16 * kq);
#pragma unroll
      for (int t = 0; t < GTN; ++t) {
        const __bf16* bt = bw + t * 32 * RS + 16 * kq;
        const bf16x8 b0 = *(const bf16x8*)(bt);
        const bf16x8 b1 = *(const bf16x8*)(bt + BPL);
        const bf16x8 b2 = *(const bf16x8*)(bt + 2 * BPL);
        floatx16 c = acc[t];
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, c, 0, 0, 0);
        acc[t] = c;
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


// ---- f16x3 FC GEMM: A fragments straight into registers ---------------------------------
// In the FC layers every wave owns its 64 A rows (no Toeplitz overlap, nothing shared between
// the waves), so staging A through LDS is pure overhead: 8 LDS-DMA pieces + 8 ds_reads per
// wave and K block, next to 5 B pieces (tools/gemm_bench fc1: 364 fp32-equivalent TF/s, 538
// with the in-loop LDS-DMA removed).  Here each lane loads its own MFMA fragments (row l & 15
// of a 16-row block, k 8*(l >> 4)..+7: 16 B per plane) with global_load_dwordx4 two K blocks
// ahead into a 3-deep register ring; only B (shared by the 4 waves) goes through an LDS ring.
// Same operands, products and k order per output as gemm_planes_body<PL=2>: bitwise equal.
constexpr int FCH_BSTAGE = 2 * X6P_B_PLANE;           // one B stage: 160 cols x 32 k x 2 planes
// NB: 16-column blocks per tile (10: 160-column tiles; 21: 336-column tiles, 6 of which cover
// FC1's 2016 padded outputs with 0.6 % padding instead of 13 x 160 = 2080's 3.8 %, and each A
// fragment feeds 2.1x the MFMAs: half the A traffic from L2 / Infinity Cache per MFMA).
// NW: waves per workgroup (4: 64 rows each, one per SIMD; 8: 32 rows each, two per SIMD, so a
// 336-column tile's 168 accumulators fit the 256 registers of a wave).
template <int NB, int NW = 4>
struct FcGeo {
  static constexpr int BN = 16 * NB;
  static constexpr int MBW = 16 / NW;                  // 16-row blocks per wave (tile: 256 rows)
  static constexpr int PLANE = NB * 1024;              // one plane of a B stage
  static constexpr int STAGE = 2 * PLANE;
  static constexpr int PIECES = 2 * NB;                // 1 KiB LDS-DMA pieces per stage
  static constexpr int NBP = (PIECES + NW - 1) / NW;   // pieces per wave (the last repeated)
};

// NS: ring depth of both operands (A register sets and B LDS slots): K block s+NS-1 is loaded
// while block s computes.
template <int LAYER, int EPI, int TM, int NS, int NB = 10, int NW = 4>
__device__ __forceinline__ void gemm_fc_h3_body(const GemmArgs& p, char* smem) {
  static_assert(NS >= 2 && NS <= 4, "ring depth");
  using F = FcGeo<NB, NW>;
  constexpr int MBW = F::MBW;
  constexpr int ROW_KB = 128;                          // bytes per row and 32-deep K block (2 planes)
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
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const long long m0 = mt * X6P_BM;
  const int n0 = nt * F::BN;
  const int kb_total = (int)(p.ldb / GBK);
  const int gs0 = ks * (p.kper / GBK);
  const long long lda_kb = p.lda / GBK;
  const int nk = p.kper / GBK;
  auto swz = [](int r) { return (-(r >> 2)) & 3; };
  const int fr = lane & 15, fq = lane >> 4;
  // this lane's A source: row m0 + wave*16*MBW + 16*mb + fr (clamped), bytes 16*fq of each plane
  const char* aptr[MBW];
#pragma unroll
  for (int mb = 0; mb < MBW; ++mb) {
    long long m = m0 + wave * 16 * MBW + mb * 16 + fr;
    if (m > p.M - 1) m = p.M - 1;
    const long long kb0 = (p.a_rows ? p.a_rows[m] / GBK : m * lda_kb) + gs0;
    aptr[mb] = (const char*)p.A + kb0 * ROW_KB + 16 * fq;
  }
  const char* Bb = (const char*)p.Bp + ((long long)n0 * kb_total + gs0) * ROW_KB;
  unsigned boff[F::NBP];
#pragma unroll
  for (int j = 0; j < F::NBP; ++j) {
    const int g = min(wave + NW * j, F::PIECES - 1);   // piece g: plane g / NB, cols 16*(g % NB)
    const int pl = g / NB, r = 16 * (g % NB) + (lane >> 2);
    const int c = (lane & 3) ^ swz(r);
    boff[j] = (unsigned)((long long)r * kb_total * ROW_KB + pl * 64 + 16 * c);
  }
  const __amdgpu_buffer_rsrc_t brsrc = __builtin_amdgcn_make_buffer_rsrc((void*)Bb, (short)0, 0x7fffffff, 0x00020000);
  auto issue_b = [&](int s, int slot, int j0, int nj) {
    if constexpr ((TM & 8) != 0) s = 0;
    char* base = smem + slot * F::STAGE;
    for (int j = j0; j < j0 + nj; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(brsrc, (lds_void*)(base + min(wave + NW * j, F::PIECES - 1) * 1024), 16, boff[j],
                                               (unsigned)(s * ROW_KB), 0, 0);
  };
  // A fragments of K block s into ring set `set` (two loads per row block: hi, lo plane)
  bf16x8 afr[NS][MBW][3];
  auto load_a = [&](int s, bf16x8 (&a)[MBW][3], int mb0, int nmb) {
    if constexpr ((TM & 8) != 0) s = 0;
    const long long off = (long long)s * ROW_KB;
    for (int mb = mb0; mb < mb0 + nmb; ++mb) {
      a[mb][0] = *(const bf16x8*)(aptr[mb] + off);
      a[mb][1] = *(const bf16x8*)(aptr[mb] + off + 64);
    }
  };

  floatx4v acc[MBW][NB];
#pragma unroll
  for (int mb = 0; mb < MBW; ++mb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[mb][nb][r] = 0.f;
  const int brow = fr * 64 + 16 * (fq ^ swz(fr));
  auto read_b = [&](const char* base, int nb, bf16x8 (&b)[3]) {
    const char* br = base + brow + nb * 1024;
    b[0] = *(const bf16x8*)(br);
    b[1] = *(const bf16x8*)(br + F::PLANE);
  };
  auto pin = [&](int nv) {
    constexpr int MF = 3 * MBW;                        // MFMAs per unit
#pragma unroll
    for (int i = 0; i < MF; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      if ((i % (MF / 2)) == 0 && i < (MF / 2) * nv) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      if ((i & 1) == 0) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
    }
  };

  // prologue: A and B of K blocks 0 .. NS-2
  load_a(0, afr[0], 0, MBW);
  issue_b(0, 0, 0, F::NBP);
  if constexpr (NS >= 3) {
    load_a(min(1, nk - 1), afr[1], 0, MBW);
    issue_b(min(1, nk - 1), 1, 0, F::NBP);
  }
  if constexpr (NS == 4) {
    load_a(min(2, nk - 1), afr[2], 0, MBW);
    issue_b(min(2, nk - 1), 2, 0, F::NBP);
  }
  __builtin_amdgcn_s_waitcnt(0);     // (prologue only) everything above landed
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  // one K block: compute on ring set I (block s); load A and B of block s+NS-1 into the A set and
  // the B slot that block s-1 used
  auto stage = [&](auto I, int s, int& slot) {
    constexpr int cur = decltype(I)::value, nxt = (cur + NS - 1) % NS;
    const int sa = (TM & 2) ? s : min(s + NS - 1, nk - 1);
    const int sb = (TM & 2) ? s : min(s + NS - 1, nk - 1);
    const int nslot = slot + 1 == NS ? 0 : slot + 1;
    const int lslot = slot == 0 ? NS - 1 : slot - 1;
    const char* base = smem + slot * F::STAGE;
    bf16x8 b0[3], b1[3];
    read_b(base, 0, b0);
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      int nv = 0;
      if (!(TM & 2)) {
        if (nb < MBW) {                    // A of block s+NS-1: 2 loads per unit
          if (!(TM & 16)) load_a(sa, afr[nxt], nb, 1);
          nv = 2;
        } else if (nb < MBW + F::NBP) {    // B of block s+NS-1: 1 piece per unit
          if (!(TM & 32)) issue_b(sb, lslot, nb - MBW, 1);
          nv = 1;
        }
      }
      if (nb + 1 < NB) read_b(base, nb + 1, (nb & 1) ? b0 : b1);
#pragma unroll
      for (int mb = 0; mb < MBW; ++mb)
        acc[mb][nb] = planes_mfma<2>(acc[mb][nb], afr[cur][mb], (nb & 1) ? b1 : b0);
      pin(nv);
    }
    if constexpr (!(TM & 4)) {
      // A and B of block s+1 landed in every wave (in flight: blocks s+2 .. s+NS-1, 13 loads
      // each).  The builtin, not asm: the compiler's own wait insertion then knows what has
      // landed (simm16 = vmcnt[3:0] | expcnt 7 << 4 | lgkmcnt 0 << 8 | vmcnt[5:4] << 14).
      constexpr int VM = (NS - 2) * (2 * MBW + F::NBP);   // loads of blocks s+2 .. s+NS-1 in flight
      static_assert(VM < 64, "vmcnt field");
      __builtin_amdgcn_s_waitcnt((VM & 15) | (7 << 4) | ((VM >> 4) << 14));   // vmcnt(VM) lgkmcnt(0)
      __builtin_amdgcn_s_barrier();
    }
    asm volatile("" ::: "memory");
    slot = nslot;
  };
  // unconditional NS-stage loop body (the compiler's own vmcnt tracking then sees every back
  // edge with all loads issued after the set it waits for), tail after the loop
  int slot = 0, s = 0;
  for (; s + NS <= nk; s += NS) {
    stage(std::integral_constant<int, 0>{}, s, slot);
    stage(std::integral_constant<int, 1>{}, s + 1, slot);
    if constexpr (NS >= 3) stage(std::integral_constant<int, 2>{}, s + 2, slot);
    if constexpr (NS == 4) stage(std::integral_constant<int, 3>{}, s + 3, slot);
  }
  if (s < nk) stage(std::integral_constant<int, 0>{}, s, slot);
  if constexpr (NS >= 3)
    if (s + 1 < nk) stage(std::integral_constant<int, 1>{}, s + 1, slot);
  if constexpr (NS == 4)
    if (s + 2 < nk) stage(std::integral_constant<int, 2>{}, s + 2, slot);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the ring's duplicate tail loads
  gemm_epilogue16<EPI, 2, NB, MBW>(p, acc, m0 + wave * 16 * MBW, n0, ks, lane);
}

template <int LAYER, int EPI, int TM = 0, int NS = 3, int NB = 10, int NW = 4>
__global__ __launch_bounds__(64 * NW, 1) void beluga_fc_h3(GemmArgs p) {
  __shared__ __attribute__((aligned(1024))) char smem[NS * FcGeo<NB, NW>::STAGE];
  gemm_fc_h3_body<LAYER, EPI, TM, NS, NB, NW>(p, smem);
}


// ---- f16x3 conv GEMM, 8 waves (two per SIMD) ---------------------------------------------
// gemm_conv_h3_body's tile split over 8 waves of 16*MB rows x 80 columns (tile 64*MB x 160:
// MB 4 = 256 rows, MB 6 = 384 rows with the 400-row slab of SlabGeo<6>; wave w: rows
// 16*MB*(w & 3), columns 80*(w >> 2); MB x 5 accumulator blocks), so the two waves of a SIMD
// cover each other's barrier waits, LDS-DMA issue and LDS reads (with one wave per SIMD the
// MFMA pipe idles through them).  Same slab / ring staging (A slab pieces P = wave + 8*i, B
// pieces wave + 8*j of 20).  tools/gemm_bench, 2000 windows, fp32-equivalent TF/s: conv3 465
// (4-wave 256-row h3q 456) -> 487 at MB 6, conv5 466 -> 489 at MB 6, conv6 484 at MB 4 (468 at
// MB 6); the pool layers stay on the 4-wave 384-row beluga_conv_h3r (conv4 517 vs 507).
// STG 1 (measured slower, 3-8 %: kept as a probe) staggers the two waves of a SIMD (w and w+4) by half a K stage
// (MI355X_MICROARCH.md "Two waves per SIMD" item 9): waves 4-7 run units 3,4 of stage s-1
// (their B fragments read into registers before that stage's barrier, since the slot is
// refilled right after it) and units 0-2 of stage s between barriers s-1 and s, so the
// partners' LDS-read bursts and MFMA runs interleave instead of colliding.  Load issue per
// barrier interval, LDS ring and slab schedule are the same for both halves.  Same products
// and k order per output as every other f16x3 conv kernel: bitwise equal.
template <int MB>
__device__ __forceinline__ void epilogue_relu_h2_lds8m(const GemmArgs& p, const floatx4v (&acc)[MB][5], long long m0,
                                                       int wm, int wn, int n0, int lane, int tid, char* lds) {
  constexpr int WR = 16 * MB;                          // rows per wave
  const int fr = lane & 15, fq = lane >> 4;
  const long long ldb = p.ldc >> 5;
  const long long w0 = m0 / p.s_in;
  const int t0 = (int)(m0 - w0 * p.s_in);
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    if ((wm >> 1) == pass) {            // this pass stages rows 2*WR*pass .. +2*WR-1 (waves wm = 2*pass, 2*pass+1)
#pragma unroll
      for (int nb = 0; nb < 5; ++nb) {
        const int c = wn * 80 + nb * 16 + fr, n = n0 + c;
        const float bn = n < p.n_store ? p.bias[n] : 0.f;
        const float cs = n < p.n_store ? p.col_scale[n] : 0.f;
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float x = fmaxf(acc[mb][nb][j] * cs + bn, 0.f) * p.out_scale;
            if (!(fabsf(x) < 65504.f)) *p.ovf = 1;
            _Float16 hi, lo;
            split_h2(x, hi, lo);
            char* d = lds + ((wm & 1) * WR + mb * 16 + 4 * fq + j) * H3E_ROW + (c >> 5) * 128 + (c & 31) * 2;
            *(_Float16*)d = hi;
            *(_Float16*)(d + 64) = lo;
          }
      }
    }
    __syncthreads();
    // 2*WR rows x 40 chunks of 16 B over 512 threads
#pragma unroll 2
    for (int i = 0; i < (2 * WR * 40) / 512; ++i) {
      const int k = i * 512 + tid, row = k / 40, ch = k - row * 40;
      const long long m = m0 + pass * 2 * WR + row;
      if (m < p.M) {
        long long w;
        int tpos;
        row_wt(w0, t0, pass * 2 * WR + row, p.s_in, w, tpos);
        if (tpos < p.t_valid && n0 + (ch >> 3) * 32 < p.n_store) {
          char* g = (char*)p.C + ((w * p.s_out + tpos) * ldb + (n0 >> 5)) * 128 + ch * 16;
          *(floatx4v*)g = *(const floatx4v*)(lds + row * H3E_ROW + ch * 16);
        }
      }
    }
    __syncthreads();
  }
}

template <int LAYER, int EPI, int TM, int MB, int STG>
__device__ __forceinline__ void gemm_conv_h3s_body(const GemmArgs& p, char* smem) {
  using G = SlabGeo<MB>;
  constexpr int ROW_KB = 128;
  constexpr int NSB = 3;
  constexpr int NA8 = (G::PIECES + 7) / 8;            // slab pieces per wave and chunk (max)
  static_assert(NA8 <= 7, "slab pieces must be issued by tap 6");
  const unsigned nblk = gridDim.x, bid = blockIdx.x;
  const unsigned xcd = bid & 7u, q = nblk >> 3, rr = nblk & 7u;
  const unsigned lin = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  const int nt = (int)(lin % (unsigned)p.n_tiles);
  const long long mt = (long long)(lin / (unsigned)p.n_tiles) % p.m_tiles;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 3, wn = wave >> 2;
  const long long m0 = mt * G::BM;
  const int n0 = nt * GBN;
  const int kb_total = (int)(p.ldb / GBK);
  const long long lda_kb = p.lda / GBK;
  const int nchunk = (int)lda_kb;
  const int nk = nchunk * 8;
  auto swz = [](int r) { return conv_swz<TM>(r); };
  const char* Ab = (const char*)p.A + m0 * lda_kb * ROW_KB;
  const long long last_row = p.M - 1 + 7;
  const int na = (G::PIECES - wave + 7) / 8;          // A slab pieces P = wave + 8*i < PIECES
  unsigned aoff[NA8];
#pragma unroll
  for (int i = 0; i < NA8; ++i) {
    const int P = min(wave + 8 * i, G::PIECES - 1), g = P >> 1, pl = P & 1;
    const int r = 16 * g + (lane >> 2);
    const long long m = min(m0 + r, last_row);
    const int c = (lane & 3) ^ swz(r);
    aoff[i] = (unsigned)((m - m0) * lda_kb * ROW_KB + pl * 64 + 16 * c);
  }
  const char* Bb = (const char*)p.Bp + (long long)n0 * kb_total * ROW_KB;
  const int nbp = wave < 4 ? 3 : 2;              // B pieces P = wave + 8*j < 20
  unsigned boff[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int g = min(wave + 8 * j, 19);
    const int pl = g / 10, r = 16 * (g % 10) + (lane >> 2);
    const int c = (lane & 3) ^ swz(r);
    boff[j] = (unsigned)((long long)r * kb_total * ROW_KB + pl * 64 + 16 * c);
  }
  const __amdgpu_buffer_rsrc_t arsrc = __builtin_amdgcn_make_buffer_rsrc((void*)Ab, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t brsrc = __builtin_amdgcn_make_buffer_rsrc((void*)Bb, (short)0, 0x7fffffff, 0x00020000);
  char* const aslab = smem;
  char* const bring = smem + 2 * G::ASLAB;
  auto issue_a = [&](int chunk, int i) {
    if (i >= na) return;
    const int P = wave + 8 * i;
    char* dst = aslab + (chunk & 1) * G::ASLAB + (P & 1) * G::APLANE + (P >> 1) * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(arsrc, (lds_void*)dst, 16, aoff[i], (unsigned)(chunk * ROW_KB), 0, 0);
  };
  auto issue_b = [&](int s, int slot) {
    if constexpr ((TM & 8) != 0) s = 0;
    char* base = bring + slot * H3C_BSTAGE;
#pragma unroll
    for (int j = 0; j < 3; ++j)
      if (j < nbp)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(brsrc, (lds_void*)(base + (wave + 8 * j) * 1024), 16, boff[j],
                                                 (unsigned)(s * ROW_KB), 0, 0);
  };
  // slab c+1 pieces issued at tap t (unit 0): pieces 0,1 at tap 0, piece t+1 at taps 1..NA8-2
  auto issue_a_tap = [&](int c, int t) -> int {
    if (t == 0) {
      issue_a(c + 1, 0);
      issue_a(c + 1, 1);
      return 2;
    }
    if (t <= NA8 - 2) {
      issue_a(c + 1, t + 1);
      return 1;
    }
    return 0;
  };

  floatx4v acc[MB][5];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int nb = 0; nb < 5; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[mb][nb][r] = 0.f;
  const int fr = lane & 15, fq = lane >> 4;
  const int brow = (wn * 5) * 1024 + fr * 64 + 16 * (fq ^ swz(fr));
  auto read_a = [&](const char* slab, int t, bf16x8 (&a)[MB][3]) {
    const int rr2 = fr + t;
    const int off = (wm * 16 * MB + rr2) * 64 + 16 * (fq ^ swz(rr2));
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
  // nv VMEM issues and nd ds_reads spread over this unit's 3*MB MFMAs
  auto pin = [&](int nv, int nd) {
#pragma unroll
    for (int i = 0; i < 3 * MB; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      if ((i % 4) == 0 && i < 4 * nv) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      if ((i & 1) == 0 && (i >> 1) < nd) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
    }
  };
  auto stage_wait = [&]() {
    if constexpr (!(TM & 4)) {
      if (wave < 4)
        asm volatile("s_waitcnt vmcnt(3) lgkmcnt(0)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    asm volatile("" ::: "memory");
  };

  for (int i = 0; i < NA8; ++i) issue_a(0, i);
  issue_b(0, 0);
  issue_b(min(1, nk - 1), 1);
  if (wave < 4)
    asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  bf16x8 as[MB][3];
  read_a(aslab, 0, as);
  int slot = 0;
  if (!STG || wn == 0) {
    for (int c = 0; c < nchunk; ++c) {
      const char* slab = aslab + (c & 1) * G::ASLAB;
      const bool more_a = (c + 1 < nchunk) && !(TM & 2);
      for (int t = 0; t < 8; ++t) {
        const int s = c * 8 + t;
        const int nslot = slot + 1 == NSB ? 0 : slot + 1;
        const int lslot = slot == 0 ? NSB - 1 : slot - 1;
        const char* base = bring + slot * H3C_BSTAGE;
        bf16x8 b0[3], b1[3];
        read_b(base, 0, b0);
#pragma unroll
        for (int nb = 0; nb < 5; ++nb) {
          int nv = 0;
          if (nb == 0 && more_a) nv = issue_a_tap(c, t);
          if (nb == 1 && !(TM & 2)) {
            issue_b(min(s + 2, nk - 1), lslot);
            nv = 3;
          }
          if (nb + 1 < 5) read_b(base, nb + 1, (nb & 1) ? b0 : b1);
          unit(as, nb, (nb & 1) ? b1 : b0);
          pin(nv, 2 * MB);
        }
        if (t < 7) read_a(slab, t + 1, as);
        stage_wait();
        slot = nslot;
      }
      if (c + 1 < nchunk) read_a(aslab + ((c + 1) & 1) * G::ASLAB, 0, as);
    }
  } else {
    // staggered half: interval s = units 3,4 of stage s-1 (A in `as`, B in bs3/bs4), then A of
    // stage s and its units 0-2; B of units 3,4 read before barrier s
    bf16x8 bs3[3], bs4[3];
    for (int c = 0; c < nchunk; ++c) {
      const char* slab = aslab + (c & 1) * G::ASLAB;
      const bool more_a = (c + 1 < nchunk) && !(TM & 2);
      for (int t = 0; t < 8; ++t) {
        const int s = c * 8 + t;
        const int nslot = slot + 1 == NSB ? 0 : slot + 1;
        const int lslot = slot == 0 ? NSB - 1 : slot - 1;
        const char* base = bring + slot * H3C_BSTAGE;
        bf16x8 b0[3], b1[3];
        if (s > 0) {
          // units 3,4 of stage s-1 row block by row block; each block's A registers are
          // refilled with stage s's fragments as soon as its 6 MFMAs have issued
          const int nv = more_a ? issue_a_tap(c, t) : 0;
          const int rr2 = fr + t;
          const int off = (wm * 16 * MB + rr2) * 64 + 16 * (fq ^ swz(rr2));
#pragma unroll
          for (int mb = 0; mb < MB; ++mb) {
            acc[mb][3] = planes_mfma<2>(acc[mb][3], as[mb], bs3);
            acc[mb][4] = planes_mfma<2>(acc[mb][4], as[mb], bs4);
            as[mb][0] = *(const bf16x8*)(slab + off + mb * 1024);
            as[mb][1] = *(const bf16x8*)(slab + off + mb * 1024 + G::APLANE);
          }
          read_b(base, 0, b0);
#pragma unroll
          for (int mb = 0; mb < MB; ++mb) {
            if (mb < nv) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
          }
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        } else {
          if (more_a) issue_a_tap(c, t);
          read_b(base, 0, b0);
        }
#pragma unroll
        for (int nb = 0; nb < 3; ++nb) {
          int nv = 0;
          if (nb == 0 && !(TM & 2)) {
            issue_b(min(s + 2, nk - 1), lslot);
            nv = 3;
          }
          if (nb == 0) read_b(base, 1, b1);
          if (nb == 1) read_b(base, 2, b0);
          if (nb == 2) {
            read_b(base, 3, bs3);
            read_b(base, 4, bs4);
          }
          unit(as, nb, (nb & 1) ? b1 : b0);
          pin(nv, nb == 2 ? 4 : 2);
        }
        stage_wait();
        slot = nslot;
      }
    }
    unit(as, 3, bs3);
    unit(as, 4, bs4);
  }
  if constexpr (EPI == EPI_RELU) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    epilogue_relu_h2_lds8m<MB>(p, acc, m0, wm, wn, n0, lane, tid, smem);
  } else {
    gemm_epilogue16<EPI, 2, 5, MB>(p, acc, m0 + wm * 16 * MB, n0 + wn * 80, 0, lane);
  }
}

// MB 4 / 6 row blocks per wave, STG 0 / 1 (see gemm_conv_h3s_body)
template <int LAYER, int EPI, int TM = 0, int MB = 6, int STG = 0>
__global__ __launch_bounds__(512, 1) void beluga_conv_h3s(GemmArgs p) {
  __shared__ __attribute__((aligned(1024))) char smem[h3c_lds_mb<3, MB>()];
  gemm_conv_h3s_body<LAYER, EPI, TM, MB, STG>(p, smem);
}


template <int LAYER, int EPI, int TM = 0, int NS = 3>
__global__ __launch_bounds__(256, 1) void beluga_gemm_h3q(GemmArgs p) {
  __shared__ __attribute__((aligned(1024))) char smem[NS * PlaneGeo<2>::STAGE];
  gemm_planes_body<LAYER, EPI, TM, 2, NS>(p, smem);
}


// f16x3 conv layers (taps == 8, no split-K): the chunk-slab kernel above
template <int LAYER, int EPI, int TM = 0, int NSB = 3>
__global__ __launch_bounds__(256, 1) void beluga_conv_h3q(GemmArgs p) {
  __shared__ __attribute__((aligned(1024))) char smem[h3c_lds<NSB>()];
  gemm_conv_h3_body<LAYER, EPI, TM, NSB>(p, smem);
}


// ---- f16x3 conv GEMM, persistent producer / consumer workgroups -------------------------
// gemm_conv_h3p_body (NSB 4, PF) with one workgroup per CU looping over tiles (virtual block
// v = blockIdx.x + k * gridDim.x, mapped to (M tile, N tile) by the same XCD remap as a
// one-tile-per-workgroup launch of all tiles; gridDim.x a multiple of 8 keeps v's XCD).  The B
// ring and the slab double buffer run on a global stage / chunk counter across tiles, so the
// producers stage the next tile's chunk-0 slab and its first 3 B stages during the current
// tile's last chunk, and the consumers start the next tile right after their epilogue instead
// of behind a new workgroup's prologue.  The epilogue's global stores (160 KB per tile; every CU
// stores at once when tiles run in lockstep rounds) then drain while the next tile's MFMAs run:
// a consumer wave issues no vector-memory loads, so it never waits for them.
// Epilogue staging: 16-row passes, per wave 16 x 656 B in LDS the producers do not touch
// until every consumer has passed one extra barrier per tile ("E"): waves 0-2 in the slab the
// tile's last chunk used, wave 3 in the B ring slot of the tile's last stage.  Producers enter
// barrier E first thing in every tile but the first, before issuing that tile's slab pieces of
// chunk 1 (which go to that slab) and B stage 3 (which goes to that slot).
// Same products and k order per output as every f16x3 conv kernel: bitwise equal.
// Measured (profiles/r03/gemm_bench_fc1_order_convpp.txt): conv2 551 vs 546, conv3 474 vs 481,
// conv4 548 vs 540, conv5 495 vs 503, conv6 498 vs 500 fp32-eq TF/s against the per-tile
// kernel, the 200-window pipeline unchanged (996-998 vs 995-999 variants/s); TM 4096 (odd
// workgroups start half a tile late, so the CUs' epilogue store bursts alternate) slower still.
// Not used by the library.
template <int MB16 = 4>
__device__ __forceinline__ void epilogue_relu_h2_q16(const GemmArgs& p, const floatx4v (&acc)[4][10], long long mw,
                                                     int n0, int lane, char* lds) {
  const int fr = lane & 15, fq = lane >> 4;
  const long long w0 = mw / p.s_in;
  const int t0 = (int)(mw - w0 * p.s_in);
  const long long ldb = p.ldc >> 5;
  float vmax = 0.f;
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) {
#pragma unroll
    for (int nb = 0; nb < 10; ++nb) {
      const int n = n0 + nb * 16 + fr;
      const float cso = n < p.n_store ? p.col_scale[n] * p.out_scale : 0.f;
      const float bo = n < p.n_store ? p.bias[n] * p.out_scale : 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float x = fmaxf(fmaf(acc[mb][nb][j], cso, bo), 0.f);
        vmax = fmaxf(vmax, x);
        _Float16 hi, lo;
        split_h2p(x, hi, lo);
        char* d = lds + (4 * fq + j) * H3E_ROW + (nb >> 1) * 128 + ((nb & 1) * 16 + fr) * 2;
        *(_Float16*)d = hi;
        *(_Float16*)(d + 64) = lo;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll 5
    for (int i = 0; i < 10; ++i) {
      const int k = i * 64 + lane, row = k / 40, ch = k - row * 40;
      const long long m = mw + mb * 16 + row;
      if (m < p.M) {
        long long w;
        int tpos;
        row_wt(w0, t0, mb * 16 + row, p.s_in, w, tpos);
        if (tpos < p.t_valid && n0 + (ch >> 3) * 32 < p.n_store) {
          char* g = (char*)p.C + ((w * p.s_out + tpos) * ldb + (n0 >> 5)) * 128 + ch * 16;
          *(floatx4v*)g = *(const floatx4v*)(lds + row * H3E_ROW + ch * 16);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if (!(vmax < 65504.f)) *p.ovf = 1;
}

// (mt, nt) of virtual block v of a launch of `nv` blocks (the XCD remap of the conv kernels)
__device__ __forceinline__ void conv_tile_of(const GemmArgs& p, unsigned v, unsigned nv, long long& mt, int& nt) {
  const unsigned xcd = v & 7u, q = nv >> 3, rr = nv & 7u;
  const unsigned lin = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (v >> 3);
  nt = (int)(lin % (unsigned)p.n_tiles);
  mt = (long long)(lin / (unsigned)p.n_tiles) % p.m_tiles;
}

template <int LAYER, int EPI, int TM>
__device__ __forceinline__ void gemm_conv_h3pp_body(const GemmArgs& p, char* smem) {
  static_assert(EPI == EPI_RELU || EPI == EPI_RELU_POOL4, "conv epilogues only");
  constexpr int NSB = 4;
  using G = SlabGeo<4>;
  constexpr int ROW_KB = 128;
  constexpr int NAP = (G::PIECES + 3) / 4;            // slab pieces per producer wave and chunk (9)
  const unsigned nv = (unsigned)(p.m_tiles * p.n_tiles), gstep = gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kb_total = (int)(p.ldb / GBK);
  const long long lda_kb = p.lda / GBK;
  const int nchunk = (int)lda_kb;
  const int nk = nchunk * 8;
  auto swz = [](int r) { return conv_swz<TM>(r); };
  char* const aslab = smem;
  char* const bring = smem + 2 * G::ASLAB;
  const int ntile = (int)((nv - blockIdx.x + gstep - 1) / gstep);   // tiles of this workgroup (>= 1)
  if constexpr ((TM & 4096) != 0) {   // probe: odd workgroups start half a tile late (epilogues out of phase)
    if (blockIdx.x & 1)
      for (int i = 0; i < nk; ++i) __builtin_amdgcn_s_sleep(15);
  }

  if (wave >= 4) {
    // ---------------- producer: all LDS-DMA issue, on a global stage / chunk counter ----------------
    const int pw = wave - 4;
    const long long last_row = p.M - 1 + 7;
    unsigned boffs[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const int g = pw + 4 * j;
      const int pl = g / 10, r = 16 * (g % 10) + (lane >> 2);
      const int c = (lane & 3) ^ swz(r);
      boffs[j] = (unsigned)((long long)r * kb_total * ROW_KB + pl * 64 + 16 * c);
    }
    // per-tile sources (tile k of this workgroup)
    auto a_base = [&](int k, unsigned (&aoff)[NAP]) -> __amdgpu_buffer_rsrc_t {
      long long mt;
      int nt;
      conv_tile_of(p, blockIdx.x + (unsigned)k * gstep, nv, mt, nt);
      const long long m0 = mt * G::BM;
#pragma unroll
      for (int i = 0; i < NAP; ++i) {
        const int P = min(pw + 4 * i, G::PIECES - 1), g = P >> 1, pl = P & 1;
        const int r = 16 * g + (lane >> 2);
        const long long m = min(m0 + r, last_row);
        const int c = (lane & 3) ^ swz(r);
        aoff[i] = (unsigned)((m - m0) * lda_kb * ROW_KB + pl * 64 + 16 * c);
      }
      return __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.A + m0 * lda_kb * ROW_KB), (short)0, 0x7fffffff,
                                               0x00020000);
    };
    auto b_base = [&](int k) -> __amdgpu_buffer_rsrc_t {
      long long mt;
      int nt;
      conv_tile_of(p, blockIdx.x + (unsigned)k * gstep, nv, mt, nt);
      return __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.Bp + (long long)nt * GBN * kb_total * ROW_KB),
                                               (short)0, 0x7fffffff, 0x00020000);
    };
    unsigned aoff_c[NAP], aoff_n[NAP];
    __amdgpu_buffer_rsrc_t ars_c = a_base(0, aoff_c), ars_n = ars_c;
    __amdgpu_buffer_rsrc_t brs_c = b_base(0), brs_n = brs_c;
    if (ntile > 1) {
      ars_n = a_base(1, aoff_n);
      brs_n = b_base(1);
    } else {
#pragma unroll
      for (int i = 0; i < NAP; ++i) aoff_n[i] = aoff_c[i];
    }
    auto issue_a = [&](const __amdgpu_buffer_rsrc_t& rs, const unsigned (&aoff)[NAP], int chunk, int gchunk, int i0,
                       int ni) {
      char* base = aslab + (gchunk & 1) * G::ASLAB;
      const int src_chunk = (TM & 8) ? 0 : chunk;
      for (int i = i0; i < i0 + ni; ++i) {
        const int P = min(pw + 4 * i, G::PIECES - 1);
        char* dst = base + (P & 1) * G::APLANE + (P >> 1) * 1024;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)dst, 16, aoff[i], (unsigned)(src_chunk * ROW_KB), 0, 0);
      }
    };
    // B of global stage gs into its ring slot; past this workgroup's last stage the data is the
    // last stage's again (dummy reissues keep every stage's piece count uniform for the counted
    // vmcnt; they land in the slots of stages that never come, never in the last stage's slot,
    // which wave 3's epilogue uses)
    const long long gs_last = (long long)ntile * nk - 1;
    auto issue_b = [&](long long gs, int kt) {
      char* base = bring + (int)(gs % NSB) * H3C_BSTAGE;
      if (gs > gs_last) gs = gs_last;
      const int k = (int)(gs / nk), s = (TM & 8) ? 0 : (int)(gs - (long long)k * nk);
      const __amdgpu_buffer_rsrc_t& rs = k == kt ? brs_c : brs_n;
#pragma unroll
      for (int j = 0; j < 5; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(base + (pw + 4 * j) * 1024), 16, boffs[j],
                                                 (unsigned)(s * ROW_KB), 0, 0);
    };
    issue_a(ars_c, aoff_c, 0, 0, 0, NAP);
    issue_b(0, 0);
    issue_b(1, 0);
    issue_b(2, 0);
    asm volatile("s_waitcnt vmcnt(5)" ::: "memory");    // stages 0 and 1 landed
    __builtin_amdgcn_s_barrier();
    for (int kt = 0; kt < ntile; ++kt) {
      if (kt > 0) {
        __builtin_amdgcn_s_barrier();                   // E: the consumers' epilogue left the LDS
        ars_c = ars_n;
        brs_c = brs_n;
#pragma unroll
        for (int i = 0; i < NAP; ++i) aoff_c[i] = aoff_n[i];
        if (kt + 1 < ntile) {
          ars_n = a_base(kt + 1, aoff_n);
          brs_n = b_base(kt + 1);
        }
      }
      for (int c = 0; c < nchunk; ++c) {
        const int gc = kt * nchunk + c;
        const bool last_c = c + 1 == nchunk;
        const bool more_a = !(TM & 2) && (!last_c || kt + 1 < ntile);
        for (int t = 0; t < 8; ++t) {
          const long long gs = (long long)kt * nk + c * 8 + t;
          if (more_a && t < 6) {                        // slab pieces 2,2,2,1,1,1,0,0
            const int i0 = t < 3 ? 2 * t : t + 3, ni = t < 3 ? 2 : 1;
            if (last_c)
              issue_a(ars_n, aoff_n, 0, gc + 1, i0, ni);   // the next tile's chunk 0
            else
              issue_a(ars_c, aoff_c, c + 1, gc + 1, i0, ni);
          }
          if (!(TM & 2)) issue_b(gs + NSB - 1, kt);
          asm volatile("s_waitcnt vmcnt(5)" ::: "memory");   // all but this stage's pieces
          __builtin_amdgcn_s_barrier();
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return;
  }

  // ---------------- consumer: LDS reads, MFMAs, epilogue ----------------
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
  __builtin_amdgcn_s_barrier();                         // slab 0 and B stages 0, 1 landed
  asm volatile("" ::: "memory");
  bf16x8 as[4][3];
  bf16x8 b0[3], b1[3];
  for (int kt = 0; kt < ntile; ++kt) {
    long long mt;
    int nt;
    conv_tile_of(p, blockIdx.x + (unsigned)kt * gstep, nv, mt, nt);
    const long long m0 = mt * G::BM;
    const int n0 = nt * GBN;
    floatx4v acc[4][10];
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
      for (int nb = 0; nb < 10; ++nb)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[mb][nb][r] = 0.f;
    const long long gs0 = (long long)kt * nk;
    read_a(aslab + ((kt * nchunk) & 1) * G::ASLAB, 0, as);
    read_b(bring + (int)(gs0 % NSB) * H3C_BSTAGE, 0, b0);
    for (int c = 0; c < nchunk; ++c) {
      const int gc = kt * nchunk + c;
      const char* slab = aslab + (gc & 1) * G::ASLAB;
      for (int t = 0; t < 8; ++t) {
        const long long gs = gs0 + c * 8 + t;
        const char* base = bring + (int)(gs % NSB) * H3C_BSTAGE;
        const bool tile_end = c + 1 == nchunk && t == 7;
#pragma unroll
        for (int nb = 0; nb < 10; ++nb) {
          if (nb + 1 < 10) read_b(base, nb + 1, (nb & 1) ? b0 : b1);
#pragma unroll
          for (int mb = 0; mb < 4; ++mb) acc[mb][nb] = planes_mfma<2>(acc[mb][nb], as[mb], (nb & 1) ? b1 : b0);
          pin();
        }
        if (!tile_end) {      // next stage's first fragments (landed at barrier s-1), read before barrier s
          if (t < 7)
            read_a(slab, t + 1, as);
          else
            read_a(aslab + ((gc + 1) & 1) * G::ASLAB, 0, as);   // next slab landed by tap 6's barrier
          read_b(bring + (int)((gs + 1) % NSB) * H3C_BSTAGE, 0, b0);
        }
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
    }
    // epilogue: waves 0-2 stage in the slab of the tile's last chunk, wave 3 in its last B slot
    const long long gl = gs0 + nk - 1;
    char* e = wave < 3 ? aslab + ((kt * nchunk + nchunk - 1) & 1) * G::ASLAB + wave * 16 * H3E_ROW
                       : bring + (int)(gl % NSB) * H3C_BSTAGE;
    if constexpr ((TM & 2048) != 0) {   // timing probe (wrong results): no epilogue, one store per lane
      float t = 0.f;
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < 10; ++nb) t += acc[mb][nb][0] + acc[mb][nb][1] + acc[mb][nb][2] + acc[mb][nb][3];
      p.C[(m0 + wave * 64 + lane) % p.M] = t;
    } else if constexpr (EPI == EPI_RELU) {
      epilogue_relu_h2_q16(p, acc, m0 + wave * 64, n0, lane, e);
    } else {
      epilogue_pool_h2_lds<4, LAYER == 4>(p, acc, m0 + wave * 64, n0, lane, e);
    }
    if (kt + 1 < ntile) __builtin_amdgcn_s_barrier();   // E
  }
}

template <int LAYER, int EPI, int TM = 0>
__global__ __launch_bounds__(512, 1) void beluga_conv_h3pp(GemmArgs p) {
  __shared__ __attribute__((aligned(1024))) char smem[h3c_lds<4>()];
  gemm_conv_h3pp_body<LAYER, EPI, TM>(p, smem);
}


// ---- timing probe (wrong results): the producer / consumer conv kernel with 32x32x16 MFMAs ----
// beluga_conv_h3p with each consumer unit's 12 v_mfma_f32_16x16x32_f16 issued as 6
// v_mfma_f32_32x32x16_f16 on the same fragment registers: the same FLOPs, LDS reads, loads and
// epilogue (fed the 32x32 accumulators as they lie), so gemm_bench compares the two MFMA forms at
// equal data movement (MI355X_MICROARCH.md 'DVFS give-back' item 7).
typedef float floatx16v __attribute__((ext_vector_type(16)));
template <int LAYER, int EPI, int TM, int NSB>
__device__ __forceinline__ void gemm_conv_h3p32_body(const GemmArgs& p, char* smem) {
  static_assert(NSB == 3 || NSB == 4, "B ring depth");
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
  const int n0 = nt * GBN;
  const int kb_total = (int)(p.ldb / GBK);
  const long long lda_kb = p.lda / GBK;
  const int nchunk = (int)lda_kb;
  const int nk = nchunk * 8;
  auto swz = [](int r) { return conv_swz<TM>(r); };
  char* const aslab = smem;
  char* const bring = smem + 2 * G::ASLAB;

  if (wave >= 4) {
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
    unsigned boff[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const int g = pw + 4 * j;
      const int pl = g / 10, r = 16 * (g % 10) + (lane >> 2);
      const int c = (lane & 3) ^ swz(r);
      boff[j] = (unsigned)((long long)r * kb_total * ROW_KB + pl * 64 + 16 * c);
    }
    const __amdgpu_buffer_rsrc_t arsrc = __builtin_amdgcn_make_buffer_rsrc((void*)Ab, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t brsrc = __builtin_amdgcn_make_buffer_rsrc((void*)Bb, (short)0, 0x7fffffff, 0x00020000);
    auto issue_a = [&](int chunk, int i0, int ni) {
      char* base = aslab + (chunk & 1) * G::ASLAB;
      const int src_chunk = (TM & 8) ? 0 : chunk;
      for (int i = i0; i < i0 + ni; ++i) {
        const int P = min(pw + 4 * i, G::PIECES - 1);
        char* dst = base + (P & 1) * G::APLANE + (P >> 1) * 1024;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(arsrc, (lds_void*)dst, 16, aoff[i], (unsigned)(src_chunk * ROW_KB), 0, 0);
      }
    };
    auto issue_b = [&](int s, int slot) {
      if constexpr ((TM & 8) != 0) s = 0;
      char* base = bring + slot * H3C_BSTAGE;
#pragma unroll
      for (int j = 0; j < 5; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(brsrc, (lds_void*)(base + (pw + 4 * j) * 1024), 16, boff[j],
                                                 (unsigned)(s * ROW_KB), 0, 0);
    };
    issue_a(0, 0, NAP);
    issue_b(0, 0);
    issue_b(min(1, nk - 1), 1);
    if constexpr (NSB == 4) {
      issue_b(min(2, nk - 1), 2);
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
        // everything but the B pieces of the last NSB-2 stages: B(s+1), and slab c+1 by tap 7
        // (PF: all but this stage's pieces, so B(s+2) has landed at barrier s and the
        // consumers read stage s+1's first fragments before that barrier)
        if constexpr (NSB == 4 && !PF)
          asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
        else
          asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        slot = slot + 1 == NSB ? 0 : slot + 1;
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (EPI == EPI_RELU || EPI == EPI_RELU_POOL4) {
      __builtin_amdgcn_s_barrier();                    // consumers' epilogue reuses the LDS
    }
    return;
  }

  // ---------------- consumer: LDS reads and MFMAs ----------------
  floatx16v acc32[2][5];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int cb = 0; cb < 5; ++cb)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc32[rb][cb][r] = 0.f;
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
  auto pin = [&]() {   // 6 MFMAs of 32 cycles per unit
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
    }
  };
  __builtin_amdgcn_s_barrier();                       // slab 0 and B stage 0 landed
  asm volatile("" ::: "memory");
  bf16x8 as[4][3];
  bf16x8 b0[3], b1[3];
  read_a(aslab, 0, as);
  if constexpr (PF) read_b(bring, 0, b0);
  int slot = 0;
  for (int c = 0; c < nchunk; ++c) {
    const char* slab = aslab + (c & 1) * G::ASLAB;
    for (int t = 0; t < 8; ++t) {
      const char* base = bring + slot * H3C_BSTAGE;
      const int nslot = slot + 1 == NSB ? 0 : slot + 1;
      if constexpr (!PF) read_b(base, 0, b0);
#pragma unroll
      for (int nb = 0; nb < 10; ++nb) {
        if (nb + 1 < 10) read_b(base, nb + 1, (nb & 1) ? b0 : b1);
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {   // unit nb = 2 cb + h: k-half h of column block cb
          const bf16x8(&b)[3] = (nb & 1) ? b1 : b0;
          const bf16x8(&a)[3] = as[2 * rb + (nb & 1)];
          floatx16v& c = acc32[rb][nb >> 1];
          c = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(halfx8, a[1]), __builtin_bit_cast(halfx8, b[0]), c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(halfx8, a[0]), __builtin_bit_cast(halfx8, b[1]), c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(halfx8, a[0]), __builtin_bit_cast(halfx8, b[0]), c, 0, 0, 0);
        }
        pin();
      }
      if (t < 7)
        read_a(slab, t + 1, as);   // slab reads stay in flight across the barrier
      else if (PF && c + 1 < nchunk)
        read_a(aslab + ((c + 1) & 1) * G::ASLAB, 0, as);   // next slab landed by tap 6's barrier
      if constexpr (PF) {
        if (c * 8 + t + 1 < nk) read_b(bring + nslot * H3C_BSTAGE, 0, b0);   // stage s+1 landed at barrier s-1
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      slot = nslot;
    }
    if (!PF && c + 1 < nchunk) read_a(aslab + ((c + 1) & 1) * G::ASLAB, 0, as);
  }
  floatx4v acc[4][10];
  __builtin_memcpy(acc, acc32, sizeof(acc));
  if constexpr ((TM & 2048) != 0) {   // timing probe (wrong results): no epilogue, one store per lane
    __builtin_amdgcn_s_barrier();
    float t = 0.f;
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
      for (int nb = 0; nb < 10; ++nb) t += acc[mb][nb][0] + acc[mb][nb][1] + acc[mb][nb][2] + acc[mb][nb][3];
    p.C[(m0 + wave * 64 + lane) % p.M] = t;
    return;
  }
  if constexpr (EPI == EPI_RELU || EPI == EPI_RELU_POOL4) {
    __builtin_amdgcn_s_barrier();                     // producers drained their tail pieces
    if constexpr (EPI == EPI_RELU)
      epilogue_relu_h2_lds<4, (TM & 8192) == 0>(p, acc, m0 + wave * 64, n0, lane, smem + wave * H3E_WAVE);
    else
      epilogue_pool_h2_lds<4, LAYER == 4, (TM & 8192) == 0>(p, acc, m0 + wave * 64, n0, lane, smem + wave * H3E_WAVE);
  } else {
    gemm_epilogue16<EPI, 2, 10, 4>(p, acc, m0 + wave * 64, n0, 0, lane);
  }
}


template <int LAYER, int EPI, int TM = 0, int NSB = 4>
__global__ __launch_bounds__(512, 1) void beluga_conv_h3p32(GemmArgs p) {
  __shared__ __attribute__((aligned(1024))) char smem[h3c_lds<NSB>()];
  gemm_conv_h3p32_body<LAYER, EPI, TM, NSB>(p, smem);
}

}  // namespace expecto
