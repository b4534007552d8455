// gram_rs.hpp -- the FmtH2 distance Gram with split roles (VERDICT r5 next
// #1: "take the Gram's D stores and epilogue off the MFMA wave").
//
// gram_w1_kernel (gram_w1.hpp) runs ONE wave per SIMD that issues the MFMAs
// and, between them, the previous tile's epilogue (D value, bracket
// accounting, 16-byte D stores).  Its counters on MI355X (profiles/r14a):
// 5.4 VALU + 0.9 LDS + 0.7 SALU + 0.4 VMEM instructions per 32-cycle MFMA,
// i.e. about 30 of the 32 issue cycles one wave has per MFMA (an MFMA holds
// vector issue for 8, a VALU op of a lone wave takes 4) -- issue-bound, and
// every store that waits for queue space stalls the only wave that feeds the
// matrix pipe: 42 % MFMA-busy.
//
// Here each SIMD runs two waves of one 512-thread workgroup:
//   * an M wave (waves 0-3) issues only the MFMAs of the unit's 64 columns it
//     owns (the same 128 x 64 tile, fragments, product order and K-step
//     pipeline as gram_w1, so D is bit-identical) plus its B-fragment loads
//     and LDS fragment reads; at the tile's end it writes its 128
//     accumulators per lane to an LDS hand-off buffer (32 ds_write_b128,
//     1 KiB each, conflict-free) and starts the next tile.  The strip's A
//     image reaches LDS by LDS-DMA the M waves issue two K-steps ahead (a
//     3-stage ring);
//   * an E wave (waves 4-7), during the next tile's 16 K-steps, runs the
//     hand-off's epilogue one slice per K-step:
//     the D value, the bracket accounting, the permlane pairing and the
//     16-byte nt stores of gram_w1, reading the accumulators from LDS in the
//     M wave's own lane layout.
// The two waves of a SIMD interleave dynamically: two waves can issue a VALU
// op every 2 cycles where one wave needs 4, so the epilogue's VALU fits in the
// issue cycles the MFMAs leave, and an E wave parked on a full store queue no
// longer stops the MFMAs.  M waves run at priority 1 (MI355X_MICROARCH.md
// "static priority").
//
// LDS: 3 x 8 KiB A stages + 4 x 32 KiB hand-off = 152 KiB: one block per CU.
// The bracket's candidate stage reuses the hand-off chunks a slice has
// already read (depth 128, one flush per tile instead of one per slice: the
// per-slice flush's LDS read latency was most of the E wave's time).  Registers: <= 256 per wave (waves_per_eu 2): the M wave holds one
// accumulator set (128), two fragment sets (64) and a two-deep B ring (32).
//
// Barriers: one per K-step (the A stage, as in gram_w1), plus two per tile
// around the hand-off (X: the E waves have read the previous tile's last
// slice; Y: the M waves' writes have landed).
#pragma once
#include <cfloat>

#include "gram_w1.hpp"

namespace dsvgd {

struct GramRS {
  static constexpr int kThreads = 512;
  static constexpr int BM = 128;
  static constexpr int P = 2;
  static constexpr int SA = P * BM * 32;            // one K-step of the strip's image (8 KiB)
  static constexpr int kHWave = 128 * 64 * 4;       // one M wave's accumulators (32 KiB)
  static constexpr int kHOff = 3 * SA;               // 3 A stages, then the hand-off
  static constexpr int kSOff = kHOff + 4 * kHWave;  // the last slice's candidate stage
  static constexpr int kSmemBytes = kSOff + 4 * 64 * 8 * 4;
  static constexpr int kSlots = 4;                  // candidate slots per unit (one per E wave)
};
static_assert(GramRS::kSmemBytes <= 160 * 1024, "gram_rs LDS");  // exactly 160 KiB

// OUT = 1: the W2 cost matrix (dsvgd_w2_cost_h2) -- D row-major with leading
// dimension ldc instead of the panel layout, and every entry whose Gram form
// may have cancelled (C < tau (|x_i - c|^2 + |y_j - c|^2)) recomputed from
// explicit fp32 differences of the raw rows in w2_cost_kernel's order (the
// same bits as the VALU cost tiles there)
struct W2Out {
  const float* X = nullptr;   // m rows (the Gram's rows), ldx
  const float* Y = nullptr;   // n rows (its columns), ldy
  int64_t ldx = 0, ldy = 0, ldc = 0;
  int d = 0;
  float tau = 0.f;
  int vec = 0;                // rows 16-byte aligned and d % 4 == 0: 16-byte loads
  // stat[0]: the largest entry's bits, stat[1]: 1 if an entry is not finite
  // (what w2_cmax_kernel finds in a pass over C; zeroed by the caller)
  uint32_t* stat = nullptr;
  int nt = 1;                 // C's stores non-temporal (dsvgd_w2_set_cost_nt)
  int lines = 1;              // C's stores as whole 128-byte lines (dsvgd_w2_set_cost_lines)
};

// VAR (timing probes, dsvgd_gram_set_rs(5 / 6 / 7)): 4 = the E waves skip
// the epilogue (D is not written) -- the MFMA waves' own rate; 8 = the M
// waves skip the MFMAs (D is wrong) -- the epilogue waves' own rate; 16 = the
// E waves at priority 1 instead of the M waves; 32 = barrier stamps (below);
// 64 = the M waves' B ring 4 deep (B two K-steps ahead)
template <int smode, bool SYM, int OUT = 0, int VAR = 0, int KG = GramW1::kGroup>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void gram_rs_kernel(
    const _Float16* __restrict__ Yg, int64_t img_rows, const float* __restrict__ norms,
    const float* __restrict__ rsc, int64_t row0, int64_t m, int64_t n, int64_t n_pad, int nk,
    float* __restrict__ D, dsvgd_select_state* __restrict__ st, float* __restrict__ cand,
    int64_t total_units, int Tm, int Tc, int jp_off, int64_t slot_base, int64_t ns_total,
    int w2all = 0, const float* __restrict__ gate = nullptr, W2Out wo = W2Out{}) {
  static_assert(OUT == 0 || (smode == kSelNone && !SYM), "the W2 cost form: no select, no symmetry");
  using V8 = FmtH2::V8;
  constexpr bool kBr = smode == kSelBracket;
  __builtin_assume(nk >= 16 && nk % 16 == 0);  // checked by the host
  __shared__ __attribute__((aligned(16))) char smem[GramRS::kSmemBytes];
  const int t = threadIdx.x, lane = t & 63, r = lane & 31, h = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
  const bool mwave = wv < 4;
  const int w = wv & 3;  // the 64 columns of the unit this wave computes / writes out
  const int T = (int)(n_pad >> 7);

  const int64_t x = blockIdx.x % kXcds, u = blockIdx.x / kXcds, U = gridDim.x / kXcds;
  int64_t units = total_units;
  if constexpr (smode == kSelNone) units = (gate && *gate == 0.f) ? 0 : total_units;
  const int64_t q = units / kXcds, rr = units % kXcds;
  const int64_t lo = x * q + min(x, rr);
  const int64_t hi = (int64_t)__builtin_amdgcn_readfirstlane((int)(lo + q + (x < rr ? 1 : 0)));
  SlotLayout sl(cand, ns_total, kBr ? st->cand_cap : 0);
  if (kBr) sl.publish(st, blockIdx.x);

  GramUnitWalk walk(Tm, Tc, SYM, KG);
  // skipped units' slots are zeroed by the E waves only (one writer per slot)
  auto next_valid = [&](int64_t L, int& I, int& J2) -> int64_t {
    for (; L < hi; L += U) {
      if (walk.at(L, I, J2)) {
        I = __builtin_amdgcn_readfirstlane(I);
        J2 = __builtin_amdgcn_readfirstlane(J2);
        return L;
      }
      if (kBr && !mwave) {
        sl.cnt[slot_base + L * GramRS::kSlots + w] = 0u;
        sl.below[slot_base + L * GramRS::kSlots + w] = 0u;
      }
    }
    return L;
  };
  struct Unit {
    int64_t L;
    int I, J2;
  };
  int I0 = 0, J0 = 0;
  const int64_t L0 = next_valid((int64_t)__builtin_amdgcn_readfirstlane((int)(lo + u)), I0, J0);
  if (L0 >= hi) return;  // block-uniform
  Unit cur{L0, I0, J0};
  int In = 0, Jn = 0;
  const int64_t Ln = next_valid(L0 + U, In, Jn);
  Unit nxt{Ln < hi ? Ln : L0, Ln < hi ? In : I0, Ln < hi ? Jn : J0};
  bool has_next = Ln < hi;
  auto advance = [&]() {
    cur = nxt;
    int I2 = 0, J22 = 0;
    const int64_t L2 = next_valid(cur.L + U, I2, J22);
    has_next = L2 < hi;
    if (has_next) nxt = Unit{L2, I2, J22};
  };

  const int pstride = (int)(img_rows * 32);  // bytes of one part of one image K-step
  // workgroup-wide: LDS writes landed, every wave past its LDS reads
  // VAR & 32 (a timing probe): each wave of blocks 0-7 stamps the shader
  // clock on arriving at and leaving every barrier into wo.X (int64
  // [block][wave][512]); lane 0's vector store
  int ev = 0;
  auto stamp = [&]() {
    if constexpr ((VAR & 32) != 0) {
      const int64_t tnow = (int64_t)__builtin_amdgcn_s_memtime();
      if (blockIdx.x < 8 && ev < 512 && lane == 0)
        reinterpret_cast<int64_t*>(const_cast<float*>(wo.X))[(blockIdx.x * 8 + wv) * 512 + ev] = tnow;
      ++ev;
    }
  };
  auto barrier = [&]() {
    stamp();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    stamp();
  };
  float* const hbuf = reinterpret_cast<float*>(smem + GramRS::kHOff + w * GramRS::kHWave);

  // the strip's image rows of unit un (K-step part 0 at byte 0, part 1 at pstride)
  auto rsrc_A = [&](const Unit& un) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)(Yg + (row0 + (int64_t)un.I * 128) * 16),
                                             (short)0, 0x7fffffff, 0x00020000);
  };

  if (mwave) {
    // =================== M wave: MFMAs only ===================
    // The strip's A image goes to a 3-stage LDS ring by LDS-DMA issued by the
    // M waves themselves (16-byte chunk t of a K-step's 8 KiB per thread, the
    // gram_w1 staging map): their vmcnt queue holds only loads, so waiting
    // for a stage never waits for an epilogue store.  A(k + 2) is issued at
    // the start of K-step k into the stage A(k - 1) left (read before the
    // last barrier), waited for at the barrier of K-step k + 1.
    if constexpr (!(VAR & 16)) __builtin_amdgcn_s_setprio(1);
    const int vB = x3_off(r, h);
    const int voffA = (t >> 1) * 32 + (t & 1) * 16;
    const int voffA1 = voffA + (int)img_rows * 32;
    auto rsrc_B = [&](const Unit& un) {
      return __builtin_amdgcn_make_buffer_rsrc(
          (void*)(Yg + ((int64_t)(un.J2 + jp_off) * 256 + 64 * w) * 16), (short)0, 0x7fffffff,
          0x00020000);
    };
    // VAR & 64: a 4-deep ring, B issued two K-steps ahead (probe 9)
    constexpr int kRB = (VAR & 64) ? 4 : 2;
    V8 rb[kRB][2][2];  // [ring][bj][part]
    auto load_B = [&](int sb, int kk) {  // step kk's B (kk >= nk: the next unit's)
      const bool nx = kk >= nk;
      const int ks = nx ? (has_next ? kk - nk : nk - 1) : kk;
      const __amdgpu_buffer_rsrc_t rB = rsrc_B(nx && has_next ? nxt : cur);
      const int so = ks * 2 * pstride;
#pragma unroll
      for (int bj = 0; bj < 2; ++bj)
#pragma unroll
        for (int p = 0; p < 2; ++p)
          rb[sb][bj][p] = __builtin_bit_cast(V8, gw1_load(rB, vB + bj * 1024, so + p * pstride));
    };
    auto dma_A = [&](int kk, int stg) {  // step kk's A (kk >= nk: the next unit's) -> stage stg
      const bool nx = kk >= nk;
      const int ks = nx ? (has_next ? kk - nk : nk - 1) : kk;
      const __amdgpu_buffer_rsrc_t rA = rsrc_A(nx && has_next ? nxt : cur);
      const int so = ks * 2 * pstride;
      char* dst = smem + stg * GramRS::SA + w * 64 * 16;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rA, (__attribute__((address_space(3))) void*)dst, 16, voffA, so, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rA, (__attribute__((address_space(3))) void*)(dst + GramRS::BM * 32), 16, voffA1, so, 0, 0);
    };
    V8 af[2][4][2];
    auto read_frags = [&](V8 (&a)[4][2], const char* st_) {
#pragma unroll
      for (int bi = 0; bi < 4; ++bi)
#pragma unroll
        for (int p = 0; p < 2; ++p)
          a[bi][p] = *reinterpret_cast<const V8*>(st_ + p * GramRS::BM * 32 + x3_off(32 * bi + r, h));
    };
    int sD = 2, sR = 1;  // the stages of the next A DMA and of the next fragment read
    auto nxt3 = [](int v) { return v == 2 ? 0 : v + 1; };
    f32x16 acc[4][2];
    // one K-step: 24 MFMAs in gram_w1's order (product p of block idx % 8,
    // consecutive MFMAs independent); the next step's B and the A two steps
    // ahead issued in the first group, the barrier and the next step's
    // fragments at mid-step
    auto step = [&](auto KS_, auto FIRST_, int k) {
      constexpr int KS = decltype(KS_)::value;
      constexpr bool FIRST = decltype(FIRST_)::value;
      V8 (&a)[4][2] = af[KS & 1];
#pragma unroll
      for (int grp = 0; grp < 8; ++grp) {
#pragma unroll
        for (int qq = 0; qq < 3; ++qq) {
          const int idx = 3 * grp + qq, p = idx / 8, bi = (idx % 8) >> 1, bj = idx & 1;
          f32x16 c = (p == 0 && FIRST) ? f32x16{} : acc[bi][bj];
          const V8 bx = rb[KS & (kRB - 1)][bj][p == 1 ? 1 : 0];
          const V8 ax = a[bi][p == 0 ? 1 : 0];
          if constexpr (VAR & 8)
            acc[bi][bj] = c;
          else
            acc[bi][bj] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bx, ax, c, 0, 0, 0);
        }
        if (grp == 0) {
          if constexpr (kRB == 4)
            load_B((KS + 2) & 3, k + 2);
          else
            load_B((KS + 1) & 1, k + 1);
          dma_A(k + 2, sD);
          sD = nxt3(sD);
        }
        if (grp == 3) {
          // A(k + 1)'s DMA (issued last K-step) landed: only this step's four
          // B loads and two A DMAs are younger (4-deep ring: the four of
          // B(k + 2); B(k + 1), issued last step, older than A(k + 1)'s DMA,
          // is waited for here too)
          __builtin_amdgcn_sched_barrier(0);
          asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
          barrier();
          read_frags(af[(KS + 1) & 1], smem + sR * GramRS::SA);
          sR = nxt3(sR);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    };
    // prologue: A(0) -> stage 0, A(1) -> stage 1, B(0)
    dma_A(0, 0);
    dma_A(1, 1);
    load_B(0, 0);
    if constexpr (kRB == 4) load_B(1, 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier();
    read_frags(af[0], smem);
    for (;;) {
#define DSVGD_GRS_STEP(KK) \
  step(std::integral_constant<int, (KK) & 3>{}, std::integral_constant<bool, KK == 0>{}, KK);
      DSVGD_GRS_STEP(0) DSVGD_GRS_STEP(1) DSVGD_GRS_STEP(2) DSVGD_GRS_STEP(3)
      DSVGD_GRS_STEP(4) DSVGD_GRS_STEP(5) DSVGD_GRS_STEP(6) DSVGD_GRS_STEP(7)
      DSVGD_GRS_STEP(8) DSVGD_GRS_STEP(9) DSVGD_GRS_STEP(10) DSVGD_GRS_STEP(11)
      DSVGD_GRS_STEP(12) DSVGD_GRS_STEP(13) DSVGD_GRS_STEP(14) DSVGD_GRS_STEP(15)
#undef DSVGD_GRS_STEP
      for (int k = 16; k < nk; k += 4) {
        constexpr std::integral_constant<bool, false> later{};
        step(std::integral_constant<int, 0>{}, later, k);
        step(std::integral_constant<int, 1>{}, later, k + 1);
        step(std::integral_constant<int, 2>{}, later, k + 2);
        step(std::integral_constant<int, 3>{}, later, k + 3);
      }
      // hand-off: X (the E waves are done with the previous tile's last
      // slice), the accumulators in the lane layout (chunk c = 4 (2 bi + bj)
      // + q holds registers 4q .. 4q + 3 of block (bi, bj)), Y (landed)
      barrier();
#pragma unroll
      for (int bi = 0; bi < 4; ++bi)
#pragma unroll
        for (int bj = 0; bj < 2; ++bj)
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            const int c = 4 * (2 * bi + bj) + qq;
            const f32x16 v = acc[bi][bj];
            *reinterpret_cast<f32x4*>(hbuf + (c * 64 + lane) * 4) =
                f32x4{v[4 * qq], v[4 * qq + 1], v[4 * qq + 2], v[4 * qq + 3]};
          }
      barrier();
      if (!has_next) break;
      advance();
    }
    return;
  }

  // =================== E wave: the epilogue ===================
  // The epilogue state of the tile being written out ("active") and the raw
  // row / column data of the tile the M waves are computing ("pending",
  // loaded early in that tile so the hand-off at its end waits for no load).
  // Each lane's columns are 32 bj + 8 g + 4 h + e (bj < 2, g < 4, e < 4): 32
  // per lane, kept in registers (no LDS column table).
  float nr[4], si2[4];
  uint32_t vrow = 0u, vcol = 0u;  // OUT 1: the real rows (bit bi) / columns (16 bj + 4 g + e)
  uint32_t cmx = 0u;              // OUT 1: the largest real entry's bits so far
  bool cbad = false;
  int tg[4];
  f32x4 cnA[2][4], csA[2][4];
  __amdgpu_buffer_rsrc_t rD = __builtin_amdgcn_make_buffer_rsrc((void*)D, (short)0, 0, 0x00020000);
  int64_t eslot = -1;
  int64_t ei0 = 0, ej0 = 0;   // OUT 1: the tile's first row (of X) and column (of Y)
  bool ew2 = false, ediag = false;
  float pn[4], pr[4];
  f32x4 pcn[2][4], pcr[2][4];
  Unit pend = cur;
  // the candidate stage is the hand-off region itself: slice SL has read
  // chunks 2 SL, 2 SL + 1 (4 levels of 64 lanes each) and stages levels
  // <= 8 SL + 7, so every level lands in an already-read chunk; one flush per
  // tile, before X (where the M waves overwrite the region)
  GramSlotWriter<128> sw;
  float* const cstage = reinterpret_cast<float*>(hbuf);
  // slice 15 runs after X (the M waves already overwriting the hand-off):
  // its candidates go to a stage of their own, depth 8
  float* const sstage = reinterpret_cast<float*>(smem + GramRS::kSOff) + w * 64 * 8;
  // the bracket is fixed for the launch: read once, not per tile
  uint32_t klo0 = 0x7FFFFFFFu, kspan0 = 0u;
  if constexpr (kBr) {
    const float blo = st->lo, bhi = st->hi;
    const bool ok = bhi >= blo && blo >= 0.f;  // as SlotWriterLdsT::begin
    klo0 = ok ? __float_as_uint(blo) : 0x7FFFFFFFu;
    kspan0 = ok ? __float_as_uint(bhi) - klo0 : 0u;
  }
  // in three parts (K-steps 8, 10, 12: one batch of 24 loads had the E wave
  // arrive ~1600 cycles late at its barrier, profiles/r14n; each part, the
  // previous slot's close (K-step 3) and the walk's advance (K-step 5) in a
  // K-step of its own, where the wave has ~400 cycles of slack)
  auto prefetch_epi = [&](const Unit& un, auto PART_) {
    constexpr int PART = decltype(PART_)::value;
    const __amdgpu_buffer_rsrc_t rN =
        __builtin_amdgcn_make_buffer_rsrc((void*)norms, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rS =
        __builtin_amdgcn_make_buffer_rsrc((void*)rsc, (short)0, 0x7fffffff, 0x00020000);
    if constexpr (PART == 0) {
      pend = un;
#pragma unroll
      for (int bi = 0; bi < 4; ++bi) {
        // rows past m read row 0's data (clamped); activate() masks them
        const int64_t il = (int64_t)un.I * 128 + 32 * bi + r;
        const int64_t gi = row0 + (il < m ? il : 0);
        pn[bi] = norms[gi];
        pr[bi] = rsc[gi];
      }
    } else {
      constexpr int bj = PART - 1;
      const int64_t gj0 = (int64_t)(pend.J2 + jp_off) * 256 + 64 * w;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        // columns >= n read whatever lies there (the image's slack rows): masked below
        const int c = (int)(gj0 + 32 * bj + 8 * g + 4 * h);
        pcn[bj][g] = gw1_load(rN, c * 4, 0);
        pcr[bj][g] = gw1_load(rS, c * 4, 0);
      }
    }
  };
  auto activate = [&]() {
    const Unit& un = pend;
    const int64_t gi0 = row0 + (int64_t)un.I * 128;
    const int64_t gj0 = (int64_t)(un.J2 + jp_off) * 256 + 64 * w;
    const int Jt = (int)(gj0 >> 7);
    const bool valid = Jt < T && (!SYM || Jt >= un.I);
#pragma unroll
    for (int bi = 0; bi < 4; ++bi) {
      const int64_t il = (int64_t)un.I * 128 + 32 * bi + r;
      const bool ok = valid && il < m;
      nr[bi] = ok ? pn[bi] : INFINITY;
      if constexpr (OUT == 1) vrow = bi == 0 ? (ok ? 1u : 0u) : (vrow | (ok ? 1u << bi : 0u));
      si2[bi] = 2.f * pow2_inv(ok ? pr[bi] : 1.f);
      tg[bi] = ok ? (int)(gi0 + 32 * bi + r - gj0) - 4 * h : (1 << 20);
    }
    if (gj0 + 64 <= n) {  // (wave-uniform) every column of the tile is real
#pragma unroll
      for (int bj = 0; bj < 2; ++bj)
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            cnA[bj][g][e] = pcn[bj][g][e];
            csA[bj][g][e] = pow2_inv(pcr[bj][g][e]);
          }
      if constexpr (OUT == 1) vcol = ~0u;
    } else {
      if constexpr (OUT == 1) vcol = 0u;
      const int nl = (int)(n - gj0);  // < 64
#pragma unroll
      for (int bj = 0; bj < 2; ++bj)
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const bool ok = 32 * bj + 8 * g + 4 * h + e < nl;
            cnA[bj][g][e] = ok ? pcn[bj][g][e] : INFINITY;
            csA[bj][g][e] = pow2_inv(ok ? pcr[bj][g][e] : 1.f);
            if constexpr (OUT == 1) vcol |= ok ? 1u << (16 * bj + 4 * g + e) : 0u;
          }
    }
    if constexpr (OUT == 1) {
      // rows I*128 .. +128 (the caller's C has roundup(m, 128) rows), the wave's 64 columns
      float* dt = D + (int64_t)un.I * 128 * wo.ldc + gj0;
      rD = __builtin_amdgcn_make_buffer_rsrc(
          (void*)dt, (short)0, valid ? (int)((127 * wo.ldc + 64) * 4) : 0, 0x00020000);
      ei0 = (int64_t)un.I * 128;
      ej0 = gj0;
    } else {
      float* dt = D + ((int64_t)un.I * (n_pad >> 4) + (int64_t)Jt * 8 + 4 * (w & 1)) * kPanelElems;
      rD = __builtin_amdgcn_make_buffer_rsrc((void*)dt, (short)0, valid ? 4 * kPanelElems * 4 : 0,
                                             0x00020000);
    }
    eslot = slot_base + un.L * GramRS::kSlots + w;
    ew2 = (SYM && Jt != un.I) || w2all != 0;
    ediag = valid && gj0 + 64 > gi0 && gj0 < gi0 + 128;
  };
  // the hand-off's values of slice SL: chunk c = 4 (2 bi + bj) + 2 (SL & 1), + 1
  f32x4 hv[2][2];
  auto read_h = [&](int SL, f32x4 (&dst)[2]) {
    const int c0 = 4 * (2 * (SL >> 2) + ((SL >> 1) & 1)) + 2 * (SL & 1);
    dst[0] = *reinterpret_cast<const f32x4*>(hbuf + (c0 * 64 + lane) * 4);
    dst[1] = *reinterpret_cast<const f32x4*>(hbuf + ((c0 + 1) * 64 + lane) * 4);
  };
  // slice SL (compile time): block (bi, bj) = (SL >> 2, (SL >> 1) & 1), register
  // runs g = 2 (SL & 1), + 1 -- gram_w1's slice() and store_slice() on values
  // read from the hand-off one slice ahead
  auto slice = [&](auto SL_, f32x4 (&v)[2]) {
    constexpr int SL = decltype(SL_)::value;
    constexpr int bi = SL >> 2, bj = (SL >> 1) & 1, g0 = 2 * (SL & 1);
    const float nrv = nr[bi], siv = si2[bi];
#pragma unroll
    for (int gg = 0; gg < 2; ++gg)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[gg][e] = fmaxf(0.f, (nrv + cnA[bj][g0 + gg][e]) - siv * (csA[bj][g0 + gg][e] * v[gg][e]));
        if constexpr (kBr) sw.add(v[gg][e]);
      }
    if constexpr (OUT == 1) {
      // near pairs: the explicit-difference cost, rare (the diagonal of an
      // SVGD-shaped plan).  All lanes at once, each lane one of its entries
      // per round (rounds = the most any lane has, 1 on the diagonal), the
      // rows read 16 bytes at a time where aligned -- the same fmaf order
      // as w2_cost_kernel either way.  (Per (g, e) entry with scalar loads
      // this cost up to 8 serial 256-load chains per diagonal slice.)
      uint32_t nm = 0u;
#pragma unroll
      for (int gg = 0; gg < 2; ++gg)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          nm |= v[gg][e] < wo.tau * (nrv + cnA[bj][g0 + gg][e]) ? 1u << (4 * gg + e) : 0u;
      if (__ballot(nm != 0u) != 0ull) {
        const int64_t i = ei0 + 32 * bi + r;
        const float* xi = wo.X + i * wo.ldx;
        while (__ballot(nm != 0u) != 0ull) {
          const int b = nm ? __builtin_ctz(nm) : 0;
          const int64_t j = ej0 + 32 * bj + 8 * (g0 + (b >> 2)) + 4 * h + (b & 3);
          const float* yj = wo.Y + (nm ? j : 0) * wo.ldy;
          float a = 0.f;
          if (nm) {
            if (wo.vec) {
              const f32x4* x4 = reinterpret_cast<const f32x4*>(xi);
              const f32x4* y4 = reinterpret_cast<const f32x4*>(yj);
#pragma unroll 2
              for (int k = 0; k < (wo.d >> 2); ++k) {
                const f32x4 xa = x4[k], ya = y4[k];
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                  const float df = xa[c] - ya[c];
                  a = fmaf(df, df, a);
                }
              }
            } else {
#pragma unroll 4
              for (int k = 0; k < wo.d; ++k) {
                const float df = xi[k] - yj[k];
                a = fmaf(df, df, a);
              }
            }
          }
#pragma unroll
          for (int gg = 0; gg < 2; ++gg)
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (nm && b == 4 * gg + e) v[gg][e] = a;
          nm &= nm - 1u;
        }
      }
    }
    if constexpr (OUT == 1) {
      // the largest real entry and the non-finite check (w2_cmax_kernel's)
      const uint32_t rb = (vrow >> bi) & 1u;
#pragma unroll
      for (int gg = 0; gg < 2; ++gg)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool ok = (rb & (vcol >> (16 * bj + 4 * (g0 + gg) + e))) != 0u;
          const float x = v[gg][e];
          cmx = max(cmx, ok ? __float_as_uint(x) : 0u);
          cbad |= ok && !(x >= 0.f && x <= FLT_MAX);
        }
    }
    if (!kBr && ediag) {
      const int tgv = tg[bi];
#pragma unroll
      for (int gg = 0; gg < 2; ++gg)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (tgv == e + 8 * (g0 + gg) + 32 * bj) v[gg][e] = 0.f;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const auto sv = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[0][e]),
                                                       __float_as_uint(v[1][e]), false, false);
      v[0][e] = __uint_as_float(sv[0]);
      v[1][e] = __uint_as_float(sv[1]);
    }
    if constexpr (OUT == 1) {
      // lane: row 32 bi + (lane & 15) (+16 for v[1]), columns 16 (2 bj + (SL & 1))
      // + 4 h + 8 ((lane >> 4) & 1) .. + 3 of the wave's 64
      if (wo.lines && SL < 14) {
        // full 128-byte lines (dsvgd_w2_set_cost_lines): a slice pair (even,
        // odd) holds both 64-byte halves of the same 32 rows' lines.  Each
        // slice parks its values in the hand-off chunks it has just read; the
        // odd one then reads them back transposed -- lanes 2k and 2k + 1 (rows
        // 2k', 2k' + 1) swap one chunk -- so that one store writes 8 even
        // rows whole and the next 8 odd rows whole (was 16 half lines per
        // store).  Slices 14 and 15 keep half lines: slice 15 runs after X,
        // where the M waves overwrite the hand-off.
        constexpr int ce = 4 * (2 * (SL >> 2) + ((SL >> 1) & 1));  // the even slice's chunks
        constexpr int cs = ce + 2 * (SL & 1);                       // this slice's chunks
        f32x4* const hb = reinterpret_cast<f32x4*>(hbuf);
        hb[cs * 64 + lane] = v[0];
        hb[(cs + 1) * 64 + lane] = v[1];
        if constexpr ((SL & 1) == 1) {
          asm volatile("" ::: "memory");
          const bool ev = (lane & 1) == 0;
          // the per-lane part of every line store's offset (row 2k' of the
          // pair, columns 4 h + 8 ((lane >> 4) & 1) + 16 (lane & 1)); the
          // slice's rows and columns go in the scalar offset
          const int vl = (int)((((lane & 15) & ~1) * wo.ldc + 4 * h + 8 * ((lane >> 4) & 1) +
                                16 * (lane & 1)) * 4);
          const int xo = ev ? ce * 64 + lane : (ce + 2) * 64 + (lane ^ 1);
          const int yo = ev ? ce * 64 + (lane ^ 1) : (ce + 2) * 64 + lane;
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            // X: row 2k' of the pair, Y: row 2k' + 1
            const f32x4 X = hb[xo + 64 * q];
            const f32x4 Y = hb[yo + 64 * q];
            const int so = (int)((32 * bi + 16 * q) * wo.ldc * 4) + 128 * bj;
            const int sy = so + (int)(wo.ldc * 4);
            if (wo.nt) {
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, X), rD, vl, so, 2);
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, Y), rD, vl, sy, 2);
            } else {
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, X), rD, vl, so, 0);
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, Y), rD, vl, sy, 0);
            }
          }
        }
      } else {
        // half-line pieces (the other 64 bytes of each row's line come one
        // slice later): nt, or the default policy so the L2 merges the halves
        // before they go out (dsvgd_w2_set_cost_nt, A/B); the per-lane offset
        // (row lane & 15, columns 4 h + 8 ((lane >> 4) & 1)) in a VGPR, the
        // slice's rows and columns in the scalar offset
        const int vh = (int)(((lane & 15) * wo.ldc + 4 * h + 8 * ((lane >> 4) & 1)) * 4);
        const int s0 = (int)(32 * bi * wo.ldc * 4) + 64 * (2 * bj + (SL & 1));
        const int s1 = s0 + (int)(16 * wo.ldc * 4);
        if (wo.nt) {
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v[0]), rD, vh, s0, 2);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v[1]), rD, vh, s1, 2);
        } else {
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v[0]), rD, vh, s0, 0);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v[1]), rD, vh, s1, 0);
        }
      }
    } else {
      const int vo = (32 * bi + (lane & 15)) * 64 + 16 * h + 32 * ((lane >> 4) & 1);
      constexpr int so = (2 * bj + (SL & 1)) * kPanelElems * 4;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v[0]), rD, vo, so, 2);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v[1]), rD, vo + 1024, so, 2);
    }
  };

  if constexpr (VAR & 16) __builtin_amdgcn_s_setprio(1);
  barrier();  // the prologue's (the M waves' first A stage)
  bool epi = false;  // a tile's accumulators are in the hand-off buffer
  // the previous tile's slot is closed (its last slice's stage flushed, the
  // counts stored) after slice 3 of the next, and the walk advanced after
  // slice 5 -- both off the hand-off, where the M waves wait for this wave
  GramSlotWriter<128> sw_old;
  int64_t eslot_old = 0;
  bool ew2_old = false, old_pending = false, adv_pending = false;
  for (;;) {
    // K-step k: after its barrier, slice k of the handed-off tile with slice
    // k + 1's values read ahead; the next tile's row / column data at k = 8,
    // 10, 12
#define DSVGD_GRS_E(KK)                                                        \
  if ((KK) == 8) prefetch_epi(cur, std::integral_constant<int, 0>{});        \
  if ((KK) == 10) prefetch_epi(cur, std::integral_constant<int, 1>{});       \
  if ((KK) == 12) prefetch_epi(cur, std::integral_constant<int, 2>{});       \
  barrier();                                                                   \
  if (epi && !(VAR & 4)) {                                                     \
    if ((KK) + 1 < 16) read_h((KK) + 1, hv[((KK) + 1) & 1]);                   \
    slice(std::integral_constant<int, KK>{}, hv[(KK) & 1]);                    \
  }                                                                            \
  if ((KK) == 3 && kBr && old_pending) {                                       \
    sw_old.finish_tile(sl, eslot_old, ew2_old);                                \
    old_pending = false;                                                       \
  }                                                                            \
  if ((KK) == 5 && adv_pending) {                                              \
    advance();                                                                 \
    adv_pending = false;                                                       \
  }
    DSVGD_GRS_E(0) DSVGD_GRS_E(1) DSVGD_GRS_E(2) DSVGD_GRS_E(3)
    DSVGD_GRS_E(4) DSVGD_GRS_E(5) DSVGD_GRS_E(6) DSVGD_GRS_E(7)
    DSVGD_GRS_E(8) DSVGD_GRS_E(9) DSVGD_GRS_E(10) DSVGD_GRS_E(11)
    DSVGD_GRS_E(12) DSVGD_GRS_E(13) DSVGD_GRS_E(14)
#undef DSVGD_GRS_E
    // K-step 15: the stage in the hand-off is flushed before X; slice 15
    // (its values read at slice 14) runs after X beside the M waves'
    // hand-off writes, its candidates in the stage of its own
    barrier();
    if (kBr && epi) {
      sw.flush4();
      sw.stage = sstage + lane;
    }
    for (int k = 16; k < nk; ++k) barrier();  // K-steps past the epilogue's 16 (dp > 256)
    // X: this tile's MFMAs are done, the previous tile's hand-off is read
    barrier();
    if (epi && !(VAR & 4)) slice(std::integral_constant<int, 15>{}, hv[1]);
    // Y: the M waves' hand-off writes have landed
    barrier();
    if (kBr && epi) {
      sw_old = sw;
      eslot_old = eslot;
      ew2_old = ew2;
      old_pending = true;
    }
    activate();
    if (kBr) {
      sw = GramSlotWriter<128>{};
      sw.klo = klo0;
      sw.kspan = kspan0;
      sw.dst = sl.data + eslot * sl.cap;
      sw.cap = (uint32_t)sl.cap;
      sw.stage = cstage + lane;
    }
    epi = true;
    read_h(0, hv[0]);
    if (!has_next) break;
    adv_pending = true;
  }
  if (kBr && old_pending) sw_old.finish_tile(sl, eslot_old, ew2_old);
  auto publish_stat = [&]() {
    if constexpr (OUT == 1) {
      if (wo.stat) {
        uint32_t mx = cmx;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
        const bool bad = __ballot(cbad) != 0ull;
        if (lane == 0) {
          atomicMax(wo.stat, mx);
          if (bad) atomicOr(wo.stat + 1, 1u);
        }
      }
    }
  };
  // drain: the last tile's epilogue, with the M waves gone
  if constexpr (!(VAR & 4)) {
#define DSVGD_GRS_D(KK)                                              \
  if ((KK) + 1 < 16) read_h((KK) + 1, hv[((KK) + 1) & 1]);           \
  slice(std::integral_constant<int, KK>{}, hv[(KK) & 1]);
    DSVGD_GRS_D(0) DSVGD_GRS_D(1) DSVGD_GRS_D(2) DSVGD_GRS_D(3)
    DSVGD_GRS_D(4) DSVGD_GRS_D(5) DSVGD_GRS_D(6) DSVGD_GRS_D(7)
    DSVGD_GRS_D(8) DSVGD_GRS_D(9) DSVGD_GRS_D(10) DSVGD_GRS_D(11)
    DSVGD_GRS_D(12) DSVGD_GRS_D(13) DSVGD_GRS_D(14) DSVGD_GRS_D(15)
#undef DSVGD_GRS_D
  }
  if (kBr) sw.finish_tile(sl, eslot, ew2);
  publish_stat();
}

}  // namespace dsvgd
