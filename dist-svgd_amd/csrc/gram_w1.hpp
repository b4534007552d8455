// gram_w1.hpp -- the FmtH2 distance Gram (D_ij = |y_i|^2 + |y_j|^2 - 2 y_i.y_j
// in the panel layout, plus the median select's accounting) with ONE wave per
// SIMD and TWO accumulator sets, so that a tile's epilogue runs between the
// next tile's MFMAs instead of after them.
//
// What the 8-wave sqdist_x3w_kernel (sqdist.hip) does differently: all eight
// waves stop their MFMAs for every tile's epilogue (D stores, bracket
// accounting, ~10 VALU per value), which left the matrix pipes idle ~60 % of
// the kernel (36 % MFMA-busy).  Here:
//   * unit = one 128-row strip x a pair of 128-column tiles; wave w owns the
//     unit's columns [64 w, 64 w + 64): 4 x 2 blocks of 32 x 32, i.e. 128
//     accumulators per set, two sets in the 256 AGPRs;
//   * the MFMAs run with the column fragment as the A operand, so a lane's 16
//     results of a block are 4 runs of 4 consecutive columns of one row; a
//     v_permlane16_swap per register pairs two runs so that every 16-byte
//     store instruction writes 16 whole 64-byte panel rows (1 KiB of whole
//     lines: the stores with half lines measured 1.44x the D bytes written
//     plus as many fetched);
//   * tile t accumulates into set t & 1 while its epilogue slice s (8 values
//     per lane) of tile t - 1 runs inside K-step s of tile t (16 K-steps at
//     d = 256), spread between the MFMAs;
//   * the strip's image rows (shared by the 4 waves) are staged through LDS
//     (2 x 8 KiB, loaded two K-steps ahead into VGPRs); each wave loads its
//     own column fragments straight from the image, two K-steps ahead;
//   * unit order: groups of 8 strips walk their column pairs together, so
//     the 32 blocks an XCD runs at once work on 8 strips x 4 column pairs
//     (1 MiB + 1 MiB of image, L2 resident) while the column pairs stream.
// The wave tile's D region is addressed through a buffer resource whose
// size is 0 for tiles that are not stored (below the diagonal of the
// symmetric layout, past the padded matrix): those stores are dropped by the
// hardware, no branch in the epilogue.  Padding rows / columns get +inf
// norms, so their entries come out +inf (skipped by the select).  The
// diagonal: without the select accounting it is set to exactly 0 on the tiles
// that hold it (a wave-uniform fix-up); with the bracket accounting it is
// stored as computed -- |y_i|^2 + |y_i|^2 - 2 y_i.y_i, a rounding residue
// ~2^-22 |y_i|^2, far below the bracket, so counted below it as an exact 0
// would be -- and phi_mm skips it by index either way.  (A compare + select
// per value cost two VALU and a VCC hazard nop on every value of every tile.)
//
// Limits (the host falls back to sqdist_x3w_kernel otherwise): FmtH2, the
// none / bracket select modes, no mirror stores (layout 1 or a rectangle),
// row0 % 16 == 0, dp % 256 == 0 (16 K-steps per epilogue).
#pragma once
#include "gemm_x3.hpp"
#include "select.hpp"

namespace dsvgd {

struct GramW1 {
  static constexpr int kThreads = 256;
  static constexpr int BM = 128;   // unit rows: one 128-row strip
  static constexpr int BN = 256;   // unit columns: two 128-column tiles, 64 per wave
  static constexpr int P = 2;
  static constexpr int SA = P * BM * 32;   // one K-step of the strip's image (8 KiB)
  static constexpr int kGroup = 8;         // strips per unit group (4, 16, 32: slower, profiles/r9e)
  // SlotWriterLdsT list depth: a tile's 128 values per lane, flushed once at
  // the tile's end (no loop inside the K-steps)
  static constexpr int kCandDepth = 128;
  static constexpr int kColOff = 2 * SA;   // per wave: [norm | 1/s][64 columns]
  static constexpr int kCandOff = kColOff + 4 * 2 * 64 * 4;
  static constexpr int kSmemBytes = kCandOff + 4 * 64 * kCandDepth * 4;
  static constexpr int kSlots = 4;         // candidate slots per unit (one per wave)
};

// Unit L -> (strip I, column pair J2).  Group g = strips [G g, G g + G)
// (G = kGroup) over column pairs [j0(g), Tc) (symmetric: j0(g) = G g / 2,
// the pair holding the group's first diagonal tile), strip-fastest.
// A row block of fewer than kGroup strips (the wide Gauss-Seidel pass: one
// strip) groups them all: phantom strips in the walk would leave 7 of 8
// blocks idle (96 us for a 64-row block on r11d, one unit per live block).
// The symmetric walk keeps kGroup (a compile-time group: no spills).
struct GramUnitWalk {
  int Tm, Tc, G, ng;
  bool sym;
  int g = 0;
  int64_t goff = 0;
  __host__ __device__ GramUnitWalk(int Tm_, int Tc_, bool sym_, int G_ = GramW1::kGroup)
      : Tm(Tm_), Tc(Tc_),
        G(sym_ || Tm_ >= G_ ? G_ : (Tm_ > 0 ? Tm_ : 1)),
        ng((Tm_ + G - 1) / G), sym(sym_) {}
  __host__ __device__ int j0(int gg) const { return sym ? gg * (G / 2) : 0; }
  __host__ __device__ int64_t count(int gg) const {
    const int c = Tc - j0(gg);
    return c > 0 ? (int64_t)c * G : 0;
  }
  __host__ __device__ int64_t total() const {
    int64_t s = 0;
    for (int gg = 0; gg < ng; ++gg) s += count(gg);
    return s;
  }
  // L must not decrease between calls
  __device__ __forceinline__ bool at(int64_t L, int& I, int& J2) {
    while (g < ng && L >= goff + count(g)) {
      goff += count(g);
      ++g;
    }
    if (g >= ng) return false;
    const int64_t rem = L - goff;
    J2 = j0(g) + (int)(rem / G);
    I = g * G + (int)(rem % G);
    return I < Tm && J2 < Tc && (!sym || I <= 2 * J2 + 1);
  }
};

// SlotWriterLdsT with a level-major flush: list entry k of every lane goes
// out as one ballot-compacted run (k = 0, 1, ... while any lane has one), so
// no wave prefix sum; the slot's order is deterministic, its content is the
// same set (the select passes only histogram it).
template <int DEPTH>
struct GramSlotWriter : SlotWriterLdsT<DEPTH> {
  using B = SlotWriterLdsT<DEPTH>;
  // branch-free but for the uniform loop exit: inactive lanes' stores go out
  // of the slot's buffer range and are dropped (as are entries past cap)
  __device__ __forceinline__ void flush() {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)B::dst, (short)0, (int)(B::cap * 4), 0x00020000);
    for (uint32_t k = 0;; ++k) {
      const bool act = k < B::pos;
      const uint64_t bal = __ballot(act);
      if (bal == 0ull) break;
      const uint32_t p = B::cnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
      const float v = B::stage[k * 64];
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, act ? (int)(p * 4) : -1, 0, 0);
      B::cnt += (uint32_t)__popcll(bal);
    }
    B::pos = 0u;
  }
  // the same, four levels per round of LDS reads (gram_rs: one flush per tile
  // over up to 128 levels, so the read latency is paid per four)
  __device__ __forceinline__ void flush4() {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)B::dst, (short)0, (int)(B::cap * 4), 0x00020000);
    for (uint32_t k0 = 0;; k0 += 4) {
      if (__ballot(k0 < B::pos) == 0ull) break;
      float v4[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) v4[i] = B::stage[(k0 + i) * 64];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool act = k0 + i < B::pos;
        const uint64_t bal = __ballot(act);
        const uint32_t p = B::cnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v4[i]), rs, act ? (int)(p * 4) : -1, 0, 0);
        B::cnt += (uint32_t)__popcll(bal);
      }
    }
    B::pos = 0u;
  }
  // finish() for a wave whose lanes saw at most 255 values each since begin
  // (gram_rs: one tile, 128 per lane): the below count summed by eight
  // ballots on the scalar unit instead of a six-step shuffle chain through
  // the LDS crossbar, the stage flushed four levels per round
  __device__ __forceinline__ void finish_tile(const SlotLayout& L, int64_t slot, bool weight2) {
    flush4();
    uint32_t b = 0u;
#pragma unroll
    for (int k = 0; k < 8; ++k) b += (uint32_t)__popcll(__ballot((B::below >> k) & 1u)) << k;
    const uint32_t flag = weight2 ? DSVGD_SLOT_WEIGHT2 : 0u;
    L.cnt[slot] = (B::cnt < DSVGD_SLOT_WEIGHT2 ? B::cnt : DSVGD_SLOT_WEIGHT2 - 1u) | flag;
    L.below[slot] = b;
  }
  __device__ __forceinline__ void finish(const SlotLayout& L, int64_t slot, bool weight2) {
    flush();
    uint32_t b = B::below;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) b += __shfl_xor(b, o, 64);
    // every lane stores the same words (no divergent branch)
    const uint32_t flag = weight2 ? DSVGD_SLOT_WEIGHT2 : 0u;
    L.cnt[slot] = (B::cnt < DSVGD_SLOT_WEIGHT2 ? B::cnt : DSVGD_SLOT_WEIGHT2 - 1u) | flag;
    L.below[slot] = b;
  }
};

__device__ __forceinline__ f32x4 gw1_load(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

// Yg: FmtH2 row image [kstep][part][img_rows][16] (swizzled, per-row scales
// rsc); this launch covers strips [0, Tm) of the owned rows [row0, row0 + m)
// against global column pairs [jp_off, jp_off + Tc); SYM: the whole matrix
// (row0 = 0, m = n), upper-triangle tiles only (layout 1, weight 2 off the
// diagonal).  Candidate slots slot_base + 4 L + w.
template <int smode, bool SYM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gram_w1_kernel(
    const _Float16* __restrict__ Yg, int64_t img_rows, const float* __restrict__ norms,
    const float* __restrict__ rsc, int64_t row0, int64_t m, int64_t n, int64_t n_pad, int nk,
    float* __restrict__ D, dsvgd_select_state* __restrict__ st, float* __restrict__ cand,
    int64_t total_units, int Tm, int Tc, int jp_off, int64_t slot_base, int64_t ns_total,
    int w2all = 0, const float* __restrict__ gate = nullptr) {
  using V8 = FmtH2::V8;
  constexpr bool kBr = smode == kSelBracket;
  __builtin_assume(nk >= 16 && nk % 16 == 0);  // checked by the host
  __shared__ __attribute__((aligned(16))) char smem[GramW1::kSmemBytes];
  const int t = threadIdx.x, lane = t & 63, r = lane & 31, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int T = (int)(n_pad >> 7);  // 128-column tiles of the padded matrix

  // this XCD's contiguous range of units, strided by its blocks
  const int64_t x = blockIdx.x % kXcds, u = blockIdx.x / kXcds, U = gridDim.x / kXcds;
  // gate: a fallback-only part of the pair-split layout (dsvgd_sqdist_h2_parts)
  // has units iff the FmtH2 range guard word is set (folded into the unit
  // count: an early return here cost the kernel 73 VGPRs and 160 B of spills)
  int64_t units = total_units;
  if constexpr (smode == kSelNone)  // (fallback parts never do select accounting)
    units = (gate && *gate == 0.f) ? 0 : total_units;
  const int64_t q = units / kXcds, rr = units % kXcds;
  const int64_t lo = x * q + min(x, rr);
  const int64_t hi = (int64_t)__builtin_amdgcn_readfirstlane((int)(lo + q + (x < rr ? 1 : 0)));
  SlotLayout sl(cand, ns_total, kBr ? st->cand_cap : 0);
  if (kBr) sl.publish(st, blockIdx.x);

  GramUnitWalk walk(Tm, Tc, SYM);
  auto next_valid = [&](int64_t L, int& I, int& J2) -> int64_t {
    for (; L < hi; L += U) {
      if (walk.at(L, I, J2)) {
        I = __builtin_amdgcn_readfirstlane(I);
        J2 = __builtin_amdgcn_readfirstlane(J2);
        return L;
      }
      if (kBr) {  // every lane stores the same zeros
        sl.cnt[slot_base + L * GramW1::kSlots + w] = 0u;
        sl.below[slot_base + L * GramW1::kSlots + w] = 0u;
      }
    }
    return L;
  };

  // ---- per-unit scalars ----------------------------------------------------
  struct Unit {
    int64_t L;
    int I, J2;
  };
  // the strip's image rows / the wave's image columns of unit un
  auto rsrc_A = [&](const Unit& un) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)(Yg + (row0 + (int64_t)un.I * 128) * 16),
                                             (short)0, 0x7fffffff, 0x00020000);
  };
  auto rsrc_B = [&](const Unit& un) {
    return __builtin_amdgcn_make_buffer_rsrc(
        (void*)(Yg + ((int64_t)(un.J2 + jp_off) * 256 + 64 * w) * 16), (short)0, 0x7fffffff,
        0x00020000);
  };
  auto make_unit = [&](int64_t L, int I, int J2) {
    Unit un;
    un.L = L;
    un.I = I;
    un.J2 = J2;
    return un;
  };

  int I0 = 0, J0 = 0;
  int64_t L0 = next_valid((int64_t)__builtin_amdgcn_readfirstlane((int)(lo + u)), I0, J0);
  if (L0 >= hi) return;  // block-uniform
  Unit cur = make_unit(L0, I0, J0);
  int In = 0, Jn = 0;
  int64_t Ln = next_valid(L0 + U, In, Jn);
  Unit nxt = make_unit(Ln < hi ? Ln : L0, Ln < hi ? In : I0, Ln < hi ? Jn : J0);
  bool has_next = Ln < hi;

  const int pstride = (int)(img_rows * 32);  // bytes of one part of one image K-step
  // staging: thread t copies the 16-byte chunks t (part 0) and t + 256 (part
  // 1) of the K-step's 8 KiB (row (t >> 1), half t & 1: consecutive threads,
  // consecutive LDS addresses)
  const int voffA = (t >> 1) * 32 + (t & 1) * 16;
  const int voffA1 = voffA + (int)img_rows * 32;
  const int ldsA = t * 16;
  const int vB = x3_off(r, h);

  // ---- accumulators (two sets) and the epilogue state ----------------------
  // epi*: the tile whose epilogue runs during the current tile's K-steps
  f32x16 acc[2][4][2];
  float nr[4], si2[4];  // row norms (+inf: padding / not stored), 2 / s_i
  int tg[4];            // diagonal target: c_row(q) + 32 bj == tg <=> i == j
  __amdgpu_buffer_rsrc_t rD = __builtin_amdgcn_make_buffer_rsrc((void*)D, (short)0, 0, 0x00020000);
  int64_t eslot = -1;
  bool ew2 = false;
  bool ediag = false;  // the wave's tile region holds diagonal entries (i == j)
  float* const colbase = reinterpret_cast<float*>(smem + GramW1::kColOff) + w * 128;
  GramSlotWriter<GramW1::kCandDepth> sw;
  float* const cstage = reinterpret_cast<float*>(smem + GramW1::kCandOff) + w * 64 * GramW1::kCandDepth;
  if (kBr) sw.begin(st, sl, 0, cstage);  // the empty pseudo tile before the first: +inf only

#pragma unroll
  for (int bi = 0; bi < 4; ++bi) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int bj = 0; bj < 2; ++bj)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[s2][bi][bj][e] = 0.f;
    nr[bi] = INFINITY;
    si2[bi] = 0.f;
    tg[bi] = 1 << 20;
  }

  // epilogue state <- unit un (rows: per lane; columns: the wave's LDS)
  auto load_epi = [&](const Unit& un) {
    const int64_t gi0 = row0 + (int64_t)un.I * 128;
    const int64_t gj0 = (int64_t)(un.J2 + jp_off) * 256 + 64 * w;
    const int Jt = (int)(gj0 >> 7);
    const bool valid = Jt < T && (!SYM || Jt >= un.I);
#pragma unroll
    for (int bi = 0; bi < 4; ++bi) {
      const int64_t il = (int64_t)un.I * 128 + 32 * bi + r;  // row within the owned block
      const bool ok = valid && il < m;
      nr[bi] = ok ? norms[row0 + il] : INFINITY;
      si2[bi] = 2.f * pow2_inv(ok ? rsc[row0 + il] : 1.f);
      tg[bi] = ok ? (int)(gi0 + 32 * bi + r - gj0) - 4 * h : (1 << 20);
    }
    const int64_t j = gj0 + lane;
    colbase[lane] = j < n ? norms[j] : INFINITY;
    colbase[64 + lane] = pow2_inv(j < n ? rsc[j] : 1.f);  // rsc holds >= n floats
    float* dt = D + ((int64_t)un.I * (n_pad >> 4) + (int64_t)Jt * 8 + 4 * (w & 1)) * kPanelElems;
    rD = __builtin_amdgcn_make_buffer_rsrc((void*)dt, (short)0, valid ? 4 * kPanelElems * 4 : 0,
                                           0x00020000);
    eslot = slot_base + un.L * GramW1::kSlots + w;
    ew2 = (SYM && Jt != un.I) || w2all != 0;  // w2all: a pair-split forward block
    ediag = valid && gj0 + 64 > gi0 && gj0 < gi0 + 128;
  };

  // runs g (columns 4 h + 0..3) and g + 1 (8 + 4 h + 0..3) of panel
  // 2 bj + (SL & 1), rows 32 bi + lane & 31: one v_permlane16_swap per
  // register turns them into rows 32 bi + 0..15 / 16..31 x all 16 columns
  // (lane l: row l & 15, columns 4 (l >> 5) + 8 ((l >> 4) & 1)), so each
  // 16-byte store covers 1 KiB of whole 128-byte lines
  auto store_slice = [&](f32x4 (&v)[2], auto SL_) {
    constexpr int SL = decltype(SL_)::value;
    constexpr int bi = SL >> 2, bj = (SL >> 1) & 1;
    // no select accounting: the diagonal (i == j) set to exactly 0 here, on
    // the tiles that hold it only (a wave-uniform branch) instead of a
    // compare + select per value between the MFMAs: the Gram without the
    // median select 3.92 -> 3.61 ms (profiles/r9u).  With the accounting the
    // per-value form stays (measured: no gain there)
    if (!kBr && ediag) {
      const int tgv = tg[bi];
#pragma unroll
      for (int gg = 0; gg < 2; ++gg) {
        const int g = 2 * (SL & 1) + gg;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (tgv == e + 8 * g + 32 * bj) v[gg][e] = 0.f;
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const auto sv = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[0][e]),
                                                       __float_as_uint(v[1][e]), false, false);
      v[0][e] = __uint_as_float(sv[0]);
      v[1][e] = __uint_as_float(sv[1]);
    }
    const int vo = (32 * bi + (lane & 15)) * 64 + 16 * h + 32 * ((lane >> 4) & 1);
    const int so = (2 * bj + (SL & 1)) * kPanelElems * 4;
    // nt (aux 2): measured against default, sc1 and nt sc1 -- equal or
    // faster (profiles/r8i)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v[0]), rD, vo, so, 2);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v[1]), rD, vo + 1024, so, 2);
  };

  // epilogue slice SL (0..15) of accumulator set S: block (bi, bj) = (SL >> 2,
  // (SL >> 1) & 1), register runs g = 2 (SL & 1), +1
  auto slice = [&](auto S_, auto SL_) {
    constexpr int S = decltype(S_)::value, SL = decltype(SL_)::value;
    constexpr int bi = SL >> 2, bj = (SL >> 1) & 1;
    // per-slice copies (keeps the compiler from hoisting the row values
    // and products of them over the whole tile into SGPRs; not volatile: a
    // side-effecting asm would cut the K-step's scheduling region in two)
    float nrv = nr[bi], siv = si2[bi];
    asm("" : "+v"(nrv), "+v"(siv));
    f32x4 v[2];
#pragma unroll
    for (int gg = 0; gg < 2; ++gg) {
      const int g = 2 * (SL & 1) + gg;
      const int co = 32 * bj + 4 * h + 8 * g;
      const f32x4 cn = *reinterpret_cast<const f32x4*>(colbase + co);
      const f32x4 cs = *reinterpret_cast<const f32x4*>(colbase + 64 + co);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        // straight from the accumulator register (keeps the set in AGPRs)
        float a;
        asm("v_accvgpr_read_b32 %0, %1" : "=v"(a) : "a"(acc[S][bi][bj][4 * g + e]));
        v[gg][e] = fmaxf(0.f, (nrv + cn[e]) - siv * (cs[e] * a));
      }
      if constexpr (kBr) {
#pragma unroll
        for (int e = 0; e < 4; ++e) sw.add(v[gg][e]);
        // settle the per-lane counts here: left alone, the compiler defers
        // the below-count sum to the tile's end and keeps all 128 keys live
        asm("" : "+v"(sw.below), "+v"(sw.pos));
      }
    }
    store_slice(v, SL_);
  };

  // ---- the K pipeline -------------------------------------------------------
  // image K-step k of the current unit: A loaded at step k - 2 into ra[k & 1],
  // staged to LDS at step k - 1; B loaded at step k - 2 into rb[k & 3]
  f32x4 ra[2][2];
  V8 rb[4][2][2];
  auto load_A = [&](int sa, int kk) {  // step kk's A (may be the next unit's)
    const bool nx = kk >= nk;
    const int ks = nx ? (has_next ? kk - nk : nk - 1) : kk;
    const __amdgpu_buffer_rsrc_t rA = rsrc_A(nx && has_next ? nxt : cur);
    const int so = ks * 2 * pstride;
    ra[sa][0] = gw1_load(rA, voffA, so);
    ra[sa][1] = gw1_load(rA, voffA1, so);
  };
  auto load_B = [&](int sb, int kk) {
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
  auto stage = [&](char* dst, int sa) {
    *reinterpret_cast<f32x4*>(dst + ldsA) = ra[sa][0];
    *reinterpret_cast<f32x4*>(dst + ldsA + GramW1::BM * 32) = ra[sa][1];
  };
  // the strip's fragments of one K-step from its LDS stage
  V8 af[2][4][2];
  auto read_frags = [&](V8 (&a)[4][2], const char* st_) {
#pragma unroll
    for (int bi = 0; bi < 4; ++bi)
#pragma unroll
      for (int p = 0; p < 2; ++p)
        a[bi][p] = *reinterpret_cast<const V8*>(st_ + p * GramW1::BM * 32 + x3_off(32 * bi + r, h));
  };
  // LDS writes landed, every wave past its LDS reads; and a scheduling
  // fence, so no instruction migrates across it
  auto barrier = []() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };

  // one K-step k (compile-time ring position KS = k mod 4) of set S, with
  // epilogue slice SL (< 0: none) of set S ^ 1; FIRST: the tile's K-step 0.
  // Written as 8 fenced groups of 3 MFMAs + one epilogue value (+ a load):
  // with one wave per SIMD nothing else fills the matrix pipe while this
  // wave issues VALU, so the VALU has to sit between the MFMAs (the
  // compiler's own schedule put the whole epilogue after the last MFMA).
  auto step = [&](auto S_, auto K_, auto SL_, auto FIRST_, int k) {
    constexpr int S = decltype(S_)::value, KS = decltype(K_)::value, SL = decltype(SL_)::value;
    constexpr bool FIRST = decltype(FIRST_)::value;
    constexpr int E = S ^ 1;                           // the set being written out
    constexpr int ebi = (SL < 0 ? 0 : SL) >> 2, ebj = ((SL < 0 ? 0 : SL) >> 1) & 1;
    char* nxt_st = smem + ((KS + 1) & 1) * GramW1::SA;
    V8 (&a)[4][2] = af[KS & 1];  // this K-step's strip fragments (read last K-step)
    stage(nxt_st, (KS + 1) & 1);
    // epilogue operands of this slice (see slice())
    float nrv = 0.f, siv = 0.f;
    f32x4 cn[2], cs[2], v[2];
    if constexpr (SL >= 0) {
      nrv = nr[ebi];
      siv = si2[ebi];
      asm("" : "+v"(nrv), "+v"(siv));
#pragma unroll
      for (int gg = 0; gg < 2; ++gg) {
        const int co = 32 * ebj + 4 * h + 8 * (2 * (SL & 1) + gg);
        cn[gg] = *reinterpret_cast<const f32x4*>(colbase + co);
        cs[gg] = *reinterpret_cast<const f32x4*>(colbase + 64 + co);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    f32x16 c[4][2];
#pragma unroll
    for (int grp = 0; grp < 8; ++grp) {
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        // MFMA 3 grp + q: product p = idx / 8 of block idx % 8 (consecutive
        // MFMAs independent; a block's products 8 apart)
        const int idx = 3 * grp + q, p = idx / 8, bi = (idx % 8) >> 1, bj = idx & 1;
        if (p == 0) c[bi][bj] = FIRST ? f32x16{} : acc[S][bi][bj];
        const V8 bx = rb[KS][bj][p == 1 ? 1 : 0];
        const V8 ax = a[bi][p == 0 ? 1 : 0];
        c[bi][bj] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bx, ax, c[bi][bj], 0, 0, 0);
        if (p == 2) {
          // both sets live in the AGPRs: the epilogue reads the other set's
          // values one by one (v_accvgpr_read) instead of copying it out
          asm("" : "+a"(c[bi][bj]));
          acc[S][bi][bj] = c[bi][bj];
        }
      }
      if constexpr (SL >= 0) {  // epilogue value grp: run gg = grp / 4, register e = grp % 4
        const int gg = grp >> 2, e = grp & 3, g = 2 * (SL & 1) + gg;
        float av;
        asm("v_accvgpr_read_b32 %0, %1" : "=v"(av) : "a"(acc[E][ebi][ebj][4 * g + e]));
        v[gg][e] = fmaxf(0.f, (nrv + cn[gg][e]) - siv * (cs[gg][e] * av));
        if constexpr (kBr) {
          sw.add(v[gg][e]);
          // settle the per-lane counts here: left alone, the compiler defers
          // the below-count sum to the tile's end and keeps all 128 keys live
          asm("" : "+v"(sw.below), "+v"(sw.pos));
        }
      }
      if (grp == 1) load_A(KS & 1, k + 2);
      if (grp == 2) load_B((KS + 2) & 3, k + 2);
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (grp == 3) {
        // mid-step: every wave's staging of K-step k + 1 has landed (and
        // every wave's reads of the buffer it replaced were done a K-step
        // ago); the next K-step's fragments are read now, behind the
        // remaining 12 MFMAs, so no K-step starts waiting on LDS
        barrier();
        read_frags(af[(KS + 1) & 1], nxt_st);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if constexpr (SL >= 0) store_slice(v, std::integral_constant<int, SL>{});
  };

  // prologue: A(0), A(1), B(0), B(1) loaded, A(0) staged and read
  load_A(0, 0);
  load_A(1, 1);
  load_B(0, 0);
  load_B(1, 1);
  stage(smem, 0);
  barrier();
  read_frags(af[0], smem);

  auto tile = [&](auto S_) {
#define DSVGD_GW1_STEP(KK)                                                                      \
  step(S_, std::integral_constant<int, (KK) & 3>{}, std::integral_constant<int, KK>{},          \
       std::integral_constant<bool, KK == 0>{}, KK);
    DSVGD_GW1_STEP(0) DSVGD_GW1_STEP(1) DSVGD_GW1_STEP(2) DSVGD_GW1_STEP(3)
    DSVGD_GW1_STEP(4) DSVGD_GW1_STEP(5) DSVGD_GW1_STEP(6) DSVGD_GW1_STEP(7)
    DSVGD_GW1_STEP(8) DSVGD_GW1_STEP(9) DSVGD_GW1_STEP(10) DSVGD_GW1_STEP(11)
    DSVGD_GW1_STEP(12) DSVGD_GW1_STEP(13) DSVGD_GW1_STEP(14) DSVGD_GW1_STEP(15)
#undef DSVGD_GW1_STEP
    for (int k = 16; k < nk; k += 4) {
      constexpr std::integral_constant<int, -1> none{};
      constexpr std::integral_constant<bool, false> later{};
      step(S_, std::integral_constant<int, 0>{}, none, later, k);
      step(S_, std::integral_constant<int, 1>{}, none, later, k + 1);
      step(S_, std::integral_constant<int, 2>{}, none, later, k + 2);
      step(S_, std::integral_constant<int, 3>{}, none, later, k + 3);
    }
    // the previous tile's epilogue is complete: its slot; this tile's opens
    if (kBr && eslot >= 0) sw.finish(sl, eslot, ew2);
    load_epi(cur);
    if (kBr) {
      sw = GramSlotWriter<GramW1::kCandDepth>{};
      sw.begin(st, sl, eslot, cstage);
    }
  };
  auto drain = [&](auto S_) {  // the last tile's epilogue, without MFMAs
#define DSVGD_GW1_SLICE(KK) slice(S_, std::integral_constant<int, KK>{});
    DSVGD_GW1_SLICE(0) DSVGD_GW1_SLICE(1) DSVGD_GW1_SLICE(2) DSVGD_GW1_SLICE(3)
    DSVGD_GW1_SLICE(4) DSVGD_GW1_SLICE(5) DSVGD_GW1_SLICE(6) DSVGD_GW1_SLICE(7)
    DSVGD_GW1_SLICE(8) DSVGD_GW1_SLICE(9) DSVGD_GW1_SLICE(10) DSVGD_GW1_SLICE(11)
    DSVGD_GW1_SLICE(12) DSVGD_GW1_SLICE(13) DSVGD_GW1_SLICE(14) DSVGD_GW1_SLICE(15)
#undef DSVGD_GW1_SLICE
    if (kBr) sw.finish(sl, eslot, ew2);
  };
  auto advance = [&]() {
    cur = nxt;
    int I2 = 0, J22 = 0;
    const int64_t L2 = next_valid(cur.L + U, I2, J22);
    has_next = L2 < hi;
    if (has_next) nxt = make_unit(L2, I2, J22);
  };

  for (;;) {
    const bool more0 = has_next;
    tile(std::integral_constant<int, 0>{});
    if (!more0) {
      drain(std::integral_constant<int, 0>{});
      break;
    }
    advance();
    const bool more1 = has_next;
    tile(std::integral_constant<int, 1>{});
    if (!more1) {
      drain(std::integral_constant<int, 1>{});
      break;
    }
    advance();
  }
}

}  // namespace dsvgd
