// gemm_x3.hpp -- the NN engine (C = exp-fused K . Y, gemm_tiles.hpp) on the
// bf16 MFMA (v_mfma_f32_32x32x16_bf16) with fp32 accuracy: both operands are
// split three ways into bf16,
//     v = v0 + v1 + v2 (+ a remainder of about 2^-26 |v|),  v0 = bf16(v),
//     v1 = bf16(v - v0), v2 = bf16(v - v0 - v1),
// and the six products with i + j <= 2 are accumulated in fp32 (a_i b_j is
// exact in fp32: 8 x 8 significant bits).  The dropped terms (a1 b2, a2 b1,
// a2 b2) are ~2^-26 of |a b| -- below fp32's own rounding of the product sum
// -- so the result carries fp32 GEMM error, not bf16 error (scripts/
// precision_x3.py compares it entry by entry with the exact-fp32 engine).
// Six bf16 MFMAs do the work of eight f32 ones at 1/16 of the cost each:
// 2.67x the f32 MFMA rate (MI355X_MICROARCH.md: 32x32x16 bf16 = 32 cycles,
// 32x32x2 f32 = 64 cycles for 1/8 of the k-depth).
//
// Operand images (one 16-column K-step; LDS and HBM use the same byte image):
//   * A (K = exp(-D/h), staged from D by the block): part p, row i: 32 B =
//     16 bf16 (k = 0..15), the two 16-B halves swapped on rows with bit 3 set
//     -- a fragment read (lane (r, h) reads row r, half h) then touches every
//     bank once per 16-lane group (MI355X_MICROARCH.md ds_read_b128 groups).
//   * B (Y = [Xc | S]): pre-split once per step by dsvgd_ysplit into
//     Yx[kstep][part][column][16 k] with the same half swizzle on column bit 3,
//     so a block's 3 x BC x 32 B of one K-step is contiguous per part and
//     lands in LDS by a lane-linear copy.
#pragma once
#include "gemm_tiles.hpp"

namespace dsvgd {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// 32x32x16 bf16 MFMA: lane (r = l&31, h = l>>5) holds A[r][8h + e] and
// B[8h + e][r] in element e; C/D layout identical to the f32 32x32x2 form.
__device__ __forceinline__ f32x16 mfma_bf16(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// v = s[0] + s[1] + s[2] to ~2^-26 |v| (|v| below bf16's overflow threshold)
struct Split3 {
  __bf16 s0, s1, s2;
};
__device__ __forceinline__ Split3 split3(float v) {
  Split3 o;
  o.s0 = (__bf16)v;
  float r = v - (float)o.s0;
  o.s1 = (__bf16)r;
  r -= (float)o.s1;
  o.s2 = (__bf16)r;
  return o;
}

constexpr int kX3Parts = 3;
constexpr int kX3Step = 16;  // K-step (columns of D / rows of Y)

// mask-bit set ? a : b, per lane, on a compile-time lane mask (v_cndmask_b32
// with the mask in an SGPR pair)
__device__ __forceinline__ float lane_select(uint64_t mask, float a, float b) {
  float d;
  asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(d) : "v"(b), "v"(a), "s"(mask));
  return d;
}

// ---- split formats: how an fp32 operand becomes MFMA inputs -------------
// FmtX3: three bf16 parts, six products a_i b_j (i + j <= 2).
// FmtH2: two fp16 parts of the operand scaled by a power of two,
//     s v = v0 + v1 (+ r, |r| <= 2^-22 |s v|),  v0 = f16(s v), v1 = f16(s v - v0),
// and the three products a0 b0 + a0 b1 + a1 b0 (each exact in fp32: 11 x 11
// significant bits; the dropped a1 b1 is <= 2^-22 |a b|).  The power-of-two
// scale s puts the operand's largest magnitude in [2^14, 2^15) (fp16's
// normal range spans 2^-14 .. 65504), so every element within 2^-18 of it
// keeps 22 significant bits; the caller divides the scale back out of the
// fp32 result exactly.  Half the MFMAs of FmtX3 at the same fp32-level
// error (a GEMM's own fp32 accumulation rounding dominates both).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

struct FmtX3 {
  using E = __bf16;
  using V8 = bf16x8;
  using V4 = bf16x4;
  static constexpr int P = 3;
  static constexpr float kAScale = 1.f;        // A operand (K, G) staging scale
  static constexpr float kAScaleLog2 = 0.f;
};
struct FmtH2 {
  using E = _Float16;
  using V8 = f16x8;
  using V4 = f16x4;
  static constexpr int P = 2;
  static constexpr float kAScale = 32768.f;    // |K| <= 1, |G| <= 1  ->  < 2^15
  static constexpr float kAScaleLog2 = 15.f;
};

// 32x32x16 MFMA of the format (C layout of mfma_bf16)
template <class F>
__device__ __forceinline__ f32x16 mfma_fmt(typename F::V8 a, typename F::V8 b, f32x16 c) {
  if constexpr (F::P == 3)
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// the P parts of v (already scaled for FmtH2)
template <class F>
__device__ __forceinline__ void split_fmt(float v, typename F::E (&o)[F::P]) {
  if constexpr (F::P == 3) {
    const Split3 s = split3(v);
    o[0] = s.s0;
    o[1] = s.s1;
    o[2] = s.s2;
  } else {
    o[0] = (_Float16)v;
    o[1] = (_Float16)(v - (float)o[0]);
  }
}

// products of one K-step into acc: small terms first
template <class F, int TM>
__device__ __forceinline__ void mfma_products(const typename F::V8 (&a)[TM][F::P],
                                              const typename F::V8 (&b)[F::P], f32x16* acc) {
  if constexpr (F::P == 3) {
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) acc[mi] = mfma_fmt<F>(a[mi][2], b[0], acc[mi]);
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) acc[mi] = mfma_fmt<F>(a[mi][1], b[1], acc[mi]);
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) acc[mi] = mfma_fmt<F>(a[mi][0], b[2], acc[mi]);
  }
#pragma unroll
  for (int mi = 0; mi < TM; ++mi) acc[mi] = mfma_fmt<F>(a[mi][1], b[0], acc[mi]);
#pragma unroll
  for (int mi = 0; mi < TM; ++mi) acc[mi] = mfma_fmt<F>(a[mi][0], b[1], acc[mi]);
#pragma unroll
  for (int mi = 0; mi < TM; ++mi) acc[mi] = mfma_fmt<F>(a[mi][0], b[0], acc[mi]);
}

// byte offset of (row or column x, 16-B half h) inside a part image
__device__ __forceinline__ int x3_off(int x, int h) { return x * 32 + ((h ^ ((x >> 3) & 1)) << 4); }

// C[128 x BC] = f(A)[128 x K] . B[K x BC], f = exp2(scale * a) with the
// diagonal skipped (EXP path of NNTile, same row-sum bookkeeping), 8 waves as
// 2 (rows) x 4 (columns), each 64 x 32*TN, double-buffered LDS, 16-deep
// K-steps (48 MFMAs per wave at TN = 4).
//
// Pipeline (one register set, cdna_hip_programming.md "Pipelining across
// barriers"): iteration k computes from LDS stage k&1; halfway through its
// MFMAs it writes tile k+1 (loaded one iteration earlier) into stage
// (k+1)&1, then issues the loads of tile k+2, so a load has a whole
// iteration to land.  The barrier closing an iteration is a raw s_barrier
// after lgkmcnt(0): __syncthreads() would also wait vmcnt(0) and drain the
// tile k+2 loads every K-step.
//
// DMA: both operands reach LDS by LDS-DMA (the B image is lane-linear; D
// lands raw in a 2-slot ring and is staged from there), issued at the start
// of iteration k for B of tile k+1 and D of tile k+2; counted vmcnt waits.
// EXP = false: f = identity (logreg G . Xd): no exp, no diagonal, no row sums.
// M16: v_mfma_f32_16x16x32_bf16 instead of 32x32x16 (the chip holds a higher
// clock on it, MI355X_MICROARCH.md "DVFS give-back" (7)).  Its k = 32 spans
// two parts side by side ("concatenated k"): [a0|a1].[b0|b1] = a0b0 + a1b1,
// [a1|a0].[b0|b1] = a1b0 + a0b1, [a0|a2].[b2|b0] = a0b2 + a2b0 -- the same six
// products in three MFMAs of half the cycles, two B and three A fragments.  Its fragment reads (16 rows x
// 2 halves per 16-lane group) are conflict-free on UNswizzled images
// (ysplit swz = 0).
// RW: row waves (8 waves = RW x 8/RW, each 64 x 32*TN).  RW = 2: 128-row
// blocks (phi_mm); RW = 4 (DMA, EXP = false only): 256-row blocks staging two
// D panels per K-step -- twice the MFMAs per B image (logreg G . Xd, where the
// B side is only 256 columns wide).
// NB (DMA path): ring stages.  2: iteration k DMAs tile k+1's B image (one
// iteration to land); 3: tile k+2's B and D (two iterations; the closing
// barrier then waits for no DMA at all).
// (Measured and dropped, DESIGN.md 3: D panels DMA'd three K-steps ahead, a
// ping-pong staging order, DMA issue after the first MFMA half, branch-free
// staging interleaved by sched_group_barrier.)
template <int TN, bool DMA = true, bool EXP = true, bool M16 = false, int RW = 2, class F = FmtX3,
          int NB = 2>
struct NNX3Tile {
  static constexpr int P = F::P;
  static_assert(NB == 2 || (NB == 3 && DMA), "3-stage ring: DMA path");
  static constexpr int ND = NB;  // raw D slots
  using V8 = typename F::V8;
  static_assert(!M16 || P == 3, "the 16x16x32 concatenated-k form is the 3-part format's");
  // (DMA needs the same DMA count in every wave: whole 512-chunk rounds)
  static constexpr int kThreads = 512;
  static constexpr int TM = 2;
  static constexpr int kCW = 8 / RW;     // column waves
  static constexpr int BM = 64 * RW;
  static constexpr int AR = BM / 128;    // D panels (128-row) per K-step
  static constexpr int BC = kCW * 32 * TN;
  static_assert(RW == 2 || (RW == 4 && DMA && !EXP), "256-row blocks: DMA path, no exp");
  static constexpr int BJ = kX3Step;
  static constexpr int SA = P * BM * 32;  // bytes of one stage's A image
  static constexpr int SB = P * BC * 32;
  static constexpr int kStage = SA + SB;
  static constexpr int kSmemBytes = NB * kStage + (DMA ? ND * AR * kPanelElems * 4 : 0);
  static constexpr int kBChunks = SB / 16;
  static constexpr int LB = (kBChunks + kThreads - 1) / kThreads;
  static constexpr int kHalf = TN > 1 ? TN / 2 : 1;  // column tiles before the mid-step write
  static_assert(kSmemBytes <= 160 * 1024, "LDS budget");
  static_assert(!DMA || kBChunks % kThreads == 0, "DMA: every wave issues LB DMAs");

  f32x16 acc[TM][TN];
  f32x4 acc16[4][2 * TN];  // M16: 16 x 16 tiles (4 row tiles x 2 TN column tiles)
  bf16x8 a16[4][3];        // M16: [a0|a1], [a1|a0], [a0|a2] per row tile
  f32x4 ra;      // the D values being staged (panel a of the K-step)
  int64_t prow = 0;  // RW = 4: bytes between the block's two D panel rows
  u32x4 rb[DMA ? 1 : LB];
  float rs;
  V8 a[TM][P];

  // A: thread t stages row t >> 2, columns 4 (t & 3) .. +3 of the D panel.
  // B: 16-B chunk f = t + 512 u of the block's K-step image (part f / (2 BC)).
  __device__ __forceinline__ void load(const float* __restrict__ Apanels, const typename F::E* __restrict__ Yx,
                                       int64_t ldy, int64_t j0) {
    const int t = threadIdx.x;
    const __amdgpu_buffer_rsrc_t rA =
        __builtin_amdgcn_make_buffer_rsrc((void*)Apanels, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rB =
        __builtin_amdgcn_make_buffer_rsrc((void*)Yx, (short)0, 0x7fffffff, 0x00020000);
    const int soA = (int)((j0 >> 4) * kPanelElems * 4);
    const int soB = (int)((j0 >> 4) * P * ldy * 32);
    ra = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rA, t * 16, soA, 0));
#pragma unroll
    for (int u = 0; u < LB; ++u) {
      const int f = t + u * kThreads;
      if (kBChunks % kThreads == 0 || f < kBChunks) {
        const int p = f / (2 * BC), rem = f % (2 * BC);
        rb[u] = __builtin_bit_cast(
            u32x4, __builtin_amdgcn_raw_buffer_load_b128(rB, (int)(p * ldy * 32 + rem * 16), soB, 0));
      }
    }
  }

  __device__ __forceinline__ void store(char* st, float scale, int64_t dgl) {
    store_a(st, scale, dgl);
    const int t = threadIdx.x;
#pragma unroll
    for (int u = 0; u < LB; ++u) {
      const int f = t + u * kThreads;
      if (kBChunks % kThreads == 0 || f < kBChunks)
        *reinterpret_cast<u32x4*>(st + SA + f * 16) = rb[u];
    }
  }

  // exp / diagonal / row sum / 3-way split of this thread's 4 D values (ra)
  // of panel a (image rows 128 a + ...)
  __device__ __forceinline__ void store_a(char* st, float scale, int64_t dgl, int a = 0) {
    const int t = threadIdx.x, row = (t >> 2) + 128 * a, c4 = t & 3;
    // FmtH2: K scaled by 2^15 inside the exp2 (row sums too: the kernel's
    // epilogue divides it back out), G by 2^15 (exact)
    if (!EXP) {
      if constexpr (F::kAScale != 1.f) {
#pragma unroll
        for (int q = 0; q < 4; ++q) ra[q] *= F::kAScale;
      }
    } else if (dgl > -BM && dgl < BJ) {  // the K-step holds diagonal entries (NNTile::store)
      const int qd = (int)dgl + row - 4 * c4;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        ra[q] = (qd == q) ? 0.f : __builtin_amdgcn_exp2f(fmaf(ra[q], scale, F::kAScaleLog2));
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) ra[q] = __builtin_amdgcn_exp2f(fmaf(ra[q], scale, F::kAScaleLog2));
    }
    if (EXP) rs += (ra[0] + ra[1]) + (ra[2] + ra[3]);
    typename F::V4 sp[P];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      typename F::E v[P];
      split_fmt<F>(ra[q], v);
#pragma unroll
      for (int p = 0; p < P; ++p) sp[p][q] = v[p];
    }
    const int off = (M16 ? row * 32 + ((c4 >> 1) << 4) : x3_off(row, c4 >> 1)) + ((c4 & 1) << 3);
#pragma unroll
    for (int p = 0; p < P; ++p) *reinterpret_cast<typename F::V4*>(st + p * BM * 32 + off) = sp[p];
  }

  // ---- DMA path: both operands by LDS-DMA (buffer_load_dwordx4 ... lds:
  // wave-uniform LDS base + 16 B per lane, per-lane source offsets).  Only
  // LDS-DMA in the loop, so every vmcnt wait is counted by hand (a plain
  // load beside it makes hipcc wait vmcnt(0): cdna_hip_programming.md "three
  // .s-level traps" (b)).
  static constexpr int kRaw = NB * kStage;  // D ring: NB slots x AR x 8 KiB raw panels
  static constexpr int kSlot = AR * kPanelElems * 4;
  static constexpr int kDAux = 2;  // D panels: nt (read once) so Yx stays in L2

  // aux: cache policy (2 = nt on gfx950: the D stream is read once)
  template <int AUX = 0>
  __device__ __forceinline__ static void dma16(__amdgpu_buffer_rsrc_t r, char* lds, int voff,
                                               int soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16,
                                             voff, soff, 0, AUX);
  }

  // tile j0's B image -> LDS stage st
  __device__ __forceinline__ void dma_b(char* st, __amdgpu_buffer_rsrc_t rB, int64_t ldy,
                                        int64_t j0) {
    const int t = threadIdx.x, wbase = __builtin_amdgcn_readfirstlane(t >> 6) * 64;
    const int soB = (int)((j0 >> 4) * P * ldy * 32);
#pragma unroll
    for (int u = 0; u < LB; ++u) {
      const int f = t + u * kThreads, p = f / (2 * BC), rem = f % (2 * BC);
      dma16(rB, st + SA + (wbase + u * kThreads) * 16, (int)(p * ldy * 32 + rem * 16), soB);
    }
  }

  // tile j0's D panel (8 KiB) -> raw slot: thread t's 16 B land at t * 16,
  // where the same thread reads them (no barrier needed, only its vmcnt)
  __device__ __forceinline__ void dma_d(char* raw, __amdgpu_buffer_rsrc_t rA, int64_t j0) {
    const int t = threadIdx.x;
    if (transposed(j0)) {
      // symmetric layout, K-step in a column tile J < I: D[i][j0 + jj] is
      // stored as tile (J, I); its rows j0..j0+15 of the 8 panels covering
      // columns I*128.. are 8 contiguous 1-KiB pieces, one per wave:
      // raw[w][jj][ii] = D[I*128 + 16w + ii][j0 + jj]
      const float* src = sym_D + (((j0 >> 7) * sym_pcols + sym_I * 8) * kPanelElems +
                                   (j0 & 127) * 16);
      const __amdgpu_buffer_rsrc_t rT =
          __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 0x7fffffff, 0x00020000);
      dma16<kDAux>(rT, raw + __builtin_amdgcn_readfirstlane(t >> 6) * 1024, (t >> 6) * kPanelElems * 4 + (t & 63) * 16, 0);
      return;
    }
#pragma unroll
    for (int a = 0; a < AR; ++a)
      dma16<kDAux>(rA, raw + a * kPanelElems * 4 + __builtin_amdgcn_readfirstlane(t >> 6) * 1024, (int)(a * prow) + t * 16,
                   (int)((j0 >> 4) * kPanelElems * 4));
  }

  // this thread's 4 D values (row t >> 2, columns 4 (t & 3) ..) of K-step j0
  // from its raw slot
  __device__ __forceinline__ f32x4 raw_read(const char* raw, int64_t j0, int a = 0) const {
    const int t = threadIdx.x;
    if (RW == 2 && transposed(j0)) {
      // read e fetches column 4 c4 + ((e + c4) & 3): the four c4 lanes of a
      // row then hit four different 16-bank groups (in column order they
      // would all hit the same one, 4-way); rotated back in registers
      const int row = t >> 2, c4 = t & 3;
      const float* r = reinterpret_cast<const float*>(raw) + (row >> 4) * 256 + (row & 15) +
                       (4 * c4) * 16;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = r[((e + c4) & 3) * 16];
      // v[e] = column (e + c4) & 3  ->  out[q] = v[(q - c4) & 3]: two
      // conditional rotations on the lane masks of c4 = lane & 3 (constant
      // SGPR masks; the compiler's own selects re-derived the mask per value)
      constexpr uint64_t kOdd = 0xAAAAAAAAAAAAAAAAull, kHi2 = 0xCCCCCCCCCCCCCCCCull;
      float w[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) w[q] = lane_select(kOdd, v[(q + 3) & 3], v[q]);
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = lane_select(kHi2, w[(q + 2) & 3], w[q]);
      return f32x4{v[0], v[1], v[2], v[3]};
    }
    return *reinterpret_cast<const f32x4*>(raw + a * kPanelElems * 4 + t * 16);
  }

  // K-step stride of the 3-stage DMA path (run/step_dma3): BJ, or Z * BJ when
  // Z split-K slices interleave their K-steps (slice z: z, z + Z, ...)
  int64_t kst = BJ;
  // symmetric layout (dsvgd_sqdist_x3 layout 1): only tiles (I, J >= I) exist
  const float* sym_D = nullptr;  // whole panel-layout D, or null (full layout)
  int64_t sym_pcols = 0;         // n_pad / 16
  int64_t sym_I = 0;             // this block's row tile
  __device__ __forceinline__ bool transposed(int64_t j0) const {
    return sym_D != nullptr && (j0 >> 7) < sym_I;
  }

  __device__ __forceinline__ void read_a(const char* st, int wr) {
    if (M16) {  // lane (rr = l & 15, g = l >> 4): k-slot g >> 1 picks the part, g & 1 the half
      const int lane = threadIdx.x & 63, rr = lane & 15, g = lane >> 4, hh = g & 1;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const int off = (wr * 64 + mt * 16 + rr) * 32 + hh * 16;
        const int sl = g >> 1;
        a16[mt][0] = *reinterpret_cast<const bf16x8*>(st + sl * BM * 32 + off);        // [a0|a1]
        a16[mt][1] = *reinterpret_cast<const bf16x8*>(st + (sl ^ 1) * BM * 32 + off);  // [a1|a0]
        a16[mt][2] = *reinterpret_cast<const bf16x8*>(st + 2 * sl * BM * 32 + off);    // [a0|a2]
      }
      return;
    }
    const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
      for (int p = 0; p < P; ++p)
        a[mi][p] = *reinterpret_cast<const V8*>(st + p * BM * 32 +
                                                x3_off(wr * 32 * TM + mi * 32 + r, h));
  }

  // column tiles [N0, N1) of this wave
  template <int N0, int N1>
  __device__ __forceinline__ void compute(const char* st, int wc) {
    if (M16) {
      const int lane = threadIdx.x & 63, rr = lane & 15, g = lane >> 4, hh = g & 1;
      const int s = g >> 1;  // k-slot
#pragma unroll
      for (int nt = 2 * N0; nt < 2 * N1; ++nt) {
        const char* bb = st + SA + (wc * 32 * TN + nt * 16 + rr) * 32 + hh * 16;
        // two B fragments per column tile, three A fragments per row tile:
        // [a0|a2].[b2|b0] = a0b2 + a2b0, [a1|a0].[b0|b1] = a1b0 + a0b1,
        // [a0|a1].[b0|b1] = a0b0 + a1b1
        const bf16x8 g1 = *reinterpret_cast<const bf16x8*>(bb + s * BC * 32);            // [b0|b1]
        const bf16x8 g3 = *reinterpret_cast<const bf16x8*>(bb + (2 - 2 * s) * BC * 32);  // [b2|b0]
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          acc16[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a16[mt][2], g3, acc16[mt][nt], 0, 0, 0);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          acc16[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a16[mt][1], g1, acc16[mt][nt], 0, 0, 0);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          acc16[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a16[mt][0], g1, acc16[mt][nt], 0, 0, 0);
      }
      return;
    }
    const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
#pragma unroll
    for (int ni = N0; ni < N1; ++ni) {
      V8 b[P];
#pragma unroll
      for (int p = 0; p < P; ++p)
        b[p] = *reinterpret_cast<const V8*>(st + SA + p * BC * 32 +
                                            x3_off(wc * 32 * TN + ni * 32 + r, h));
      // small terms first; the two row tiles interleaved (independent chains)
      f32x16 c[TM];
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) c[mi] = acc[mi][ni];
      mfma_products<F, TM>(a, b, c);
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) acc[mi][ni] = c[mi];
    }
  }

  // LDS writes of this thread done, then every wave's (no vmcnt wait: the
  // next tile's loads stay in flight)
  __device__ __forceinline__ static void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }

  // Apanels: the block's 128-row panel row (panel layout); Yx: the split Y
  // image offset to the block's first column; K range [k0, k1) (multiples of 16).
  __device__ __forceinline__ void run(const float* __restrict__ Apanels, const typename F::E* __restrict__ Yx,
                                      int64_t ldy, int64_t k0, int64_t k1, float scale, char* smem,
                                      int64_t row_g0) {
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), wr = w / kCW, wc = w % kCW;
    rs = 0.f;
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
      for (int ni = 0; ni < TN; ++ni)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[mi][ni][q] = 0.f;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 2 * TN; ++nt) acc16[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (k0 >= k1) return;
    if (DMA) {
      const __amdgpu_buffer_rsrc_t rA =
          __builtin_amdgcn_make_buffer_rsrc((void*)Apanels, (short)0, 0x7fffffff, 0x00020000);
      const __amdgpu_buffer_rsrc_t rB =
          __builtin_amdgcn_make_buffer_rsrc((void*)Yx, (short)0, 0x7fffffff, 0x00020000);
      char* raw = smem + kRaw;
      if constexpr (NB == 3) {
        dma_b(smem, rB, ldy, k0);
        dma_d(raw, rA, k0);
        if (k0 + kst < k1) {
          dma_b(smem + kStage, rB, ldy, k0 + kst);
          dma_d(raw + kSlot, rA, k0 + kst);
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LB + AR) : "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
#pragma unroll
        for (int a = 0; a < AR; ++a) {
          ra = raw_read(raw, k0, a);
          store_a(smem, scale, row_g0 - k0, a);
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        for (int64_t j0 = k0; j0 < k1; j0 += 3 * kst) {
          step_dma3<0>(rA, rB, ldy, j0, k1, scale, smem, row_g0, wr, wc);
          if (j0 + kst < k1) step_dma3<1>(rA, rB, ldy, j0 + kst, k1, scale, smem, row_g0, wr, wc);
          if (j0 + 2 * kst < k1)
            step_dma3<2>(rA, rB, ldy, j0 + 2 * kst, k1, scale, smem, row_g0, wr, wc);
        }
        return;
      }
      dma_b(smem, rB, ldy, k0);
      dma_d(raw, rA, k0);
      if (k0 + BJ < k1) dma_d(raw + kSlot, rA, k0 + BJ);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int a = 0; a < AR; ++a) {
        ra = raw_read(raw, k0, a);
        store_a(smem, scale, row_g0 - k0, a);
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      for (int64_t j0 = k0; j0 < k1; j0 += 2 * BJ) {
        step_dma<0>(rA, rB, ldy, j0, k1, scale, smem, row_g0, wr, wc);
        if (j0 + BJ < k1) step_dma<1>(rA, rB, ldy, j0 + BJ, k1, scale, smem, row_g0, wr, wc);
      }
      return;
    } else {
      load(Apanels, Yx, ldy, k0);
      store(smem, scale, row_g0 - k0);
      if (k0 + BJ < k1) load(Apanels, Yx, ldy, k0 + BJ);
      lds_barrier();
    }
    // unrolled by two so both LDS stage bases are compile-time constants
    for (int64_t j0 = k0; j0 < k1; j0 += 2 * BJ) {
      step<0>(Apanels, Yx, ldy, j0, k1, scale, smem, row_g0, wr, wc);
      if (j0 + BJ < k1) step<1>(Apanels, Yx, ldy, j0 + BJ, k1, scale, smem, row_g0, wr, wc);
    }
  }

  template <int CUR>
  __device__ __forceinline__ void step(const float* __restrict__ Apanels, const typename F::E* __restrict__ Yx,
                                       int64_t ldy, int64_t j0, int64_t k1, float scale, char* smem,
                                       int64_t row_g0, int wr, int wc) {
    const char* cur = smem + CUR * kStage;
    read_a(cur, wr);
    compute<0, kHalf>(cur, wc);
    if (j0 + BJ < k1) store(smem + (CUR ^ 1) * kStage, scale, row_g0 - (j0 + BJ));
    if (j0 + 2 * BJ < k1) load(Apanels, Yx, ldy, j0 + 2 * BJ);
    compute<kHalf, TN>(cur, wc);
    lds_barrier();
  }

  // iteration k (tile j0, LDS stage CUR): DMA tile k+1's B into stage CUR^1
  // (free since the last barrier) and tile k+2's D into raw slot CUR (its
  // tile k was consumed last iteration); halfway, stage tile k+1's A from
  // raw slot CUR^1 (DMA'd last iteration: LB + 1 DMAs younger than it).
  template <int CUR>
  __device__ __forceinline__ void step_dma(__amdgpu_buffer_rsrc_t rA, __amdgpu_buffer_rsrc_t rB,
                                           int64_t ldy, int64_t j0, int64_t k1, float scale,
                                           char* smem, int64_t row_g0, int wr, int wc) {
    const char* cur = smem + CUR * kStage;
    char* raw = smem + kRaw;
    const bool more = j0 + BJ < k1, more2 = j0 + 2 * BJ < k1;
    if (more) dma_b(smem + (CUR ^ 1) * kStage, rB, ldy, j0 + BJ);
    if (more2) dma_d(raw + CUR * kSlot, rA, j0 + 2 * BJ);
    read_a(cur, wr);
    compute<0, kHalf>(cur, wc);
    if (more) {
      if (more2)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LB + AR) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LB) : "memory");
#pragma unroll
      for (int a = 0; a < AR; ++a) {
        ra = raw_read(raw + (CUR ^ 1) * kSlot, j0 + BJ, a);
        store_a(smem + (CUR ^ 1) * kStage, scale, row_g0 - (j0 + BJ), a);
      }
    }
    compute<kHalf, TN>(cur, wc);
    // this wave's B DMAs landed (the D DMA may stay in flight), LDS writes
    // done, then all waves
    if (more2)
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(AR) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }

  // 3-stage ring, iteration k (tile j0, stage CUR = k % 3): DMA tile k+2's B
  // and D into stage / raw slot (CUR + 2) % 3 (consumed at iteration k-1 and
  // k-2); halfway, wait for tile k+1's D (issued last iteration, after its B:
  // both landed) and stage its A into stage (CUR + 1) % 3.  The closing
  // barrier waits for LDS writes only.
  template <int CUR>
  __device__ __forceinline__ void step_dma3(__amdgpu_buffer_rsrc_t rA, __amdgpu_buffer_rsrc_t rB,
                                            int64_t ldy, int64_t j0, int64_t k1, float scale,
                                            char* smem, int64_t row_g0, int wr, int wc) {
    constexpr int NXT = (CUR + 1) % 3, NN = (CUR + 2) % 3;
    const char* cur = smem + CUR * kStage;
    char* raw = smem + kRaw;
    const bool more = j0 + kst < k1, more2 = j0 + 2 * kst < k1;
    if (more2) {
      dma_b(smem + NN * kStage, rB, ldy, j0 + 2 * kst);
      dma_d(raw + NN * kSlot, rA, j0 + 2 * kst);
    }
    read_a(cur, wr);
    compute<0, kHalf>(cur, wc);
    if (more) {
      if (more2)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LB + AR) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int a = 0; a < AR; ++a) {
        ra = raw_read(raw + NXT * kSlot, j0 + kst, a);
        store_a(smem + NXT * kStage, scale, row_g0 - (j0 + kst), a);
      }
    }
    compute<kHalf, TN>(cur, wc);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }

  // full row sum of row threadIdx.x >> 2 (4 consecutive lanes stage a row)
  __device__ __forceinline__ float row_sum() const {
    float v = rs;
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    return v;
  }
};

// ---- NT engine on the split images: C[BM x BN] = A[BM x K] . B[BN x K]^T
// (the Gram, logreg Z, predict).  Both operands come as row images
//     img[kstep][part][row][16 k]  (bf16, 32 B per row, halves swapped on
//     rows with bit 3 set -- dsvgd_rowsplit)
// and reach LDS verbatim by LDS-DMA (a block's 128 rows of one part are 4 KiB
// contiguous), through a 3-stage ring: iteration k issues tile k+2 and waits
// (counted vmcnt) for tile k+1 before its closing barrier, so a DMA has two
// iterations to land.  No VGPR staging, no VALU in the loop but the MFMAs.
// NS: ring stages (3: a DMA has two iterations to land; 2: one, at 2/3 of the LDS).
// M16: v_mfma_f32_16x16x32_bf16 with concatenated k (NNX3Tile); the results
// are in acc16[4][2 TN] (16x16 layout) and both images must be unswizzled.
// KS: 16-deep image K-steps per ring stage (one barrier per stage): 2 halves
// the barriers per tile at twice the stage size.
// WC: wave-contiguous DMA chunks -- wave w fills the 1 KiB chunks [w C,
// (w + 1) C) of a stage (C = kChunksPerWave), so once every wave is past the
// barrier that retires a stage, each wave's own C KiB of it stay untouched
// until that wave issues its next DMA into it: private scratch in between.
template <int TM, int TN, int WM, int WN, int NS = 3, bool M16 = false, class F = FmtX3, int KS = 1,
          bool WC = false>
struct NTX3Tile {
  static constexpr int TM_ = TM, TN_ = TN, WM_ = WM, WN_ = WN;
  static constexpr bool M16_ = M16;
  static constexpr int P = F::P;
  using V8 = typename F::V8;
  static_assert(!M16 || TM == 2, "M16: 64-row waves");
  static_assert(!M16 || P == 3, "the 16x16x32 concatenated-k form is the 3-part format's");
  static constexpr int kThreads = 64 * WM * WN;
  static constexpr int BM = 32 * TM * WM;
  static constexpr int BN = 32 * TN * WN;
  static constexpr int BK = kX3Step;
  static constexpr int SA = P * BM * 32;
  static constexpr int SB = P * BN * 32;
  static constexpr int kSub = SA + SB;          // one 16-deep image K-step
  static constexpr int kStage = KS * kSub;
  static constexpr int kStages = NS;
  static_assert(NS == 2 || NS == 3, "2- or 3-stage ring");
  static_assert(KS == 1 || (KS == 2 && !M16), "two sub-steps per stage: 32x32 form");
  static constexpr int kSmemBytes = kStages * kStage;
  static constexpr int LA = SA / 16 / kThreads;  // DMAs per thread per K-step (A)
  static constexpr int LBn = SB / 16 / kThreads;
  static constexpr int kDmas = KS * (LA + LBn);
  static_assert(SA % (16 * kThreads) == 0 && SB % (16 * kThreads) == 0, "whole DMA rounds");
  static_assert(BM * 32 % (16 * kThreads) == 0, "a DMA round stays inside one part");
  static_assert(kSmemBytes <= 160 * 1024, "LDS budget");

  f32x16 acc[TM][TN];
  f32x4 acc16[M16 ? 4 : 1][M16 ? 2 * TN : 1];

  __device__ __forceinline__ void zero() {
    if (M16) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2 * TN; ++nt) acc16[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      return;
    }
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
      for (int ni = 0; ni < TN; ++ni)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[mi][ni][q] = 0.f;
  }

  __device__ __forceinline__ static void dma16(__amdgpu_buffer_rsrc_t r, char* lds, int voff,
                                               int soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16,
                                             voff, soff, 0, 0);
  }

  // K-step kb of A (image rows from rA's base, mA image rows per part) and B
  // into stage st
  static constexpr int kChunks = kStage / 1024, kChunksPerWave = kChunks / (kThreads / 64);
  static_assert(!WC || (SA % 1024 == 0 && SB % 1024 == 0 && kChunks % (kThreads / 64) == 0 &&
                        BM % 32 == 0 && BN % 32 == 0),
                "wave-contiguous chunks: whole 1 KiB chunks per wave and per part");

  __device__ __forceinline__ void dma(char* st, __amdgpu_buffer_rsrc_t rA, int64_t mA,
                                      __amdgpu_buffer_rsrc_t rB, int64_t mB, int64_t kb) {
    if constexpr (WC) {
      // chunk c = w C + u: sub-step c / (kSub / 1K), then A or B, then 64
      // consecutive 16-byte units of that image slice (as below)
      const int lane = threadIdx.x & 63;
      const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
#pragma unroll
      for (int u = 0; u < kChunksPerWave; ++u) {
        const int c = w * kChunksPerWave + u;
        const int q = c / (kSub / 1024), r = c % (kSub / 1024);
        const int ki = (int)kb * KS + q;
        const bool isA = r < SA / 1024;
        const int rr = isA ? r : r - SA / 1024, BX = isA ? BM : BN;
        const int mX = (int)(isA ? mA : mB);  // image offsets are 32-bit (< 2^31 bytes)
        // a part is BX / 32 chunks: chunk rr = part rr / (BX / 32), 16-byte
        // units (rr % (BX / 32)) 64 + lane -- all but lane * 16 wave-uniform
        const int pp = rr / (BX / 32), in0 = (rr % (BX / 32)) * 64;
        dma16(isA ? rA : rB, st + c * 1024, lane * 16, (ki * P + pp) * mX * 32 + in0 * 16);
      }
      return;
    }
    const int t = threadIdx.x, wbase = __builtin_amdgcn_readfirstlane(t >> 6) * 64;
#pragma unroll
    for (int q = 0; q < KS; ++q) {
      const int64_t ki = kb * KS + q;  // image K-step
      const int soA = (int)(ki * P * mA * 32), soB = (int)(ki * P * mB * 32);
      char* sq = st + q * kSub;
#pragma unroll
      for (int u = 0; u < LA; ++u) {
        const int f = t + u * kThreads, pp = f / (BM * 2), in = f % (BM * 2);
        dma16(rA, sq + (wbase + u * kThreads) * 16, (int)(pp * mA * 32 + in * 16), soA);
      }
#pragma unroll
      for (int u = 0; u < LBn; ++u) {
        const int f = t + u * kThreads, pp = f / (BN * 2), in = f % (BN * 2);
        dma16(rB, sq + SA + (wbase + u * kThreads) * 16, (int)(pp * mB * 32 + in * 16), soB);
      }
    }
  }

  // a0: image row of A's row 0, mod 16 (the image swizzles on the absolute
  // row; a row block may start off a 16-row boundary).
  __device__ __forceinline__ void compute(const char* st, int wm, int wn, int a0 = 0) {
    if (M16) {  // lane (rr = l & 15, g = l >> 4): k-slot g >> 1 picks the part, g & 1 the half
      const int lane = threadIdx.x & 63, rr = lane & 15, g = lane >> 4, hh = g & 1, sl = g >> 1;
      bf16x8 f[4][3];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const char* aa = st + (wm * 64 + mt * 16 + rr) * 32 + hh * 16;
        f[mt][0] = *reinterpret_cast<const bf16x8*>(aa + sl * BM * 32);        // [a0|a1]
        f[mt][1] = *reinterpret_cast<const bf16x8*>(aa + (sl ^ 1) * BM * 32);  // [a1|a0]
        f[mt][2] = *reinterpret_cast<const bf16x8*>(aa + 2 * sl * BM * 32);    // [a0|a2]
      }
#pragma unroll
      for (int nt = 0; nt < 2 * TN; ++nt) {
        const char* bb = st + SA + (wn * 32 * TN + nt * 16 + rr) * 32 + hh * 16;
        const bf16x8 g1 = *reinterpret_cast<const bf16x8*>(bb + sl * BN * 32);            // [b0|b1]
        const bf16x8 g3 = *reinterpret_cast<const bf16x8*>(bb + (2 - 2 * sl) * BN * 32);  // [b2|b0]
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          acc16[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[mt][2], g3, acc16[mt][nt], 0, 0, 0);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          acc16[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[mt][1], g1, acc16[mt][nt], 0, 0, 0);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          acc16[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[mt][0], g1, acc16[mt][nt], 0, 0, 0);
      }
      return;
    }
    const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
#pragma unroll
    for (int q = 0; q < KS; ++q) {
      const char* sq = st + q * kSub;
      V8 a[TM][P];
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) {
        const int lr = wm * 32 * TM + mi * 32 + r;
        const int off = lr * 32 + ((h ^ (((a0 + lr) >> 3) & 1)) << 4);
#pragma unroll
        for (int p = 0; p < P; ++p) a[mi][p] = *reinterpret_cast<const V8*>(sq + p * BM * 32 + off);
      }
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        V8 b[P];
#pragma unroll
        for (int p = 0; p < P; ++p)
          b[p] = *reinterpret_cast<const V8*>(sq + SA + p * BN * 32 +
                                              x3_off(wn * 32 * TN + ni * 32 + r, h));
        f32x16 c[TM];
#pragma unroll
        for (int mi = 0; mi < TM; ++mi) c[mi] = acc[mi][ni];
        mfma_products<F, TM>(a, b, c);
#pragma unroll
        for (int mi = 0; mi < TM; ++mi) acc[mi][ni] = c[mi];
      }
    }
  }

  // this wave's DMAs but the N youngest landed, its LDS reads done; barrier
  template <int N>
  __device__ __forceinline__ static void ring_barrier() {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
  }

  // One tile: A rows from imgA (already offset to the block's first row; mA
  // image rows per part), B likewise; nk K-steps of 16.
  __device__ __forceinline__ void run(const __bf16* imgA, int64_t mA, const __bf16* imgB,
                                      int64_t mB, int nk, char* smem) {
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), wm = w / WN, wn = w % WN;
    const __amdgpu_buffer_rsrc_t rA =
        __builtin_amdgcn_make_buffer_rsrc((void*)imgA, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rB =
        __builtin_amdgcn_make_buffer_rsrc((void*)imgB, (short)0, 0x7fffffff, 0x00020000);
    zero();
    dma(smem, rA, mA, rB, mB, 0);
    if (NS == 3 && nk > 1) {
      dma(smem + kStage, rA, mA, rB, mB, 1);
      ring_barrier<kDmas>();
    } else {
      ring_barrier<0>();
    }
    if (NS == 2) {
      for (int k = 0; k < nk; k += 2) {
        step<0>(k, nk, rA, mA, rB, mB, smem, wm, wn);
        if (k + 1 < nk) step<1>(k + 1, nk, rA, mA, rB, mB, smem, wm, wn);
      }
      return;
    }
    // unrolled by three: the ring's stage bases are compile-time constants
    for (int k = 0; k < nk; k += 3) {
      step<0>(k, nk, rA, mA, rB, mB, smem, wm, wn);
      if (k + 1 < nk) step<1>(k + 1, nk, rA, mA, rB, mB, smem, wm, wn);
      if (k + 2 < nk) step<2>(k + 2, nk, rA, mA, rB, mB, smem, wm, wn);
    }
  }

  template <int S>
  __device__ __forceinline__ void step(int k, int nk, __amdgpu_buffer_rsrc_t rA, int64_t mA,
                                       __amdgpu_buffer_rsrc_t rB, int64_t mB, char* smem, int wm,
                                       int wn) {
    if (NS == 2) {  // tile k+1 into the other stage, waited for at the end
      if (k + 1 < nk) dma(smem + ((S + 1) % 2) * kStage, rA, mA, rB, mB, k + 1);
      compute(smem + S * kStage, wm, wn);
      if (k + 1 < nk) ring_barrier<0>();
      return;
    }
    const bool more2 = k + 2 < nk;
    if (more2) dma(smem + ((S + 2) % 3) * kStage, rA, mA, rB, mB, k + 2);
    compute(smem + S * kStage, wm, wn);
    if (k + 1 < nk) {
      if (more2)
        ring_barrier<kDmas>();
      else
        ring_barrier<0>();
    }
  }
};

}  // namespace dsvgd
