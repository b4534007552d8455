// phi_w1.hpp -- phi_mm (C = exp-fused K . Y on the FmtH2 split engine) with
// ONE wave per SIMD: 4 waves of 128 x 128 (256 accumulator registers each, in
// AGPRs), block 128 rows x 512 columns, 16-deep K-steps.
//
// What differs from NNX3Tile (gemm_x3.hpp, 8 waves of 64 x 128):
//   * B (the Yx image) never goes through LDS: a wave's 128 columns are its
//     own, so each lane loads its MFMA B fragments straight from the image
//     (buffer_load_dwordx4, one K-step ahead, double-buffered in VGPRs);
//   * the D panel is loaded by the thread that stages it (two dwordx4, three
//     K-steps ahead) -- no LDS-DMA anywhere, so every wait is the compiler's
//     own counted vmcnt;
//   * LDS holds only the staged A image (2 stages x 8 KiB); each wave reads
//     all 128 rows of it (64 KiB of fragment reads per K-step per block
//     instead of 96 KiB);
//   * each K-step is one basic block (branch-free staging: clamped loads past
//     the range, masked row sums, the diagonal by compare/select), so the
//     scheduler can interleave the staging VALU with the 48 MFMAs.
// Symmetric D layout: the K-steps left of a row block's diagonal tile exist
// only as the stored tiles (J, I), J < I -- transposed.  DS = 1 walks those:
// each lane loads 32 contiguous bytes of the stored tile (8 consecutive rows
// i of one column j: the same two dwordx4 as a plain K-step), the wave
// transposes its 32 x 16 share through a private 2.75 KiB LDS scratch (two
// ds_write_b128 and eight ds_read_b32 per lane, conflict-free layout) one
// K-step before staging it, and stages exactly as a plain K-step.
#pragma once
#include "gemm_x3.hpp"

namespace dsvgd {

struct PhiW1 {
  static constexpr int kThreads = 256;
  static constexpr int BM = 128, BC = 512, BJ = 16, P = 2;
  static constexpr int SA = P * BM * 32;  // one stage's A image (8 KiB)
  static constexpr int kSmemBytes = 2 * SA;
  // DS = 1: per-wave transpose scratch, [16 j][kScrLd floats] for the wave's
  // 32 rows; kScrLd = 44: the 16-byte writes of 8 lanes and the dword reads
  // of 64 lanes each hit 64 distinct banks
  static constexpr int kScrLd = 44;
  static constexpr int kScrBytes = 16 * kScrLd * 4;
};

// VALU instructions placed after each of a K-step's first 16 MFMAs (the
// staging of the next A image); 2 / 6 / 0 measured slower (profiles/r6g)
constexpr int kW1Sgb = 4;
__device__ __forceinline__ f32x4 w1_load(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
__device__ __forceinline__ f32x4 w1_load_nt(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 2));
}

// A: panel row of the block (panel layout, 128 x 16 fp32 panels); Yx: FmtH2
// image [kstep][part][column][16 k]; K range [kchunk z, +kchunk) of K.
// DS (compile-time dsplit): 0 = the K range [kchunk z, +kchunk) (full D
// layout); on the symmetric layout (m == n, row0 == 0) 1 = the transposed
// K-steps left of a row block's diagonal tile, 2 = the plain ones from it on
// (the hybrid's two launches; slices land in slice0 + z).
// The pair-split layout of a DistSampler rank:
//   DS 0 with ks_wrap > 0: a cyclic window of K-steps -- window column k is
//     global K-step (ks_begin + k) mod ks_wrap (of both D and the image);
//   DS 3: a TRANSPOSED rectangle -- output row block `by` is D's column tile
//     tcol0 + by, the K-steps run down D's rows from A (A: the first of them,
//     a panel-row boundary), and the image K-step of D row j is ks_begin + j/16
//     (the owned rows' place in the interacting set): C = K(rows, cols)^T Y_rows,
//     the partial a rank sends to the owner of those columns.
//   DS 4: the symmetric layout's whole row in ONE launch: slice z of row
//     block by takes the contiguous K range [z kchunk, +kchunk), walked
//     ascending -- its transposed K-steps (left of the row block, as DS 1)
//     first, then the plain ones (as DS 2).  Every block of a slice is at the
//     same K-step at the same time whatever its row, and the blocks of one
//     XCD share a slice (xmap), so the Yx K-steps they read are the same
//     ones: one fetch per XCD instead of one per block walk.
// NI: 32-column tiles per wave (4: the 512-column block, one wave per SIMD;
// 2: 256-column blocks of 64 columns per wave, 128 accumulators -- two
// blocks per CU).  EXP = false: f = identity with the FmtH2 A scale (logreg
// G . Xd, DS 0 only): no exp, no diagonal, no row sums, no select state.
template <int DS, int NI = 4, bool EXP = true>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void phi_w1_kernel(
    const float* A, int64_t a_npad, const _Float16* Yx, int64_t ldy,
    int64_t K, int64_t kchunk, const dsvgd_select_state* __restrict__ st, float* __restrict__ C,
    int64_t ldc, float* __restrict__ rowsum, int64_t m, int64_t row0, int sym,
    const float* __restrict__ colinv, int slice0, const float* __restrict__ gate, int gate_on,
    int ks_begin = 0, int ks_wrap = 0, int tcol0 = 0, int t_per = 0, int t_first = 0,
    int t_nblk = 1, int64_t t_ostride = 0) {
  static_assert(NI == 4 || NI == 2, "NI: 4 or 2 column tiles per wave");
  static_assert(EXP || DS == 0, "the identity form is DS 0 only");
  const bool want_rs = EXP || rowsum != nullptr;   // (before the slice offset below)
  if (gate && ((*gate != 0.f) != (gate_on != 0))) return;  // the FmtH2 range guard (nn_x3_kernel)
  using F = FmtH2;
  constexpr int BC = 4 * 32 * NI;   // block columns
  using V8 = F::V8;
  constexpr int P = PhiW1::P;
  constexpr bool TRK = DS == 1 || DS == 3 || DS == 4;  // a transposed phase exists
  __shared__ __attribute__((aligned(16))) char smem[PhiW1::kSmemBytes + (TRK ? 4 * PhiW1::kScrBytes : 0)];
  const int t = threadIdx.x, lane = t & 63, r = lane & 31, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  // DS 1 / 2: a row block's slices dispatched back to back, longest first
  // (the transposed part grows with the row, the plain part shrinks)
  const int64_t lin = (int64_t)blockIdx.z * gridDim.y + blockIdx.y;
  // DS 4 and DS 0 with xmap (t_per = 1; gridDim.z | 8, 8 | blocks): linear
  // block id 8 q + x (x: the XCD it is dispatched to) -> slice x mod Z, and
  // u = (8 / Z) q + x / Z -> column block u mod gridDim.x, row block
  // u / gridDim.x -- the blocks running on one XCD walk the same K range, so
  // they read the same Yx K-steps
  const bool xm = ((DS == 4 || DS == 0) && t_per == 1) || (DS == 3 && t_per > 0 && tcol0 == 1);
  const int64_t lid = lin * gridDim.x + blockIdx.x;
  const int64_t xu = (lid >> 3) * (8 / gridDim.z) + (lid & 7) / gridDim.z;
  const int64_t cbx = xm ? xu % gridDim.x : blockIdx.x;
  const int64_t by = xm ? xu / gridDim.x
                   : DS == 2 ? lin / gridDim.z
                   : DS == 1 ? (int64_t)gridDim.y - 1 - lin / gridDim.z : blockIdx.y;
  const int64_t bz = xm ? (lid & 7) % gridDim.z
                   : (DS == 1 || DS == 2) ? lin % gridDim.z : blockIdx.z;
  // DS 3 batched over several column blocks of D (t_per > 0: t_per row
  // blocks of output per part; part q is D's column block (t_first + q) mod
  // t_nblk, its output t_ostride floats after part q - 1's; split-K slice z
  // of all parts after slice z - 1's)
  const bool tb = DS == 3 && t_per > 0;
  const int64_t tpart = tb ? by / t_per : 0;
  const int64_t byl = tb ? by % t_per : by;
  const int64_t i0 = byl * PhiW1::BM;
  const int64_t c0 = cbx * BC + w * 32 * NI;
  // K-step k of this block is global K-step ks0 + kdir * k.  The symmetric
  // forms interleave the slices, slice z taking every Z-th K-step of its
  // range (DS 2 top-down from K, DS 1 up from 0): the blocks running together
  // then read the same Yx K-steps at the same time (L2 reuse), whatever row
  // they start from
  const int64_t kb0 = bz * kchunk, kend = min(K, kb0 + kchunk);
  int ks0 = (int)(kb0 / PhiW1::BJ) + (DS == 0 ? ks_begin : 0);
  int nsteps = kend > kb0 ? (int)((kend - kb0) / PhiW1::BJ) : 0;
  const int Z = (int)gridDim.z;
  const int kdir = DS == 2 ? -Z : DS == 1 ? Z : 1;
  // K-step index of window step ks (DS 0 cyclic window; ks_wrap == 0: none)
  auto wrapk = [&](int ks) { return (DS == 0 && ks_wrap > 0 && ks >= ks_wrap) ? ks - ks_wrap : ks; };
  // the image K-step of D-row K-step ks (DS 3: the owned rows' offset)
  const int kyoff = DS == 3 ? ks_begin : 0;
  if (DS == 2) {
    const int T = (int)((K - i0) / PhiW1::BJ);
    ks0 = (int)(K / PhiW1::BJ) - 1 - (int)bz;
    nsteps = T > bz ? (T - (int)bz + Z - 1) / Z : 0;
  } else if (DS == 1) {
    const int T = (int)(i0 / PhiW1::BJ);
    ks0 = (int)bz;
    nsteps = T > bz ? (T - (int)bz + Z - 1) / Z : 0;
  }
  // DS 4: the slice's transposed K-steps [ks0, ksp), then the plain ones
  // [ksp, ks0 + nsteps)
  const int ksp = DS == 4 ? (int)min(max(kb0, i0), kend) / PhiW1::BJ : 0;
  if (tb) {   // batched DS 3: slice z of part q at (z * parts + q) t_ostride
    const int64_t at = ((int64_t)bz * (gridDim.y / t_per) + tpart) * t_ostride;
    C += at;
    rowsum += at;
  } else {
    C += (int64_t)(slice0 + bz) * m * ldc;
    rowsum += (int64_t)(slice0 + bz) * roundup128(m);
  }
  const float scale = EXP ? -st->inv_h * kLog2e : 0.f;

  // D: the block's panel row; thread t stages row t >> 1, columns 8 (t & 1) .. +7
  const __amdgpu_buffer_rsrc_t rD = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(A + (i0 >> 7) * (a_npad >> 4) * kPanelElems), (short)0, 0x7fffffff, 0x00020000);
  // B: the wave's first column; lane (r, h) reads column r, half h of each 32-column tile
  const __amdgpu_buffer_rsrc_t rB =
      __builtin_amdgcn_make_buffer_rsrc((void*)(Yx + c0 * 16), (short)0, 0x7fffffff, 0x00020000);
  const int pstride = (int)(ldy * 32);        // bytes of one part image of one K-step
  const int vB = x3_off(r, h);                // column base is a multiple of 32
  const int vD = t * 32;
  const int srow = t >> 1, shalf = t & 1;
  const int aoff = x3_off(srow, shalf);       // this thread's 16 B of a part image row
  // diagonal: global row - the thread's first column at K-step 0, clamped to
  // int range (only |.| < 16 matters; DS 1 never meets it)
  auto diag0 = [&](int kfirst) {
    const int64_t dg = row0 + i0 + srow - 8 * shalf - (int64_t)kfirst * PhiW1::BJ;
    return (int)max(min(dg, (int64_t)(1 << 30)), (int64_t)-(1 << 30));
  };

  f32x16 acc[4][NI];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[mi][ni][q] = 0.f;
  float rs = 0.f;

  // symmetric layout (m == n, row0 == 0): K-steps left of the block's
  // diagonal tile (DS 1) read the stored tile (J, I) transposed
  const int symI = tb ? (int)(((t_first + tpart) % t_nblk) * t_per + byl)
                   : DS == 3 ? tcol0 + (int)by : (sym || DS == 4) ? (int)(i0 >> 7) : -1;
  const int64_t pcols = a_npad >> 4;
  // DS 1: lane (piece p = t >> 5, s = t & 31) loads rows i0 + 16 p + 8 (s & 1)
  // .. +7 of column j0 + (s >> 1): 32 contiguous bytes of panel I*8 + p
  const int vP = (t >> 5) * kPanelElems * 4 + (t & 31) * 32;
  // DS 1 scratch of this wave: element (i' = row - 32 w, j) at j * kScrLd + i'
  float* const scr = reinterpret_cast<float*>(smem + PhiW1::kSmemBytes + w * PhiW1::kScrBytes);
  const int sw_off = ((lane & 31) >> 1) * PhiW1::kScrLd + 16 * (lane >> 5) + 8 * (lane & 1);
  const int sr_off = 8 * shalf * PhiW1::kScrLd + (lane >> 1);

  // one phase: nsteps K-steps from global K-step ks0 (stride kdir), all
  // transposed (TR) or all plain
  auto phase = [&](auto TR_, const int ks0, const int nsteps, const int qd0) {
    constexpr bool TR = decltype(TR_)::value;
    if (nsteps <= 0) return;
    V8 b[NI][P];      // B fragments of the current K-step; column tile ni is
                      // reloaded for the next K-step right after its last MFMA
    f32x4 dr[4][2];   // D values: K-step k in dr[k & 3], loaded 3 K-steps ahead
    f32x4 tr[2];      // DS 1: K-step k+1's values, transposed during K-step k - 1
    const int last = nsteps - 1;
    auto loadB = [&](int ni, int k) {
      const int soff = (wrapk(ks0 + kdir * min(k, last)) + kyoff) * P * pstride;
#pragma unroll
      for (int p = 0; p < P; ++p)
        b[ni][p] = __builtin_bit_cast(V8, w1_load(rB, vB + ni * 1024, soff + p * pstride));
    };
    auto loadD = [&](f32x4 (&d)[2], int k) {
      const int kc = min(k, last);
      const int64_t j0 = (int64_t)wrapk(ks0 + kdir * kc) * PhiW1::BJ;
      if constexpr (TR) {
        const float* src = A + (((j0 >> 7) * pcols + symI * 8) * kPanelElems + (j0 & 127) * 16);
        const __amdgpu_buffer_rsrc_t rT =
            __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 0x7fffffff, 0x00020000);
        d[0] = w1_load_nt(rT, vP, 0);
        d[1] = w1_load_nt(rT, vP + 16, 0);
      } else {  // DS 0 (full layout) and DS 2 (from the diagonal tile on): plain
        const int soff = (int)(j0 >> 4) * kPanelElems * 4;
        d[0] = w1_load_nt(rD, vD, soff);
        d[1] = w1_load_nt(rD, vD + 16, soff);
      }
    };
    // DS 1: the wave's 32 rows x 16 columns of one K-step, from the load
    // layout (lane: 8 rows of one column) to the staging one (lane: 8
    // columns of one row), through the wave's scratch (in-order LDS: no
    // barrier, and the next transpose's writes follow this one's reads)
    auto transpose = [&](const f32x4 (&d)[2], f32x4 (&o)[2]) {
      *reinterpret_cast<f32x4*>(scr + sw_off) = d[0];
      *reinterpret_cast<f32x4*>(scr + sw_off + 4) = d[1];
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q >> 2][q & 3] = scr[sr_off + q * PhiW1::kScrLd];
    };
    // exp2 / diagonal / row sum / 2-part split of K-step k's 8 values -> stage
    auto stage = [&](char* st_, const f32x4 (&d)[2], int k) {
      // diagonal column among the thread's 8, or -1 / 8
      const int qd = max(min(qd0 - kdir * k * PhiW1::BJ, 8), -1);
      float e[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float v = q < 4 ? d[0][q] : d[1][q - 4];
        const float x = EXP ? __builtin_amdgcn_exp2f(fmaf(v, scale, F::kAScaleLog2))
                            : v * F::kAScale;   // G 2^15 (exact)
        e[q] = (EXP && !TR && qd == q) ? 0.f : x;
      }
      const float s = ((e[0] + e[1]) + (e[2] + e[3])) + ((e[4] + e[5]) + (e[6] + e[7]));
      rs += k <= last ? s : 0.f;
      V8 p0, p1;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const _Float16 a0 = (_Float16)e[q];
        p0[q] = a0;
        p1[q] = (_Float16)(e[q] - (float)a0);
      }
      *reinterpret_cast<V8*>(st_ + aoff) = p0;
      *reinterpret_cast<V8*>(st_ + PhiW1::BM * 32 + aoff) = p1;
    };
    auto barrier = []() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
    // K-step k (slot KS = k & 3) from stage cur: A(k+1) -> stage nxt; MFMAs
    // column tile by column tile, each tile's B reloaded for k+1; then D(k+3)
    // (DS 1: stages tr = K-step k+1, and transposes dt = D(k+2) into tr)
    auto step = [&](int k, const char* cur, char* nxt, const f32x4 (&ds_)[2], f32x4 (&dl)[2],
                    const f32x4 (&dt)[2]) {
      V8 a[4][P];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int p = 0; p < P; ++p)
          a[mi][p] = *reinterpret_cast<const V8*>(cur + p * PhiW1::BM * 32 + x3_off(mi * 32 + r, h));
      if constexpr (TR)
        stage(nxt, tr, k + 1);
      else
        stage(nxt, ds_, k + 1);
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        // small terms first, as mfma_products
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) acc[mi][ni] = mfma_fmt<F>(a[mi][1], b[ni][0], acc[mi][ni]);
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) acc[mi][ni] = mfma_fmt<F>(a[mi][0], b[ni][1], acc[mi][ni]);
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) acc[mi][ni] = mfma_fmt<F>(a[mi][0], b[ni][0], acc[mi][ni]);
        loadB(ni, k + 1);
      }
      if constexpr (TR) transpose(dt, tr);
      // one wave per SIMD: nothing else hides the staging VALU, so spread it
      // between the MFMAs (cdna_hip_programming.md T19): the A fragment reads,
      // then 16 MFMAs each followed by up to kW1Sgb VALU (the staging of
      // A(k+1)), its two LDS stores, then the other 32 MFMAs with the 8 B loads
      // (DS 1: and the transpose of K-step k+2 -- two stores, eight reads --
      // early among them, so its reads land before the closing barrier)
      __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
      for (int i = 0; i < 4 * NI; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, kW1Sgb, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x200, 2, 0);
#pragma unroll
      for (int i = 0; i < 8 * NI; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (TR && i == 1) __builtin_amdgcn_sched_group_barrier(0x200, 2, 0);
        if (TR && i >= 2 && i < 10) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        if (i % 4 == 3) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      }
      loadD(dl, k + 3);
    };

    // prologue: B(0), D(0..2); A(0) -> stage 0 (DS 1: D(0), D(1) transposed)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) loadB(ni, 0);
    loadD(dr[0], 0);
    loadD(dr[1], 1);
    loadD(dr[2], 2);
    if constexpr (TR) {
      transpose(dr[0], tr);
      stage(smem, tr, 0);
      transpose(dr[1], tr);
    } else {
      stage(smem, dr[0], 0);
    }
    barrier();
    // unrolled by 8 (the D ring's slots are compile-time); the compiler's
    // wait counts are exact inside the body, conservative at the loop head
    // (unroll 4 -> 8: h2:full phi_mm 11.25 -> 11.05 ms, profiles/r6g)
    for (int k = 0; k < nsteps; k += 8) {
      step(k, smem, smem + PhiW1::SA, dr[1], dr[3], dr[2]);
      barrier();
      if (k + 1 >= nsteps) break;
      step(k + 1, smem + PhiW1::SA, smem, dr[2], dr[0], dr[3]);
      barrier();
      if (k + 2 >= nsteps) break;
      step(k + 2, smem, smem + PhiW1::SA, dr[3], dr[1], dr[0]);
      barrier();
      if (k + 3 >= nsteps) break;
      step(k + 3, smem + PhiW1::SA, smem, dr[0], dr[2], dr[1]);
      barrier();
      if (k + 4 >= nsteps) break;
      step(k + 4, smem, smem + PhiW1::SA, dr[1], dr[3], dr[2]);
      barrier();
      if (k + 5 >= nsteps) break;
      step(k + 5, smem + PhiW1::SA, smem, dr[2], dr[0], dr[3]);
      barrier();
      if (k + 6 >= nsteps) break;
      step(k + 6, smem, smem + PhiW1::SA, dr[3], dr[1], dr[0]);
      barrier();
      if (k + 7 >= nsteps) break;
      step(k + 7, smem + PhiW1::SA, smem, dr[0], dr[2], dr[1]);
      barrier();
    }
  };
  if constexpr (DS == 4) {
    phase(std::true_type{}, ks0, ksp - ks0, 0);
    phase(std::false_type{}, ksp, ks0 + nsteps - ksp, diag0(ksp));
  } else {
    phase(std::integral_constant<bool, DS == 1 || DS == 3>{}, ks0, nsteps, diag0(ks0));
  }

  // epilogue (nn_x3_kernel's): C = acc * colinv * 2^-15; row sums by column block 0
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const int64_t col = c0 + ni * 32 + r;
      const float cs = colinv[col] * (1.f / F::kAScale);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int64_t row = i0 + mi * 32 + c_row(q, lane);
        if (row < m) C[row * ldc + col] = acc[mi][ni][q] * cs;
      }
    }
  // (the identity form keeps its row sums when asked for: with them dead
  // the compiler's schedule of the unrolled loop spilled ~3700 registers)
  {
    const float v = rs + __shfl_xor(rs, 1, 64);
    if (want_rs && cbx == 0 && shalf == 0 && i0 + srow < m)
      rowsum[i0 + srow] = v * (1.f / F::kAScale);
  }
}

}  // namespace dsvgd
