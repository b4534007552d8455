// sqdist.hip -- pairwise squared distances D_ij = ||x_i - x_j||^2 in the panel
// layout, plus the per-entry accounting of the exact median select.
//
// d > 2: Gram form on MFMA (v_mfma_f32_32x32x2_f32) over centred particles,
//   upper-triangle tiles only for a square block (mirror stored).  Roofline per
//   128x128 tile: 2*128*128*dp flop vs 64 KiB written -> MFMA-bound for dp >= 64.
// d <= 2: explicit differences on the VALU (torch.dist semantics) -- at d = 1
//   the Gram form's cancellation exceeds the 1e-5 phi tolerance and d = 2 is
//   within 2x of it (measured, scripts/precision_small_d.py); from d = 3 up
//   the MFMA path is as or more accurate than the pairwise one.
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "gemm_tiles.hpp"
#include "gemm_x3.hpp"
#include "gram_rs.hpp"
#include "gram_w1.hpp"
#include "select.hpp"

namespace dsvgd {

// The FmtH2 Gram (sqdist_x3w_kernel) runs 256-tile blocks, one per CU, on a
// 2-stage ring of 32-deep stages (two 16-deep image K-steps per barrier: -5 %
// vs 16-deep stages on a 3-stage ring), the bracket candidates staged 32 deep
// in the wave's own chunks of the just-retired ring stage (S = 1 4.83 -> 4.49
// ms).  Measured and dropped: half-tile blocks two per CU, with
// or without a staggered start; C = 0 first MFMAs; norms prefetched at a
// tile's first stage; transposed accumulators with 16-byte D stores.
constexpr int kGramKS = 2;
constexpr bool kGramWC = true;

using GramTile = NTTile<2, 2, 2, 2>;  // 128 x 128 block, 4 waves of 64 x 64

// Epilogue of one wave's part of a 128 x 128 distance tile (bi, bj) from the
// Gram accumulators: D = max(0, |y_i|^2 + |y_j|^2 - 2 y_i.y_j) (diagonal
// exactly 0, pads +inf) into the panel layout, the mirror tile for SYM
// off-diagonal tiles, and the select accounting (weight 2 for mirrored
// tiles).  The wave holds rows [rbase, rbase + 64) x columns [cbase, cbase +
// 32 NI) of the tile in acc[mi][ni] (mi < 2, ni < NI); srow / scol: the
// tile's 128 row / column norms.
// MIR = false: the launch never stores mirror tiles (compile-time: no
// register shuffles for them)
// RS (FmtH2 row images): the Gram comes out scaled by s_i s_j (per-row
// power-of-two scales); sirow holds 2 / s_i per row, sicol 1 / s_j per column,
// and 2 x.y = sirow_i (sicol_j acc) (exact power-of-two factors).
template <bool SYM, int smode, bool ZERO = false, class Tile = GramTile, int NI = 2,
          class SW = SlotWriter, bool MIR = true, bool RS = false>
__device__ __forceinline__ void sq_epilogue(Tile& tile, int bi, int bj, int64_t row0,
                                            int64_t m, int64_t n, int64_t n_pad,
                                            float* __restrict__ D, const float* srow,
                                            const float* scol, int rbase, int cbase,
                                            WindowHist& wh, uint32_t* shist, SW& sw,
                                            const SlotLayout& sl, int64_t slot,
                                            bool mirror_store = true, int r0t = 0,
                                            float c2 = 2.f, const float* sirow = nullptr,
                                            const float* sicol = nullptr) {
  // r0t: row0 / 128 when a row block's diagonal square runs SYM (bi is then
  // block-local, bj global; the mirror of (bi, bj) is (bj - r0t, bi + r0t))
  const int lane = threadIdx.x & 63;
  const bool mirror = SYM && bi + r0t != bj;
  const int64_t i0 = (int64_t)bi * GramTile::BM;  // within the owned block
  const int64_t j0 = (int64_t)bj * GramTile::BN;
  const uint32_t weight = mirror ? 2u : 1u;
  // one 32x32 sub-tile (16 values per lane) at a time.  Panel-layout
  // addresses: per lane one base pointer per sub-tile, the per-register part
  // ((r&3)*16 + (r>>2)*128 floats) is a compile-time immediate.
  const int h4 = 4 * (lane >> 5);
  float* const Dtile = D + ((int64_t)bi * (n_pad >> 4) + (int64_t)bj * 8) * kPanelElems;
  float* const Dmir = D + ((int64_t)(bj - r0t) * (n_pad >> 4) + (int64_t)(bi + r0t) * 8) * kPanelElems;
  // interior tiles (the bulk): no diagonal entry, every row and column valid
  // -> 3 VALU per value; edge / diagonal tiles take the guarded form
  const bool interior = (row0 + i0 + 128 <= j0 || j0 + 128 <= row0 + i0) && i0 + 128 <= m &&
                        j0 + 128 <= n;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const int cl = cbase + ni * 32 + (lane & 31);
      const int rb = rbase + mi * 32 + h4;  // this lane's first row in the sub-tile
      const float nj = scol[cl];
      const float ij = RS ? sicol[cl] : 1.f;
      // uniform tile base + zero-extended 32-bit lane offset: the SGPR-base
      // store form, no per-lane 64-bit address arithmetic
      float* const dp0 = Dtile + (uint32_t)((cl >> 4) * kPanelElems + (cl & 15) + rb * 16);
      // 2 y_i.y_j of register r (row rl)
      auto gram2 = [&](int r, int rl) {
        return RS ? sirow[rl] * (ij * tile.acc[mi][ni][r]) : c2 * tile.acc[mi][ni][r];
      };
      float v[16];
      if (interior) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rl = rb + (r & 3) + 8 * (r >> 2);
          v[r] = fmaxf(0.f, (srow[rl] + nj) - gram2(r, rl));
        }
      } else {
        const bool colok = j0 + cl < n;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rl = rb + (r & 3) + 8 * (r >> 2);
          float x;
          if (colok && i0 + rl < m)
            x = (row0 + i0 + rl == j0 + cl) ? 0.f : fmaxf(0.f, (srow[rl] + nj) - gram2(r, rl));
          else
            x = INFINITY;
          v[r] = x;
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r)
        // streamed out: nt, so D does not evict the Gram operands from L2
        __builtin_nontemporal_store(v[r], dp0 + (r & 3) * 16 + (r >> 2) * 128);
      if (MIR && mirror && mirror_store) {  // D[j][i]: 4 consecutive i per register quad -> 16-byte stores
        float* const mp0 = Dmir + (uint32_t)(cl * 16 + ((rbase >> 4) + mi * 2) * kPanelElems + h4);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          *reinterpret_cast<f32x4*>(mp0 + (q >> 1) * kPanelElems + 8 * (q & 1)) =
              f32x4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
      }
      if (smode == kSelHist) {
        if (mi == 0 && ni == 0) wh.init(v[0]);
        hist_account(wh, v, weight, shist);
      } else if (smode == kSelBracket) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          sw.add(v[r]);
          if (((mi * NI + ni) * 16 + r + 1) % SW::kDepth == 0) sw.flush();  // list depth
        }
      }
      if (ZERO) {
#pragma unroll
        for (int r = 0; r < 16; ++r) tile.acc[mi][ni][r] = 0.f;
      }
    }
  if (smode == kSelBracket) sw.finish(sl, slot, mirror);
}

// sq_epilogue for 16x16x32 tiles (NTX3Tile M16): the wave holds rows
// [rbase, rbase + 64) x columns [cbase, cbase + 32 TN) of tile (bi, bj) as
// acc16[mt][nt], lane (col lane & 15, rows 4 (lane >> 4) + r); a lane's 4
// values are 4 consecutive rows of one column, i.e. one 16-byte mirror store.
template <bool SYM, int smode, class Tile>
__device__ __forceinline__ void sq_epilogue16(Tile& tile, int bi, int bj, int64_t row0,
                                              int64_t m, int64_t n, int64_t n_pad,
                                              float* __restrict__ D, const float* srow,
                                              const float* scol, int rbase, int cbase,
                                              WindowHist& wh, uint32_t* shist, SlotWriter& sw,
                                              const SlotLayout& sl, int64_t slot,
                                              bool mirror_store, int r0t) {
  const int lane = threadIdx.x & 63, g4 = 4 * (lane >> 4);
  const bool mirror = SYM && bi + r0t != bj;
  const int64_t i0 = (int64_t)bi * 128, j0 = (int64_t)bj * 128;
  const uint32_t weight = mirror ? 2u : 1u;
  float* const Dtile = D + ((int64_t)bi * (n_pad >> 4) + (int64_t)bj * 8) * kPanelElems;
  float* const Dmir =
      D + ((int64_t)(bj - r0t) * (n_pad >> 4) + (int64_t)(bi + r0t) * 8) * kPanelElems;
  const bool interior = (row0 + i0 + 128 <= j0 || j0 + 128 <= row0 + i0) && i0 + 128 <= m &&
                        j0 + 128 <= n;
#pragma unroll
  for (int nt = 0; nt < 2 * Tile::TN_; ++nt) {
    const int cl = cbase + nt * 16 + (lane & 15);
    const float nj = scol[cl];
    const bool colok = j0 + cl < n;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int rb = rbase + mt * 16 + g4;  // this lane's first row
      float* const dp0 = Dtile + (cl >> 4) * kPanelElems + (cl & 15) + rb * 16;
      float v[4];
      if (interior) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          v[r] = fmaxf(0.f, (srow[rb + r] + nj) - 2.f * tile.acc16[mt][nt][r]);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rl = rb + r;
          float x;
          if (colok && i0 + rl < m)
            x = (row0 + i0 + rl == j0 + cl) ? 0.f
                                             : fmaxf(0.f, (srow[rl] + nj) - 2.f * tile.acc16[mt][nt][r]);
          else
            x = INFINITY;
          v[r] = x;
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
        __builtin_nontemporal_store(v[r], dp0 + r * 16);
      if (mirror && mirror_store)  // D[j][i], i = rb .. rb + 3
        *reinterpret_cast<f32x4*>(Dmir + ((rbase >> 4) + mt) * kPanelElems + (int64_t)cl * 16 +
                                  g4) = f32x4{v[0], v[1], v[2], v[3]};
      if (smode == kSelHist) {
        if (mt == 0 && nt == 0) wh.init(v[0]);
        hist_account(wh, v, weight, shist);
      } else if (smode == kSelBracket) {
#pragma unroll
        for (int r = 0; r < 4; ++r) sw.add(v[r]);
      }
      tile.acc16[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  if (smode == kSelBracket) sw.finish(sl, slot, mirror);
}

// Persistent form: a grid of (resident blocks per CU) x CUs; block b (on XCD
// b % 8 under round-robin dispatch) walks the logical tiles L = lo_x + u,
// lo_x + u + U, ... of its XCD's contiguous range (same L2-grouped order as
// above).  The first K-step of the next tile (and its norms) is loaded while
// the current tile's last K-step computes, so a tile's load latency hides
// under the previous tile's MFMAs and epilogue -- at dp = 256 a tile is only
// 8 K-steps, and that per-tile latency is what one-tile blocks lose.
// Candidate slots are per (logical tile, wave); the digit-1 histogram stays
// in LDS across a block's tiles (one global flush).
template <bool SYM, int smode>
__global__ __launch_bounds__(256, 2) void sqdist_persistent_kernel(
    const float* __restrict__ Y, int64_t ldy, const float* __restrict__ norms, int64_t row0,
    int64_t m, int64_t n, int64_t n_pad, int dp, float* __restrict__ D,
    dsvgd_select_state* __restrict__ st, float* __restrict__ cand, int64_t total) {
  __shared__ __attribute__((aligned(16))) float smem[GramTile::kSmemFloats];
  __shared__ uint32_t shist[DSVGD_RADIX_BINS];
  __shared__ float snorm[2][GramTile::BM + GramTile::BN];  // current / next tile
  float* const sA = smem;
  float* const sB = smem + GramTile::BM * GramTile::LDK;

  const int Tm = (int)(roundup128(m) / 128), Tn = (int)(n_pad / 128);
  const int t = threadIdx.x, w = t >> 6, wm = w >> 1, wn = w & 1;
  const int64_t x = blockIdx.x % kXcds, u = blockIdx.x / kXcds, U = gridDim.x / kXcds;
  const int64_t q = total / kXcds, rr = total % kXcds;
  const int64_t lo = x * q + min(x, rr);
  const int64_t hi = (int64_t)__builtin_amdgcn_readfirstlane((int)(lo + q + (x < rr ? 1 : 0)));
  SlotLayout sl(cand, total * 4, smode == kSelBracket ? st->cand_cap : 0);
  if (smode == kSelBracket) sl.publish(st, blockIdx.x);
  if (smode == kSelHist)
    for (int b = t; b < DSVGD_RADIX_BINS; b += 256) shist[b] = 0u;

  // next valid logical tile at or after L (padding tiles: empty slots)
  // (tile indices are block-uniform: readfirstlane keeps them -- and every
  // address derived from them -- in SGPRs)
  auto next_valid = [&](int64_t L, int& bi, int& bj) -> int64_t {
    for (; L < hi; L += U) {
      if (tile_at(L, Tm, Tn, SYM, bi, bj)) {
        bi = __builtin_amdgcn_readfirstlane(bi);
        bj = __builtin_amdgcn_readfirstlane(bj);
        return L;
      }
      if (smode == kSelBracket) slot_clear(sl, L * 4 + w);
    }
    return L;
  };
  auto norm_of = [&](int bi, int bj) -> float {
    return t < 128 ? norms[row0 + (int64_t)bi * 128 + t] : norms[(int64_t)bj * 128 + t - 128];
  };
  int bi, bj;
  int64_t L = next_valid((int64_t)__builtin_amdgcn_readfirstlane((int)(lo + u)), bi, bj);
  GramTile tile;
  tile.zero();  // the epilogue re-zeroes each sub-tile after consuming it
  const int nk = dp / GramTile::BK;
  int par = 0;
  if (L < hi) {  // stage K-step 0 of the first tile
    tile.load(Y + (row0 + (int64_t)bi * 128) * ldy, ldy, Y + (int64_t)bj * 128 * ldy, ldy, 0);
    snorm[0][t] = norm_of(bi, bj);
    tile.store(sA, sB);
  }
  __syncthreads();
  // Per K-step: issue the next stage's loads (the next tile's K-step 0 after
  // the last one), MFMAs on the staged one, barrier, write the next stage,
  // barrier.  The staging registers are dead again before the epilogue.
  while (L < hi) {
    int bin = 0, bjn = 0;
    const int64_t Ln = next_valid(L + U, bin, bjn);
    const bool has_next = Ln < hi;
    const float* Ab = Y + (row0 + (int64_t)bi * 128) * ldy;
    const float* Bb = Y + (int64_t)bj * 128 * ldy;
    const float* An = Y + (row0 + (int64_t)bin * 128) * ldy;
    const float* Bn = Y + (int64_t)bjn * 128 * ldy;
#pragma unroll 1
    for (int ks = 0; ks < nk; ++ks) {
      const bool last = ks + 1 == nk;
      // one load site (one register set): this tile's next K-step, or the
      // next tile's first
      const bool more = !last || has_next;
      float nrm = 0.f;
      if (more)
        tile.load(last ? An : Ab, ldy, last ? Bn : Bb, ldy, last ? 0 : (ks + 1) * GramTile::BK);
      if (last && has_next) nrm = norm_of(bin, bjn);
      tile.compute(sA, sB, wm, wn);
      __syncthreads();
      if (more) {
        tile.store(sA, sB);
        if (last) snorm[par ^ 1][t] = nrm;
      }
      __syncthreads();
    }
    const int64_t slot = L * 4 + w;
    WindowHist wh;
    SlotWriter sw;
    if (smode == kSelBracket) sw.begin(st, sl, slot);
    sq_epilogue<SYM, smode, true>(tile, bi, bj, row0, m, n, n_pad, D, snorm[par],
                                  snorm[par] + 128, wm * 64, wn * 64, wh, shist, sw, sl, slot);
    if (smode == kSelHist) wh.flush(shist);
    par ^= 1;
    L = Ln;
    bi = bin;
    bj = bjn;
  }
  if (smode == kSelHist) {
    __syncthreads();
    flush_block_hist(shist, st);
  }
}

// The persistent distance kernel on the split engines (gemm_x3.hpp): the
// Gram from the row image Yg of Y[:, :dp] (n_pad image rows), fp32-accurate,
// through a 2-stage LDS-DMA ring that runs across tile boundaries (the next
// tile's first K-step lands during this tile's last one); tile order and
// select accounting as sqdist_persistent_kernel.
// 256 x 256 tiles (8 waves of 64 x 128, one block per CU): twice the MFMAs
// per operand byte of a 128 x 128 form.  Each wave's 64 x 128
// region lies in one 128 x 128 sub-tile (2 BI + (wr >> 1), 2 BJ + wc); the
// epilogue runs per sub-tile (sub-tiles below the diagonal of a SYM diagonal
// tile, and past the padded matrix, are skipped).  Candidate slots: 8 per tile.
// M16: 16x16x32 MFMAs on an unswizzled Yg (FmtX3), else 32x32x16 on a
// swizzled one (FmtH2).
// F = FmtH2: Yg is the fp16 image of s_i Xc[i] with a power-of-two scale per
// ROW (rsc[i], dsvgd_pack_h2's / dsvgd_h2_rowscale's), so no particle's
// coordinates sit below another's fp16 window; the Gram comes out scaled by
// s_i s_j and the epilogue divides both back out (sq_epilogue RS).
// KS: 16-deep image K-steps per ring stage.
template <bool SYM, int smode, bool M16 = true, class F = FmtX3, int KS = 1, bool MIR = true>
__global__ __launch_bounds__(512, 1) void sqdist_x3w_kernel(
    const typename F::E* __restrict__ Yg, int64_t img_rows, const float* __restrict__ norms,
    int64_t row0, int64_t m, int64_t n, int64_t n_pad, int nk, float* __restrict__ D,
    dsvgd_select_state* __restrict__ st, float* __restrict__ cand, int64_t total_tiles,
    int layout, int Tm2, int Tc2, int bj_off, int r0t, int64_t slot_base, int64_t ns_total,
    const float* __restrict__ rsc) {
  // candidates staged in the retired ring stage (bracket mode, 32x32 form,
  // 32-deep stages)
  constexpr bool kWC = kGramWC && smode == kSelBracket && !M16 && KS == 2;
  using GramX3WTile = NTX3Tile<2, 4, 4, 2, 2, M16, F, KS, kWC>;
  static_assert(!kWC || GramX3WTile::kChunksPerWave * 1024 >= 64 * 32 * 4,
                "32-deep candidate lists fit the wave's chunks");
  constexpr int kT = GramX3WTile::kThreads;
  constexpr bool RS = F::P == 2;  // per-row scales
  __shared__ __attribute__((aligned(16))) char smem[GramX3WTile::kSmemBytes];
  __shared__ uint32_t shist[DSVGD_RADIX_BINS];
  __shared__ float snorm[512];  // the tile's 256 row norms, then its 256 column norms
  __shared__ float sinv[RS ? 512 : 1];  // RS: 2 / s_i of its rows, then 1 / s_j of its columns
  // bracket candidates staged per lane (SlotWriterLds) on the 32x32 form
  constexpr bool kLdsSlots = smode == kSelBracket && !M16;
  __shared__ float scand[kLdsSlots && !kWC ? (kT / 64) * 64 * kStageDepth : 1];

  // this launch: Tm2 x Tc2 256-tiles, global column tiles from bj_off
  // (SYM: the triangle of a Tm2 x Tm2 square; r0t = its row0 / 128)
  const int Tm = (int)(roundup128(m) / 128), Tn = (int)(n_pad / 128);  // 128-tiles
  // the wave index made provably uniform: tile, slot and D-tile bases derived
  // from it stay in SGPRs (stores take the SGPR-base + 32-bit offset form)
  const int t = threadIdx.x, w = __builtin_amdgcn_readfirstlane(t >> 6), wr = w / 2, wc = w % 2;
  const int64_t x = blockIdx.x % kXcds, u = blockIdx.x / kXcds, U = gridDim.x / kXcds;
  const int64_t q = total_tiles / kXcds, rr = total_tiles % kXcds;
  const int64_t lo = x * q + min(x, rr);
  const int64_t hi = (int64_t)__builtin_amdgcn_readfirstlane((int)(lo + q + (x < rr ? 1 : 0)));
  SlotLayout sl(cand, ns_total, smode == kSelBracket ? st->cand_cap : 0);
  if (smode == kSelBracket) sl.publish(st, blockIdx.x);
  if (smode == kSelHist)
    for (int b = t; b < DSVGD_RADIX_BINS; b += kT) shist[b] = 0u;

  // tile L -> 256-tile (BI, BJ); BJ returned as the global 256-column tile
  auto next_valid = [&](int64_t L, int& BI, int& BJ) -> int64_t {
    for (; L < hi; L += U) {
      if (tile_at(L, Tm2, Tc2, SYM, BI, BJ)) {
        BI = __builtin_amdgcn_readfirstlane(BI);
        BJ = __builtin_amdgcn_readfirstlane(BJ + bj_off);
        return L;
      }
      if (smode == kSelBracket) slot_clear(sl, slot_base + L * 8 + w);
    }
    return L;
  };
  GramX3WTile tile;
  auto issue = [&](char* stg, int BI, int BJ, int ks) {
    const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(Yg + (row0 + (int64_t)BI * 256) * 16), (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(Yg + (int64_t)BJ * 256 * 16), (short)0, 0x7fffffff, 0x00020000);
    tile.dma(stg, rA, img_rows, rB, img_rows, ks);
  };

  // tile (L, BI, BJ) done (its last stage retired from ring stage stg):
  // norms, per-sub-tile epilogue
  auto epilogue = [&](int64_t L, int BI, int BJ, int stg) {
    {
      const int64_t gi = t < 256 ? row0 + (int64_t)BI * 256 + t : (int64_t)BJ * 256 + t - 256;
      snorm[t] = gi < n_pad ? norms[gi] : 0.f;
      if constexpr (RS) sinv[t] = (t < 256 ? 2.f : 1.f) * pow2_inv(gi < n_pad ? rsc[gi] : 1.f);
    }
    __syncthreads();
    // this wave's 128-sub-tile
    const int bi = 2 * BI + (wr >> 1), bj = 2 * BJ + wc;
    const int64_t slot = slot_base + L * 8 + w;
    WindowHist wh;
    using SW = std::conditional_t<kWC, SlotWriterLdsT<32>,
                                  std::conditional_t<kLdsSlots, SlotWriterLds, SlotWriter>>;
    SW sw;
    if constexpr (kWC)
      sw.begin(st, sl, slot,
               reinterpret_cast<float*>(smem + stg * GramX3WTile::kStage +
                                        w * GramX3WTile::kChunksPerWave * 1024));
    else if constexpr (kLdsSlots)
      sw.begin(st, sl, slot, scand + w * 64 * kStageDepth);
    else if (smode == kSelBracket)
      sw.begin(st, sl, slot);
    if (bi >= Tm || bj >= Tn || (SYM && bi + r0t > bj)) {
      tile.zero();
      if (smode == kSelBracket) sw.finish(sl, slot, false);
    } else {
      if constexpr (M16)
        sq_epilogue16<SYM, smode>(tile, bi, bj, row0, m, n, n_pad, D, snorm + (wr >> 1) * 128,
                                  snorm + 256 + wc * 128, (wr & 1) * 64, 0, wh, shist, sw, sl,
                                  slot, layout == 0, r0t);
      else
        sq_epilogue<SYM, smode, true, GramX3WTile, 4, SW, MIR, RS>(
            tile, bi, bj, row0, m, n, n_pad, D, snorm + (wr >> 1) * 128,
            snorm + 256 + wc * 128, (wr & 1) * 64, 0, wh, shist, sw, sl, slot, layout == 0,
            r0t, 2.f, sinv + (wr >> 1) * 128, sinv + 256 + wc * 128);
    }
    if (smode == kSelHist) wh.flush(shist);
  };

  int BI = 0, BJ = 0;
  int64_t L = next_valid((int64_t)__builtin_amdgcn_readfirstlane((int)(lo + u)), BI, BJ);
  tile.zero();
  if (L < hi) issue(smem, BI, BJ, 0);
  GramX3WTile::template ring_barrier<0>();
  int ks = 0, stage = 0;
  int BIn = BI, BJn = BJ;
  int64_t Ln = L;
  while (L < hi) {
    int ksn = ks + 1;
    if (ksn == nk) {
      Ln = next_valid(L + U, BIn, BJn);
      ksn = 0;
    }
    const bool more = Ln < hi;
    if (more) issue(smem + (stage ^ 1) * GramX3WTile::kStage, BIn, BJn, ksn);
    tile.compute(smem + stage * GramX3WTile::kStage, wr, wc, (int)(row0 & 15));
    GramX3WTile::template ring_barrier<0>();
    if (ks + 1 == nk) {
      epilogue(L, BI, BJ, stage);
      L = Ln;
      BI = BIn;
      BJ = BJn;
    }
    ks = ksn;
    stage ^= 1;
  }
  if (smode == kSelHist) {
    __syncthreads();
    flush_block_hist(shist, st);
  }
}

// The one-kernel Gram units (128 x 256, four candidate slots each) run on
// gram_rs_kernel (split roles: MFMA waves + epilogue waves, gram_rs.hpp;
// default) or gram_w1_kernel (one wave per SIMD, the epilogue between the
// MFMAs); the same arguments, units, slots and D bits.  dsvgd_gram_set_rs.
static int g_gram_rs = 1;
// strips per unit group of the split-role Gram's walk (GramUnitWalk G: the
// strips whose image an XCD's L2 keeps while the column pairs stream past;
// B is fetched once per group).  8 or 16, dsvgd_gram_set_group.
static int g_gram_group = 8;
static void* g_gram_stamps = nullptr;  // dsvgd_gram_debug_stamps (probe 8)
static int gram_group() { return g_gram_rs ? g_gram_group : GramW1::kGroup; }

template <int SM, bool SY>
int launch_gram_units(const _Float16* Yg, int64_t img, const float* norms, const float* rsc,
                      int64_t row0, int64_t m, int64_t n, int64_t n_pad, int nk, float* D,
                      dsvgd_select_state* st, float* cand, int64_t tot, int Tm, int Tc, int jp_off,
                      int64_t base, int64_t ns_total, int w2all, const float* gate, hipStream_t s) {
  int bw = 0, rc = 0;
  if (g_gram_rs) {
    // the A/B probe variants (gram_rs.hpp VAR) exist for the headline's form only
    auto launch = [&](auto VAR_) {
      constexpr int VAR = decltype(VAR_)::value;
      auto go = [&](auto KG_) {
        constexpr int KG = decltype(KG_)::value;
        int r = persistent_blocks(
            reinterpret_cast<const void*>(&gram_rs_kernel<SM, SY, 0, VAR, KG>), &bw,
            GramRS::kThreads);
        if (r) return r;
        W2Out wo{};
        wo.X = (const float*)g_gram_stamps;
        hipLaunchKernelGGL((gram_rs_kernel<SM, SY, 0, VAR, KG>), dim3((unsigned)bw),
                           dim3(GramRS::kThreads), 0, s, Yg, img, norms, rsc, row0, m, n, n_pad,
                           nk, D, st, cand, tot, Tm, Tc, jp_off, base, ns_total, w2all, gate, wo);
        return check_launch("gram_rs");
      };
      // (the caller's unit count came from the same group: gram_group())
      return gram_group() == 16 ? go(std::integral_constant<int, 16>{})
                                : go(std::integral_constant<int, 8>{});
    };
    const int var = g_gram_rs - 1;
    if constexpr (SM == kSelBracket && SY) {
      if (var == 4) return launch(std::integral_constant<int, 4>{});
      if (var == 5) return launch(std::integral_constant<int, 8>{});
      if (var == 6) return launch(std::integral_constant<int, 16>{});
      if (var == 7 && g_gram_stamps) return launch(std::integral_constant<int, 32>{});
      if (var == 8) return launch(std::integral_constant<int, 64>{});
    }
    return launch(std::integral_constant<int, 0>{});
  }
  if ((rc = persistent_blocks(reinterpret_cast<const void*>(&gram_w1_kernel<SM, SY>), &bw,
                              GramW1::kThreads)))
    return rc;
  hipLaunchKernelGGL((gram_w1_kernel<SM, SY>), dim3((unsigned)bw), dim3(GramW1::kThreads), 0, s, Yg,
                     img, norms, rsc, row0, m, n, n_pad, nk, D, st, cand, tot, Tm, Tc, jp_off, base,
                     ns_total, w2all, gate);
  return check_launch("gram_w1");
}

// ---- the W2 cost on the split-role Gram (dsvgd_w2_cost_h2) -----------------
// One wave per image row: rows [0, n) hold Y - c, rows [n_pad, n_pad + m) X - c
// (c: Y's robust centre), zero-padded to dp columns; norms[row] = |row|^2 and
// rsc[row] = the row's FmtH2 power-of-two scale (1 for a zero or padding row).
__global__ __launch_bounds__(256) void w2_pack_kernel(const float* __restrict__ X, int64_t ldx,
                                                      int64_t m, const float* __restrict__ Y,
                                                      int64_t ldy, int64_t n, int64_t n_pad,
                                                      int64_t rows, int d, int dp,
                                                      const float* __restrict__ center,
                                                      float* __restrict__ Yc,
                                                      float* __restrict__ norms,
                                                      float* __restrict__ rsc) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* src = nullptr;
  if (row < n)
    src = Y + row * ldy;
  else if (row >= n_pad && row - n_pad < m)
    src = X + (row - n_pad) * ldx;
  float s2 = 0.f, mx = 0.f;
  for (int c = lane; c < dp; c += 64) {
    const float v = (src && c < d) ? src[c] - center[c] : 0.f;
    Yc[row * dp + c] = v;
    s2 = fmaf(v, v, s2);
    mx = fmaxf(mx, fabsf(v));
  }
  s2 = warp_sum(s2);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  if (lane == 0) {
    norms[row] = s2;
    rsc[row] = pow2_scale(mx);
  }
}

struct W2CostWs {
  int64_t n_pad, m_pad, dp, img, off_c, off_y, off_n, off_s, off_g, bytes;
  W2CostWs(int64_t m, int64_t n, int64_t d) {
    n_pad = roundup(n, 256);   // whole 256-column unit pairs
    m_pad = roundup(m, 128);
    dp = roundup(d, 256);      // the Gram's 16-K-step epilogue
    img = n_pad + m_pad + 256;
    auto al = [](int64_t b) { return roundup(b, 256); };
    off_c = 0;
    off_y = al(off_c + 4 * dp);
    off_n = al(off_y + 4 * img * dp);
    off_s = al(off_n + 4 * img);
    off_g = al(off_s + 4 * img);
    bytes = al(off_g + 2 * 2 * img * dp);
  }
};

// Yg's image rows per part: the padded matrix plus one 256-row tile of slack
// (a row block's last 256-row tile may start anywhere below n)
int64_t gram_img_rows(int64_t n) { return roundup(n, 128) + 256; }

template <int SM, class F = FmtX3>
int launch_sqdist_x3(const typename F::E* Yg, const float* norms, int64_t row0, int64_t m,
                     int64_t n, int64_t d, float* D, dsvgd_select_state* st, float* cand,
                     int layout, hipStream_t s, const float* rsc = nullptr) {
  const int64_t dp = roundup(d, 32), m_pad = roundup(m, 128), n_pad = roundup(n, 128);
  const int64_t img = gram_img_rows(n);
  const bool sym = m == n && row0 == 0;
  constexpr int KS = F::P == 2 ? kGramKS : 1;
  const int nk = (int)(dp / kX3Step / KS);  // ring stages per tile (dp is a multiple of 32)
  int rc = 0;
  int bs = 0, bn = 0;
  if ((rc = persistent_blocks(
           reinterpret_cast<const void*>(&sqdist_x3w_kernel<true, SM, F::P == 3, F, KS>), &bs, 512)))
    return rc;
  if ((rc = persistent_blocks(
           reinterpret_cast<const void*>(&sqdist_x3w_kernel<false, SM, F::P == 3, F, KS, false>), &bn,
           512)))
    return rc;
  const int Tn2 = (int)((n_pad / 128 + 1) / 2), Tm2 = (int)((m_pad / 128 + 1) / 2);
  struct Part {
    bool sym;
    int tm2, tc2, bj_off, r0t;
    int64_t total;
  } parts[3];
  int np = 0;
  if (sym) {
    parts[np++] = {true, Tn2, Tn2, 0, 0, tile_grid(Tn2, Tn2, true)};
  } else if (row0 % 256 == 0 && m % 256 == 0 && row0 + m <= n) {
    // a row block holds the diagonal square [row0, row0 + m)^2 of the
    // symmetric matrix: its upper triangle (+ mirror stores), and the
    // rectangles left and right of it
    const int c0 = (int)(row0 / 256), c1 = (int)((row0 + m) / 256), sq = (int)(m / 256);
    if (c0 > 0) parts[np++] = {false, sq, c0, 0, 0, tile_grid(sq, c0, false)};
    parts[np++] = {true, sq, sq, c0, (int)(row0 / 128), tile_grid(sq, sq, true)};
    if (Tn2 > c1) parts[np++] = {false, sq, Tn2 - c1, c1, 0, tile_grid(sq, Tn2 - c1, false)};
  } else {
    parts[np++] = {false, Tm2, Tn2, 0, 0, tile_grid(Tm2, Tn2, false)};
  }
  // FmtH2: the one-wave-per-SIMD Gram (gram_w1.hpp) for every part it
  // supports -- no mirror stores, the none / bracket select modes, K-steps
  // in sixteens, 16-row-aligned images; 128 x 256 units, 4 slots each
  const bool w1ok = F::P == 2 && SM != kSelHist && nk * KS % 16 == 0 && row0 % 16 == 0;
  auto w1part = [&](const Part& P) { return w1ok && !(P.sym && (sym ? layout : 0) == 0); };
  // every part spans the owned block's strips; its column pairs from bj_off
  auto w1walk = [&](const Part& P) {
    return GramUnitWalk((int)(m_pad / 128), P.tc2, P.sym, gram_group());
  };
  int64_t ns_total = 0;
  for (int i = 0; i < np; ++i)
    ns_total += w1part(parts[i]) ? w1walk(parts[i]).total() * GramW1::kSlots : parts[i].total * 8;
  int64_t base = 0;
  for (int i = 0; i < np; ++i) {
    const Part& P = parts[i];
    const int lay = sym ? layout : 0;
    if (w1part(P)) {
      const GramUnitWalk wk = w1walk(P);
      const int64_t tot = wk.total();
      if constexpr (F::P == 2) {
        rc = P.sym ? launch_gram_units<SM, true>((const _Float16*)Yg, img, norms, rsc, row0, m, n,
                                                 n_pad, nk * KS, D, st, cand, tot, wk.Tm, wk.Tc,
                                                 P.bj_off, base, ns_total, 0, nullptr, s)
                   : launch_gram_units<SM, false>((const _Float16*)Yg, img, norms, rsc, row0, m,
                                                  n, n_pad, nk * KS, D, st, cand, tot, wk.Tm,
                                                  wk.Tc, P.bj_off, base, ns_total, 0, nullptr, s);
        if (rc) return rc;
      }
      base += tot * GramW1::kSlots;
      continue;
    }
#define DSVGD_X3W(SY, B, LAY, R0T, MIR)                                                          \
  hipLaunchKernelGGL((sqdist_x3w_kernel<SY, SM, F::P == 3, F, KS, MIR>), dim3((unsigned)B),       \
                     dim3(512), 0, s, Yg, img, norms, row0, m, n, n_pad, nk, D, st, cand, P.total, \
                     LAY, P.tm2, P.tc2, P.bj_off, R0T, base, ns_total, rsc)
    if (P.sym && lay == 0)  // mirror stores
      DSVGD_X3W(true, bs, lay, P.r0t, true);
    else if (P.sym)
      DSVGD_X3W(true, bs, lay, P.r0t, false);
    else
      DSVGD_X3W(false, bn, 0, 0, false);
#undef DSVGD_X3W
    if ((rc = check_launch("sqdist_x3w"))) return rc;
    base += P.total * 8;
  }
  return 0;
}

// The pair-split layout of a DistSampler rank (dsvgd_sqdist_h2_parts):
// the owned row block's D as a list of parts -- its diagonal square (the
// 8-wave symmetric launch with mirror stores), rectangles on the
// one-wave-per-SIMD Gram (weight 2 when the rank holds the block pair
// {(r, c), (c, r)} for both owners), and rectangles computed only when the
// FmtH2 range guard trips (the fallback phi_mm then reads the whole row
// block; no select accounting).  One candidate-slot numbering over the
// accounted parts.
template <int SM>
int launch_sqdist_h2_parts(const _Float16* Yg, const float* norms, int64_t row0, int64_t m,
                           int64_t n, int64_t d, float* D, dsvgd_select_state* st, float* cand,
                           const dsvgd_gram_part* parts, int np, const float* gate,
                           hipStream_t s, const float* rsc) {
  using F = FmtH2;
  const int64_t dp = roundup(d, 32), n_pad = roundup(n, 128);
  const int64_t img = gram_img_rows(n);
  constexpr int KS = kGramKS;
  const int nk = (int)(dp / kX3Step / KS);
  int rc = 0, bs = 0;
  if ((rc = persistent_blocks(
           reinterpret_cast<const void*>(&sqdist_x3w_kernel<true, SM, false, F, KS>), &bs, 512)))
    return rc;
  auto walk = [&](const dsvgd_gram_part& P) {
    return GramUnitWalk((int)(P.rows / 128), (int)(P.cols / 256), false, gram_group());
  };
  int64_t ns_total = 0;
  for (int i = 0; i < np; ++i) {
    const dsvgd_gram_part& P = parts[i];
    if (P.kind == 1)
      ns_total += tile_grid(P.rows / 256, P.rows / 256, true) * 8;
    else if (P.kind == 0)
      ns_total += walk(P).total() * GramW1::kSlots;
  }
  int64_t base = 0;
  for (int i = 0; i < np; ++i) {
    const dsvgd_gram_part& P = parts[i];
    if (P.kind == 1) {  // the diagonal square, upper tiles + mirror stores
      const int sq = (int)(P.rows / 256);
      const int64_t tot = tile_grid(sq, sq, true);
      hipLaunchKernelGGL((sqdist_x3w_kernel<true, SM, false, F, KS, true>), dim3((unsigned)bs),
                         dim3(512), 0, s, Yg, img, norms, row0, m, n, n_pad, nk, D, st, cand, tot,
                         0, sq, sq, (int)(P.col0 / 256), (int)(row0 / 128), base, ns_total, rsc);
      if ((rc = check_launch("sqdist_x3w(diag)"))) return rc;
      base += tot * 8;
      continue;
    }
    const GramUnitWalk wk = walk(P);
    const int64_t tot = wk.total();
    float* Dp = D + P.row_off * n_pad;  // panel rows of the part's strips
    if (P.kind == 0) {
      rc = launch_gram_units<SM, false>(Yg, img, norms, rsc, row0 + P.row_off, P.rows, n, n_pad,
                                        nk * KS, Dp, st, cand, tot, wk.Tm, wk.Tc,
                                        (int)(P.col0 / 256), base, ns_total, (int)P.weight2,
                                        nullptr, s);
      base += tot * GramW1::kSlots;
    } else {
      rc = launch_gram_units<kSelNone, false>(Yg, img, norms, rsc, row0 + P.row_off, P.rows, n,
                                              n_pad, nk * KS, Dp, st, nullptr, tot, wk.Tm, wk.Tc,
                                              (int)(P.col0 / 256), 0, 0, 0, gate, s);
    }
    if (rc) return rc;
  }
  return 0;
}

// d <= 2 (supports up to 64): D_ij = sum_c (y_ic - y_jc)^2 from explicit differences on the VALU
// (what torch.dist(x, y)**2 computes per pair at experiments/logreg.py:61):
// no ||x||^2 - 2x.y cancellation, which at small d and a narrow median
// bandwidth costs more than the 1e-5 phi tolerance.  128 x 128 tile per block,
// 8 x 8 outputs per thread, both operand tiles transposed in LDS.
constexpr int kDirectMaxD = 64;     // the direct kernel's limit (dsvgd_sqdist_direct)
constexpr int kDirectDefaultD = 2;  // d <= this takes it in dsvgd_sqdist

template <int smode>
__global__ __launch_bounds__(256) void sqdist_direct_kernel(const float* __restrict__ Y,
                                                            int64_t ldy, int64_t row0, int64_t m,
                                                            int64_t n, int64_t n_pad, int d,
                                                            float* __restrict__ D,
                                                            dsvgd_select_state* __restrict__ st,
                                                            float* __restrict__ cand) {
  __shared__ __attribute__((aligned(16))) float sA[kDirectMaxD][128];
  __shared__ __attribute__((aligned(16))) float sB[kDirectMaxD][128];
  __shared__ uint32_t shist[DSVGD_RADIX_BINS];
  const int t = threadIdx.x;
  const int64_t i0 = (int64_t)blockIdx.y * 128, j0 = (int64_t)blockIdx.x * 128;
  if (smode == kSelHist)
    for (int b = t; b < DSVGD_RADIX_BINS; b += 256) shist[b] = 0u;
  for (int e = t; e < 128 * d; e += 256) {
    const int r = e / d, k = e % d;
    sA[k][r] = Y[(row0 + i0 + r) * ldy + k];
    sB[k][r] = Y[(j0 + r) * ldy + k];
  }
  __syncthreads();
  const int ty = t >> 4, tx = t & 15;
  float acc[8][8];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) acc[a][b] = 0.f;
  for (int k = 0; k < d; ++k) {
    const f32x4 a0 = *reinterpret_cast<const f32x4*>(&sA[k][ty * 8]);
    const f32x4 a1 = *reinterpret_cast<const f32x4*>(&sA[k][ty * 8 + 4]);
    const f32x4 b0 = *reinterpret_cast<const f32x4*>(&sB[k][tx * 8]);
    const f32x4 b1 = *reinterpret_cast<const f32x4*>(&sB[k][tx * 8 + 4]);
    const float av[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
    const float bv[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const float df = av[a] - bv[b];
        acc[a][b] = fmaf(df, df, acc[a][b]);
      }
  }
  WindowHist wh;
  if (smode == kSelHist)
    wh.init((i0 + ty * 8 < m && j0 + tx * 8 < n) ? acc[0][0] : INFINITY);
  const int64_t nslots = (int64_t)gridDim.x * gridDim.y * 4;
  const int64_t slot = ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 4 + (t >> 6);
  SlotWriter sw;
  SlotLayout sl(cand, nslots, smode == kSelBracket ? st->cand_cap : 0);
  if (smode == kSelBracket) {
    sl.publish(st, (int64_t)blockIdx.y * gridDim.x + blockIdx.x);
    sw.begin(st, sl, slot);
  }
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    const int64_t gi = i0 + ty * 8 + a;
    float v[8];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const int64_t gj = j0 + tx * 8 + b;
      v[b] = (gi < m && gj < n) ? acc[a][b] : INFINITY;
    }
    float* dst = D + panel_off(gi, j0 + tx * 8, n_pad);
    *reinterpret_cast<f32x4*>(dst) = f32x4{v[0], v[1], v[2], v[3]};
    *reinterpret_cast<f32x4*>(dst + 4) = f32x4{v[4], v[5], v[6], v[7]};
    if (smode == kSelHist) {
      hist_account(wh, v, 1u, shist);
    } else if (smode == kSelBracket) {
#pragma unroll
      for (int b = 0; b < 8; ++b) sw.add(v[b]);
    }
  }
  if (smode == kSelBracket) sw.finish(sl, slot, false);
  if (smode == kSelHist) {
    wh.flush(shist);
    __syncthreads();
    flush_block_hist(shist, st);
  }
}

// direct: the explicit-difference kernel (d <= kDirectMaxD), else the f32 Gram
template <int SM>
int launch_sqdist(const float* Y, int64_t ldy, const float* norms, int64_t row0, int64_t m,
                  int64_t n, int64_t d, float* D, dsvgd_select_state* st, float* cand,
                  hipStream_t s, bool direct) {
  const int64_t dp = roundup(d, 32), m_pad = roundup(m, 128), n_pad = roundup(n, 128);
  if (direct) {
    hipLaunchKernelGGL((sqdist_direct_kernel<SM>), dim3(n_pad / 128, m_pad / 128), dim3(256), 0, s,
                       Y, ldy, row0, m, n, n_pad, (int)d, D, st, cand);
    return check_launch("sqdist_direct");
  }
  const bool sym = m == n && row0 == 0;
  const int64_t T = n_pad / 128;
  const int64_t total = sym ? tile_grid(T, T, true) : tile_grid(m_pad / 128, T, false);
  {
    int blocks = 0;
    int rc = sym ? persistent_blocks(
                       reinterpret_cast<const void*>(&sqdist_persistent_kernel<true, SM>), &blocks)
                 : persistent_blocks(
                       reinterpret_cast<const void*>(&sqdist_persistent_kernel<false, SM>), &blocks);
    if (rc) return rc;
    const dim3 grid((unsigned)blocks);
    if (sym)
      hipLaunchKernelGGL((sqdist_persistent_kernel<true, SM>), grid, dim3(256), 0, s, Y, ldy, norms,
                         row0, m, n, n_pad, (int)dp, D, st, cand, total);
    else
      hipLaunchKernelGGL((sqdist_persistent_kernel<false, SM>), grid, dim3(256), 0, s, Y, ldy,
                         norms, row0, m, n, n_pad, (int)dp, D, st, cand, total);
    return check_launch("sqdist_persistent");
  }
}

}  // namespace dsvgd

using namespace dsvgd;

extern "C" {

int dsvgd_sqdist(const float* Y, int64_t ldy, const float* norms, int64_t row0, int64_t m,
                 int64_t n, int64_t d, float* D, int64_t ldd, int select_mode,
                 dsvgd_select_state* st, float* cand, void* stream) {
  DSVGD_REQUIRE(Y && norms && D, "null pointer");
  DSVGD_REQUIRE(m > 0 && n > 0 && row0 >= 0 && d > 0, "sizes");
  DSVGD_REQUIRE(select_mode >= 0 && select_mode <= 2, "select_mode must be 0, 1 or 2");
  DSVGD_REQUIRE(select_mode == 0 || st, "select mode needs a state");
  DSVGD_REQUIRE(select_mode != 2 || cand, "bracket mode needs a candidate buffer");
  const int64_t dp = roundup(d, 32);
  DSVGD_REQUIRE(ldy >= dp && ldy % 4 == 0, "ldy < roundup(d,32)");
  const int64_t m_pad = roundup(m, 128), n_pad = roundup(n, 128);
  DSVGD_REQUIRE(ldd == n_pad, "ldd must equal roundup(n,128) (panel layout)");
  DSVGD_REQUIRE(((uintptr_t)Y & 15) == 0 && ((uintptr_t)D & 15) == 0, "16-byte alignment");
  DSVGD_REQUIRE(m_pad / 128 <= 65535, "too many row tiles");
  hipStream_t s = (hipStream_t)stream;
  const bool direct = d <= kDirectDefaultD;
  switch (select_mode) {
    case kSelNone: return launch_sqdist<kSelNone>(Y, ldy, norms, row0, m, n, d, D, st, cand, s, direct);
    case kSelHist: return launch_sqdist<kSelHist>(Y, ldy, norms, row0, m, n, d, D, st, cand, s, direct);
    default: return launch_sqdist<kSelBracket>(Y, ldy, norms, row0, m, n, d, D, st, cand, s, direct);
  }
}

int dsvgd_sqdist_direct(const float* Y, int64_t ldy, const float* norms, int64_t row0, int64_t m,
                        int64_t n, int64_t d, float* D, int64_t ldd, int select_mode,
                        dsvgd_select_state* st, float* cand, void* stream) {
  DSVGD_REQUIRE(Y && D, "null pointer");
  DSVGD_REQUIRE(m > 0 && n > 0 && row0 >= 0 && d > 0, "sizes");
  DSVGD_REQUIRE(d <= kDirectMaxD, "the explicit-difference kernel supports d <= 64");
  DSVGD_REQUIRE(select_mode >= 0 && select_mode <= 2, "select_mode must be 0, 1 or 2");
  DSVGD_REQUIRE(select_mode == 0 || st, "select mode needs a state");
  DSVGD_REQUIRE(select_mode != 2 || cand, "bracket mode needs a candidate buffer");
  DSVGD_REQUIRE(ldy >= roundup(d, 32), "ldy < roundup(d,32)");
  DSVGD_REQUIRE(ldd == roundup(n, 128), "ldd must equal roundup(n,128) (panel layout)");
  DSVGD_REQUIRE(roundup(m, 128) / 128 <= 65535, "too many row tiles");
  hipStream_t s = (hipStream_t)stream;
  switch (select_mode) {
    case kSelNone: return launch_sqdist<kSelNone>(Y, ldy, norms, row0, m, n, d, D, st, cand, s, true);
    case kSelHist: return launch_sqdist<kSelHist>(Y, ldy, norms, row0, m, n, d, D, st, cand, s, true);
    default: return launch_sqdist<kSelBracket>(Y, ldy, norms, row0, m, n, d, D, st, cand, s, true);
  }
}

int dsvgd_sqdist_x3(const void* Yg, const float* norms, int64_t row0, int64_t m, int64_t n,
                    int64_t d, float* D, int64_t ldd, int select_mode, dsvgd_select_state* st,
                    float* cand, int layout, void* stream) {
  DSVGD_REQUIRE(Yg && norms && D, "null pointer");
  DSVGD_REQUIRE(m > 0 && n > 0 && row0 >= 0 && row0 + m <= n && d > 0, "sizes");
  DSVGD_REQUIRE(select_mode >= 0 && select_mode <= 2, "select_mode must be 0, 1 or 2");
  DSVGD_REQUIRE(select_mode == 0 || st, "select mode needs a state");
  DSVGD_REQUIRE(select_mode != 2 || cand, "bracket mode needs a candidate buffer");
  const int64_t m_pad = roundup(m, 128), n_pad = roundup(n, 128), dp = roundup(d, 32);
  DSVGD_REQUIRE(ldd == n_pad, "ldd must equal roundup(n,128) (panel layout)");
  DSVGD_REQUIRE(((uintptr_t)Yg & 15) == 0 && ((uintptr_t)D & 15) == 0, "16-byte alignment");
  DSVGD_REQUIRE(m_pad / 128 <= 65535, "too many row tiles");
  DSVGD_REQUIRE(dp * gram_img_rows(n) * 6 < ((int64_t)1 << 31),
                "image too large for 32-bit buffer offsets");
  DSVGD_REQUIRE(layout == 0 || (layout == 1 && m == n && row0 == 0),
                "layout 1 (symmetric) needs the whole matrix: m == n, row0 == 0");
  const __bf16* yg = (const __bf16*)Yg;
  hipStream_t s = (hipStream_t)stream;
  switch (select_mode) {
    case kSelNone: return launch_sqdist_x3<kSelNone>(yg, norms, row0, m, n, d, D, st, cand, layout, s);
    case kSelHist: return launch_sqdist_x3<kSelHist>(yg, norms, row0, m, n, d, D, st, cand, layout, s);
    default: return launch_sqdist_x3<kSelBracket>(yg, norms, row0, m, n, d, D, st, cand, layout, s);
  }
}

int dsvgd_sqdist_h2(const void* Yg, const float* norms, int64_t row0, int64_t m, int64_t n,
                    int64_t d, float* D, int64_t ldd, int select_mode, dsvgd_select_state* st,
                    float* cand, int layout, const float* rowscale, void* stream) {
  DSVGD_REQUIRE(Yg && norms && D && rowscale, "null pointer");
  DSVGD_REQUIRE(m > 0 && n > 0 && row0 >= 0 && row0 + m <= n && d > 0, "sizes");
  DSVGD_REQUIRE(select_mode >= 0 && select_mode <= 2, "select_mode must be 0, 1 or 2");
  DSVGD_REQUIRE(select_mode == 0 || st, "select mode needs a state");
  DSVGD_REQUIRE(select_mode != 2 || cand, "bracket mode needs a candidate buffer");
  const int64_t m_pad = roundup(m, 128), n_pad = roundup(n, 128), dp = roundup(d, 32);
  DSVGD_REQUIRE(ldd == n_pad, "ldd must equal roundup(n,128) (panel layout)");
  DSVGD_REQUIRE(((uintptr_t)Yg & 15) == 0 && ((uintptr_t)D & 15) == 0, "16-byte alignment");
  DSVGD_REQUIRE(m_pad / 128 <= 65535, "too many row tiles");
  DSVGD_REQUIRE(dp * gram_img_rows(n) * 4 < ((int64_t)1 << 31),
                "image too large for 32-bit buffer offsets");
  DSVGD_REQUIRE(layout == 0 || (layout == 1 && m == n && row0 == 0),
                "layout 1 (symmetric) needs the whole matrix: m == n, row0 == 0");
  const _Float16* yg = (const _Float16*)Yg;
  hipStream_t s = (hipStream_t)stream;
  switch (select_mode) {
    case kSelNone:
      return launch_sqdist_x3<kSelNone, FmtH2>(yg, norms, row0, m, n, d, D, st, cand, layout, s,
                                               rowscale);
    case kSelHist:
      return launch_sqdist_x3<kSelHist, FmtH2>(yg, norms, row0, m, n, d, D, st, cand, layout, s,
                                               rowscale);
    default:
      return launch_sqdist_x3<kSelBracket, FmtH2>(yg, norms, row0, m, n, d, D, st, cand, layout, s,
                                                  rowscale);
  }
}

size_t dsvgd_w2_cost_h2_workspace_bytes(int64_t m, int64_t n, int64_t d) {
  if (m <= 0 || n <= 0 || d <= 0) return 0;
  return (size_t)W2CostWs(m, n, d).bytes;
}

static int g_w2_cost_nt = 1;
int dsvgd_w2_set_cost_nt(int on) {
  const int prev = g_w2_cost_nt;
  g_w2_cost_nt = on ? 1 : 0;
  return prev;
}

static int g_w2_cost_lines = 1;
int dsvgd_w2_set_cost_lines(int on) {
  const int prev = g_w2_cost_lines;
  g_w2_cost_lines = on ? 1 : 0;
  return prev;
}

int dsvgd_w2_cost_h2(const float* X, int64_t ldx, int64_t m, const float* Y, int64_t ldy,
                     int64_t n, int64_t d, float* C, int64_t ldc, void* ws, float tau,
                     uint32_t* cstat, void* stream) {
  DSVGD_REQUIRE(X && Y && C && ws, "null pointer");
  DSVGD_REQUIRE(m > 0 && n > 0 && d > 0 && d <= 1024 && ldx >= d && ldy >= d, "sizes (d <= 1024)");
  const W2CostWs w(m, n, d);
  DSVGD_REQUIRE(ldc >= w.n_pad && ldc % 4 == 0 && ((uintptr_t)C & 15) == 0,
                "C: ldc >= roundup(n, 256), a multiple of 4, 16-byte aligned rows");
  DSVGD_REQUIRE(((uintptr_t)ws & 255) == 0, "workspace: 256-byte aligned");
  DSVGD_REQUIRE(w.dp * w.img * 4 < ((int64_t)1 << 31) && 127 * ldc * 4 + 1024 < ((int64_t)1 << 31),
                "too large for the Gram's 32-bit offsets");
  DSVGD_REQUIRE(tau >= 0.f && tau <= 1.f, "tau in [0, 1]");
  hipStream_t s = (hipStream_t)stream;
  char* base = (char*)ws;
  float* cen = (float*)(base + w.off_c);
  float* Yc = (float*)(base + w.off_y);
  float* nrm = (float*)(base + w.off_n);
  float* rs = (float*)(base + w.off_s);
  void* Yg = base + w.off_g;
  if (cstat && hipMemsetAsync(cstat, 0, 2 * sizeof(uint32_t), s) != hipSuccess)
    return check_launch("w2 cost stat memset");
  int rc = dsvgd_colcenter(Y, ldy, n, d, cen, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(w2_pack_kernel, dim3((unsigned)((w.img + 3) / 4)), dim3(256), 0, s, X, ldx, m,
                     Y, ldy, n, w.n_pad, w.img, (int)d, (int)w.dp, cen, Yc, nrm, rs);
  if ((rc = check_launch("w2_pack"))) return rc;
  if ((rc = dsvgd_h2_rowsplit_rows(Yc, w.dp, w.img, w.dp, w.img, w.dp, rs, Yg, stream))) return rc;
  const GramUnitWalk wk((int)(w.m_pad / 128), (int)(w.n_pad / 256), false);
  W2Out wo;
  wo.X = X;
  wo.Y = Y;
  wo.ldx = ldx;
  wo.ldy = ldy;
  wo.ldc = ldc;
  wo.d = (int)d;
  wo.tau = tau;
  wo.stat = cstat;
  wo.nt = g_w2_cost_nt;
  wo.lines = g_w2_cost_lines;
  wo.vec = (d % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0 && ((uintptr_t)X & 15) == 0 &&
            ((uintptr_t)Y & 15) == 0)
               ? 1
               : 0;
  int bw = 0;
  if ((rc = persistent_blocks(reinterpret_cast<const void*>(&gram_rs_kernel<kSelNone, false, 1>),
                              &bw, GramRS::kThreads)))
    return rc;
  hipLaunchKernelGGL((gram_rs_kernel<kSelNone, false, 1>), dim3((unsigned)bw),
                     dim3(GramRS::kThreads), 0, s, (const _Float16*)Yg, w.img, nrm, rs, w.n_pad, m,
                     n, w.n_pad, (int)(w.dp / 16), C, (dsvgd_select_state*)nullptr,
                     (float*)nullptr, wk.total(), wk.Tm, wk.Tc, 0, (int64_t)0, (int64_t)0, 0,
                     (const float*)nullptr, wo);
  return check_launch("gram_rs(w2 cost)");
}

int dsvgd_gram_debug_stamps(void* buf) {
  g_gram_stamps = buf;
  return 0;
}

int dsvgd_gram_set_group(int g) {
  const int prev = g_gram_group;
  g_gram_group = g == 16 ? 16 : 8;
  return prev;
}

int dsvgd_gram_set_rs(int on) {
  const int prev = g_gram_rs;
  g_gram_rs = on < 0 ? 0 : (on > 9 ? 1 : on);
  return prev;
}

int dsvgd_sqdist_h2_parts(const void* Yg, const float* norms, int64_t row0, int64_t m, int64_t n,
                          int64_t d, float* D, int64_t ldd, int select_mode,
                          dsvgd_select_state* st, float* cand, const dsvgd_gram_part* parts,
                          int nparts, const float* gate, const float* rowscale, void* stream) {
  DSVGD_REQUIRE(Yg && norms && D && rowscale && parts, "null pointer");
  DSVGD_REQUIRE(m > 0 && n > 0 && row0 >= 0 && row0 + m <= n && d > 0, "sizes");
  DSVGD_REQUIRE(select_mode == 0 || select_mode == 2, "select_mode must be 0 or 2 (bracket)");
  DSVGD_REQUIRE(select_mode == 0 || (st && cand), "bracket mode needs a state and candidates");
  const int64_t n_pad = roundup(n, 128), dp = roundup(d, 32);
  DSVGD_REQUIRE(ldd == n_pad, "ldd must equal roundup(n,128) (panel layout)");
  DSVGD_REQUIRE(dp % 256 == 0, "parts need roundup(d, 32) % 256 == 0 (the one-wave Gram)");
  DSVGD_REQUIRE(row0 % 256 == 0 && m % 256 == 0, "row0 and m must be multiples of 256");
  DSVGD_REQUIRE(((uintptr_t)Yg & 15) == 0 && ((uintptr_t)D & 15) == 0, "16-byte alignment");
  DSVGD_REQUIRE(dp * gram_img_rows(n) * 4 < ((int64_t)1 << 31),
                "image too large for 32-bit buffer offsets");
  DSVGD_REQUIRE(nparts > 0 && nparts <= 64, "1 .. 64 parts");
  for (int i = 0; i < nparts; ++i) {
    const dsvgd_gram_part& P = parts[i];
    DSVGD_REQUIRE(P.kind >= 0 && P.kind <= 2, "part kind must be 0, 1 or 2");
    DSVGD_REQUIRE(P.row_off >= 0 && P.rows > 0 && P.row_off + P.rows <= m &&
                      P.row_off % 128 == 0 && P.rows % 128 == 0,
                  "part rows must be a 128-aligned range of the owned block");
    DSVGD_REQUIRE(P.col0 >= 0 && P.cols > 0 && P.col0 + P.cols <= n_pad && P.col0 % 256 == 0 &&
                      P.cols % 256 == 0,
                  "part columns must be a 256-aligned range of [0, n_pad)");
    DSVGD_REQUIRE(P.kind != 1 || (P.row_off == 0 && P.rows == m && P.cols == m && P.col0 == row0),
                  "the diagonal part is the owned block's square");
    DSVGD_REQUIRE(P.kind != 2 || gate, "a fallback part needs the range-guard word");
  }
  const _Float16* yg = (const _Float16*)Yg;
  hipStream_t s = (hipStream_t)stream;
  if (select_mode == 0)
    return launch_sqdist_h2_parts<kSelNone>(yg, norms, row0, m, n, d, D, st, cand, parts, nparts,
                                            gate, s, rowscale);
  return launch_sqdist_h2_parts<kSelBracket>(yg, norms, row0, m, n, d, D, st, cand, parts, nparts,
                                             gate, s, rowscale);
}

}  // extern "C"
