// phi.hip -- the SVGD direction
//     phi_i = 1/n sum_j [ k_ij s_j + (2/h) k_ij (x_i - x_j) ],  k_ij = exp(-D_ij / h)
//           = 1/n [ (K S)_i + (2/h) (r_i x_i - (K X)_i) ],          r_i = sum_j k_ij
// (dsvgd/sampler.py:35-40, dsvgd/distsampler.py:84-101 with the RBF kernel of
// experiments/logreg.py:60-61 and its autograd gradient folded in closed form).
//
// phi_mm: K [Xc | S] on the NN MFMA engine with the exp fused into the A
// operand; D streams from HBM once (panel layout), [Xc|S] re-reads hit L2/MALL.
// Roofline: 2 * 128 * BC flop per 8 KiB D panel -> MFMA-bound for d >= 64.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <string>

#include "gemm_tiles.hpp"
#include "gemm_x3.hpp"
#include "phi_w1.hpp"

namespace dsvgd {

// every phi_w1_kernel launch
template <int DS, class... Args>
static void launch_w1(dim3 grid, hipStream_t s, Args... args) {
  hipLaunchKernelGGL((phi_w1_kernel<DS>), grid, dim3(PhiW1::kThreads), 0, s, args...);
}

// phi_mm on the FmtH2 engine (TN = 4): phi_w1_kernel (one wave per SIMD, B
// fragments straight from the image; phi_w1.hpp) -- on the full D layout (row
// blocks, S > 1) one launch; on the symmetric layout two, each row block
// split at its diagonal tile into the transposed K-steps (DS 1) and the plain
// ones (DS 2), with half the split-K slices each.

// blockIdx.z = split-K slice z: K columns [z*kchunk, min(K,(z+1)*kchunk)) into
// the partial C + z*m*ldc (and rowsum + z*m_pad); phi_finish sums the slices
// in order (deterministic, no atomics).
// row0: interacting-set index of A's row 0 (EXP: the diagonal j == row0 + i
// is skipped, see NNTile::store).
template <int TN, bool EXP, int WM, int TM, int BJ, bool SWZB = true>
__global__ __launch_bounds__(256 * WM) void nn_kernel(const float* __restrict__ A, int64_t a_npad,
                                                      const float* __restrict__ B, int64_t ldb,
                                                      int64_t K, int64_t kchunk,
                                                      const dsvgd_select_state* __restrict__ st,
                                                      float* __restrict__ C, int64_t ldc,
                                                      float* __restrict__ rowsum, int64_t m,
                                                      int64_t row0,
                                                      const float* __restrict__ gate) {
  // gate: run iff *gate != 0 (the FmtH2 range guard when no FmtX3 image fits)
  if (gate && *gate == 0.f) return;
  using Tile = NNTile<TN, EXP, WM, TM, BJ, SWZB>;
  __shared__ __attribute__((aligned(16))) float smem[Tile::kSmemFloats];
  const int64_t i0 = (int64_t)blockIdx.y * Tile::BM;
  const int64_t c0 = (int64_t)blockIdx.x * Tile::BC;
  const int64_t k0 = (int64_t)blockIdx.z * kchunk;
  const int64_t k1 = min(K, k0 + kchunk);
  C += (int64_t)blockIdx.z * m * ldc;
  if (rowsum) rowsum += (int64_t)blockIdx.z * roundup128(m);
  float scale = 0.f;
  if (EXP) scale = -st->inv_h * kLog2e;
  Tile tile;
  tile.run(A + (i0 >> 7) * (a_npad >> 4) * kPanelElems + (i0 & 127) * 16, B + c0, ldb, k0, k1,
           scale, smem, row0 + i0);

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wr = w >> 2, wc = w & 3;
  const int64_t r0 = i0 + wr * 32 * Tile::TM;
#pragma unroll
  for (int mi = 0; mi < Tile::TM; ++mi)
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
      const int64_t col = c0 + wc * 32 * TN + ni * 32 + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = r0 + mi * 32 + c_row(r, lane);
        if (row < m) C[row * ldc + col] = tile.acc[mi][ni][r];
      }
    }
  if (EXP && rowsum && blockIdx.x == 0) {
#pragma unroll
    for (int u = 0; u < Tile::RPT; ++u) {
      int p, rr, c4;
      Tile::a_map(threadIdx.x, u, p, rr, c4);
      const float v = tile.row_sum(u);
      const int64_t row = i0 + rr;
      if (c4 == 0 && row < m) rowsum[row] = v;
    }
  }
}

// phi_mm on the bf16 MFMA at fp32 accuracy (gemm_x3.hpp): the same blocks,
// split-K slices, diagonal skip and row sums as nn_kernel<TN, true>; B is the
// split image of Y (dsvgd_ysplit).
// F = FmtH2: C and rowsum come out of the MFMAs scaled by 2^15 (the A
// staging scale) and C's column c by the B image's column scale: the stores
// multiply by colinv[c] * 2^-15 (exact powers of two).
template <int TN, bool DMA, bool EXP, bool M16, int RW = 2, class F = FmtX3, int NB = 2>
__global__ __launch_bounds__(512) void nn_x3_kernel(const float* __restrict__ A, int64_t a_npad,
                                                    const typename F::E* __restrict__ Yx,
                                                    int64_t ldy, int64_t K, int64_t kchunk,
                                                    const dsvgd_select_state* __restrict__ st,
                                                    float* __restrict__ C, int64_t ldc,
                                                    float* __restrict__ rowsum, int64_t m,
                                                    int64_t row0, int sym,
                                                    const float* __restrict__ colinv,
                                                    int dsplit, int slice0,
                                                    const float* __restrict__ gate, int gate_on) {
  // gate (the FmtH2 range guard, dsvgd_h2_scales): run iff *gate != 0 equals gate_on
  if (gate && ((*gate != 0.f) != (gate_on != 0))) return;
  using Tile = NNX3Tile<TN, DMA, EXP, M16, RW, F, NB>;
  __shared__ __attribute__((aligned(16))) char smem[Tile::kSmemBytes];
  // dsplit (symmetric layout, 128-row blocks): 1 = only the K-steps left of
  // the block's diagonal tile (the transposed ones), longest rows first; the
  // z slices split that range and land in slices slice0 + z
  // (dispatch order: a row block's slices back to back, longest first)
  int64_t by = blockIdx.y, bz = blockIdx.z;
  if (dsplit == 1) {
    const int64_t lin = (int64_t)blockIdx.z * gridDim.y + blockIdx.y;
    by = gridDim.y - 1 - lin / gridDim.z;
    bz = lin % gridDim.z;
  }
  const int64_t i0 = by * Tile::BM;
  const int64_t c0 = (int64_t)blockIdx.x * Tile::BC;
  int64_t k0 = bz * kchunk, k1 = min(K, k0 + kchunk);
  Tile tile;
  if (dsplit == 1) {
    // slice z: K-steps z, z + Z, ... left of the diagonal tile, so the blocks
    // running together read the same Yx K-steps (L2 reuse)
    k0 = bz * kX3Step;
    k1 = i0;
    tile.kst = (int64_t)gridDim.z * kX3Step;
  }
  C += (int64_t)(slice0 + bz) * m * ldc;
  if (EXP) rowsum += (int64_t)(slice0 + bz) * roundup128(m);
  const float scale = EXP ? -st->inv_h * kLog2e : 0.f;
  tile.prow = (a_npad >> 4) * kPanelElems * 4;
  if (DMA && sym) {  // symmetric layout: m == n, row0 == 0 (checked by the ABI)
    tile.sym_D = A;
    tile.sym_pcols = a_npad >> 4;
    tile.sym_I = i0 >> 7;
  }
  tile.run(A + (i0 >> 7) * (a_npad >> 4) * kPanelElems, Yx + c0 * 16, ldy, k0, k1, scale, smem,
           row0 + i0);

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wr = w / Tile::kCW,
            wc = w % Tile::kCW;
  const int64_t r0 = i0 + wr * 32 * Tile::TM;
  if (M16) {  // 16x16 C layout: column lane & 15, rows 4 (lane >> 4) + reg
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 2 * TN; ++nt) {
        const int64_t col = c0 + wc * 32 * TN + nt * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t row = r0 + mt * 16 + 4 * (lane >> 4) + r;
          if (row < m) C[row * ldc + col] = tile.acc16[mt][nt][r];
        }
      }
  } else {
#pragma unroll
    for (int mi = 0; mi < Tile::TM; ++mi)
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const int64_t col = c0 + wc * 32 * TN + ni * 32 + (lane & 31);
        const float cs = F::P == 3 ? 1.f : colinv[col] * (1.f / F::kAScale);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int64_t row = r0 + mi * 32 + c_row(r, lane);
          if (row < m) C[row * ldc + col] = F::P == 3 ? tile.acc[mi][ni][r] : tile.acc[mi][ni][r] * cs;
        }
      }
  }
  if (EXP && blockIdx.x == 0) {
    const float v = tile.row_sum() * (1.f / F::kAScale);
    const int64_t row = i0 + (threadIdx.x >> 2);
    if ((threadIdx.x & 3) == 0 && row < m) rowsum[row] = v;
  }
}

// img[kstep][part][row][16 k] (bf16) = the three parts of A[row][16 kstep + k]
// for row < rows_pad, 16 kstep + k < kpad (zero outside rows x cols); halves
// swapped on rows with bit 3 set (NTX3Tile's image).
__global__ __launch_bounds__(256) void rowsplit_kernel(const float* __restrict__ A, int64_t lda,
                                                       int64_t rows, int64_t cols,
                                                       int64_t rows_pad, int64_t ksteps,
                                                       __bf16* __restrict__ img, int swz) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= ksteps * rows_pad) return;
  const int64_t kb = t / rows_pad, i = t % rows_pad;
  bf16x8 s[kX3Parts][2];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int64_t c = kb * 16 + k;
    const Split3 v = split3((i < rows && c < cols) ? A[i * lda + c] : 0.f);
    s[0][k >> 3][k & 7] = v.s0;
    s[1][k >> 3][k & 7] = v.s1;
    s[2][k >> 3][k & 7] = v.s2;
  }
  const int sw = swz ? (int)((i >> 3) & 1) : 0;
#pragma unroll
  for (int p = 0; p < kX3Parts; ++p) {
    __bf16* dst = img + ((kb * kX3Parts + p) * rows_pad + i) * 16;
    *reinterpret_cast<bf16x8*>(dst + 8 * sw) = s[p][0];
    *reinterpret_cast<bf16x8*>(dst + 8 * (sw ^ 1)) = s[p][1];
  }
}

// Yx[kstep][part][column][16 k] = the three bf16 parts of Y[16 kstep + k][column]
// (gemm_x3.hpp image: 16-B halves swapped on columns with bit 3 set).
__global__ __launch_bounds__(256) void ysplit_kernel(const float* __restrict__ Y, int64_t ldy,
                                                     int64_t ksteps, __bf16* __restrict__ Yx,
                                                     int swz, const float* __restrict__ gate) {
  if (gate && *gate == 0.f) return;  // the FmtH2 range guard's fallback image only
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= ksteps * ldy) return;
  const int64_t kb = t / ldy, c = t % ldy;
  bf16x8 s[kX3Parts][2];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const Split3 v = split3(Y[(kb * 16 + k) * ldy + c]);
    s[0][k >> 3][k & 7] = v.s0;
    s[1][k >> 3][k & 7] = v.s1;
    s[2][k >> 3][k & 7] = v.s2;
  }
  const int sw = swz ? (int)((c >> 3) & 1) : 0;
#pragma unroll
  for (int p = 0; p < kX3Parts; ++p) {
    __bf16* dst = Yx + ((kb * kX3Parts + p) * ldy + c) * 16;
    *reinterpret_cast<bf16x8*>(dst + 8 * sw) = s[p][0];
    *reinterpret_cast<bf16x8*>(dst + 8 * (sw ^ 1)) = s[p][1];
  }
}

// the symmetric layout's phi_mm: 1 = one launch per row (DS 4), 0 = the
// two-launch hybrid (DS 1 + DS 2); dsvgd_phi_set_symrow
static int g_phi_symrow = 1;
// at most this many columns per fp32 split-K accumulation chain (phi_splits)
constexpr int64_t kMaxChain = 16384;
// logreg's G . Xd (FmtH2, 256 columns) on phi_w1_kernel<0, 2, false> (1) or
// the 8-wave 256-row NN tile (0, default: the phi_w1 shape measured slower,
// scores 3.57 vs 3.38 ms at N = 16384, 0.58 vs 0.52 at 2048 -- with half
// phi_mm's MFMAs per K-step its staging is no longer hidden; profiles/r13r);
// dsvgd_phi_set_gxd_w1
static int g_gxd_w1 = 0;
// split-K slices mapped to XCDs when the grid allows it (phi_w1.hpp xmap),
// a bit mask: 1 DS 4 (default), 2 DS 0 (full layout, window), 4 the batched
// DS 3 (forward partials); dsvgd_phi_set_xmap.  DS 4 without it: 11.44 vs
// 11.09 ms at S = 1; the S = 8 window with it: 3.03 / 3.13 vs 3.01 / 3.02 ms
// (profiles/r13o)
static int g_phi_xmap = 1;
static int xmap_ok(dim3 g, int bit) {
  // one column block only: at d = 1024 (four) the map measured 45.4 vs 44.4
  // ms without it (profiles/r13q) -- there the blocks of a row sharing an
  // XCD's L2 for their D panels is what counts
  return (g_phi_xmap & bit) && g.x == 1 && g.z > 1 && 8 % g.z == 0 &&
         ((int64_t)g.y * g.z) % 8 == 0;
}

template <int TN, bool EXP, class F>
int launch_nn_x3(const float* D, int64_t K, const typename F::E* Yx, int64_t ldy, int splits,
                 const dsvgd_select_state* st, float* C, int64_t ldc, float* rowsum, int64_t m,
                 int64_t row0, int sym, int m16, const float* colinv, hipStream_t s,
                 const float* gate, int gate_on) {
  if (sym && TN == 1) return fail_arg("nn_x3: the symmetric layout needs ldy % 256 == 0");
  const int64_t kchunk = roundup((K + splits - 1) / splits, kX3Step);
  const dim3 grid(ldy / (128 * TN), roundup(m, 128) / 128, splits);
  if (F::P == 3 && m16 && TN == 1)
    return fail_arg("nn_x3: the 16x16 form needs the DMA path (ldy % 256 == 0)");
  if (TN == 1)  // TN = 1: 1.5 DMA rounds per K-step -> the register-staged form
    hipLaunchKernelGGL((nn_x3_kernel<TN, false, EXP, false, 2, F>), grid, dim3(512), 0, s, D, K, Yx,
                       ldy, K, kchunk, st, C, ldc, rowsum, m, row0, 0, colinv, 0, 0, gate, gate_on);
  else if constexpr (F::P == 3) {
    if (m16)
      hipLaunchKernelGGL((nn_x3_kernel<TN, TN != 1, EXP, TN != 1, 2, F>), grid, dim3(512), 0, s, D,
                         K, Yx, ldy, K, kchunk, st, C, ldc, rowsum, m, row0, sym, colinv, 0, 0, gate, gate_on);
    else
      hipLaunchKernelGGL((nn_x3_kernel<TN, TN != 1, EXP, false, 2, F>), grid, dim3(512), 0, s, D, K,
                         Yx, ldy, K, kchunk, st, C, ldc, rowsum, m, row0, sym, colinv, 0, 0, gate, gate_on);
  } else {  // FmtH2: the smaller stages fit a 3-stage ring
    if (TN == 4 && EXP && sym && splits >= 2 && g_phi_symrow) {
      // symmetric layout, each row's slices in ONE launch (phi_w1 DS 4):
      // contiguous K ranges walked ascending, transposed K-steps first; the
      // blocks of an XCD share a slice (xmap: 8 | row blocks x slices)
      const bool xmap = xmap_ok(grid, 1);
      launch_w1<4>(grid, s, D, K, Yx, ldy, K, kchunk, st, C, ldc, rowsum, m, row0, sym, colinv, 0,
                   gate, gate_on, 0, 0, 0, xmap ? 1 : 0);
      return check_launch("phi_w1_kernel(rows)");
    }
    if (TN == 4 && EXP && sym && splits >= 2) {
      // symmetric layout split at each row block's diagonal tile: the
      // transposed K-steps (phi_w1 DS 1: the stored tiles transposed through
      // a per-wave LDS scratch) and the plain ones (DS 2); half the split-K
      // slices each
      const int sl = splits / 2;
      // a slice of either launch spans up to K / sl columns: refuse slices
      // sized for the one-launch form (symrow switched after the engine took
      // dsvgd_phi_splits_sym) rather than run chains past 2 kMaxChain
      if (K > 2 * kMaxChain * (int64_t)sl)
        return fail_arg("phi_mm: the hybrid's split-K chains would exceed 2 x 16384 columns; "
                        "size the slices with dsvgd_phi_splits_sym under the current symrow form");
      const dim3 g1(grid.x, grid.y, sl), g2(grid.x, grid.y, splits - sl);
      launch_w1<1>(g1, s, D, K, Yx, ldy, K, kchunk, st, C, ldc, rowsum, m, row0, sym, colinv, 0,
                   gate, gate_on);
      const int rc = check_launch("phi_w1_kernel(lower)");
      if (rc) return rc;
      launch_w1<2>(g2, s, D, K, Yx, ldy, K, kchunk, st, C, ldc, rowsum, m, row0, sym, colinv, sl,
                   gate, gate_on);
      return check_launch("phi_w1_kernel(upper)");
    }
    if (TN == 4 && EXP && !sym) {
      launch_w1<0>(grid, s, D, K, Yx, ldy, K, kchunk, st, C, ldc, rowsum, m, row0, sym, colinv, 0,
                   gate, gate_on, 0, 0, 0, xmap_ok(grid, 2));
      return check_launch("phi_w1_kernel");
    }
    hipLaunchKernelGGL((nn_x3_kernel<TN, TN != 1, EXP, false, 2, F, TN != 1 ? 3 : 2>), grid,
                       dim3(512), 0, s, D, K, Yx, ldy, K, kchunk, st, C, ldc, rowsum, m, row0, sym,
                       colinv, 0, 0, gate, gate_on);
  }
  return check_launch("nn_x3_kernel");
}

// C = f(A) B on the split engine; A panel layout (m_pad x K), B = Yx image
// (K rows, ldy columns, a multiple of 128).  exp_: the phi_mm form.
template <class F>
int nn_split_gemm(bool exp_, const float* A, int64_t K, const typename F::E* Yx, int64_t ldy,
                  int splits, const dsvgd_select_state* st, float* C, int64_t ldc, float* rowsum,
                  int64_t m, int64_t row0, hipStream_t s, int sym, int m16, const float* colinv,
                  const float* gate = nullptr, int gate_on = 0) {
  if (F::P == 2) m16 = 0;  // the fp16 format runs the 32x32x16 form
  // buffer offsets are 32-bit: K rows x ldy columns x P parts x 2 bytes of
  // the image (as dsvgd_phi_mm_{h2,x3} check), K x 128 x 4 bytes of D
  if (K * ldy * 2 * F::P >= ((int64_t)1 << 31) || K * 128 * 4 >= ((int64_t)1 << 31))
    return fail_arg("nn_x3: K x ldy too large for 32-bit buffer offsets");
  if (ldy % 128 != 0) return fail_arg("nn_x3: ldy must be a multiple of 128");
  if constexpr (F::P == 2) {
    if (!exp_ && ldy % 512 != 0 && ldy % 256 == 0 && g_gxd_w1) {
      // G . Xd on phi_w1's shape: 128-row x 256-column blocks of four waves
      // of 64 columns, B straight from the image, two blocks per CU
      const int64_t kchunk = roundup((K + splits - 1) / splits, kX3Step);
      const dim3 grid(ldy / 256, roundup(m, 128) / 128, splits);
      hipLaunchKernelGGL((phi_w1_kernel<0, 2, false>), grid, dim3(PhiW1::kThreads), 0, s, A, K, Yx,
                         ldy, K, kchunk, st, C, ldc, rowsum, m, row0, 0, colinv, 0, gate, gate_on);
      return check_launch("phi_w1_kernel(G.Xd)");
    }
  }
  if (!exp_ && (m16 || F::P == 2) && ldy % 512 != 0 && ldy % 256 == 0) {
    // 256-row blocks x 256 columns (G . Xd): the A rows must exist up to a
    // multiple of 256 (the caller's panel layout; logreg pads n to 256)
    const int64_t kchunk = roundup((K + splits - 1) / splits, kX3Step);
    const dim3 grid(ldy / 256, roundup(m, 256) / 256, splits);
    hipLaunchKernelGGL((nn_x3_kernel<4, true, false, F::P == 3, 4, F, F::P == 3 ? 2 : 3>), grid,
                       dim3(512), 0, s, A, K, Yx, ldy, K, kchunk, st, C, ldc, rowsum, m, row0, 0,
                       colinv, 0, 0, gate, gate_on);
    return check_launch("nn_x3_kernel(256-row)");
  }
#define DSVGD_X3_TN(TN)                                                                        \
  return exp_ ? launch_nn_x3<TN, true, F>(A, K, Yx, ldy, splits, st, C, ldc, rowsum, m, row0,    \
                                          sym, m16, colinv, s, gate, gate_on)                  \
              : launch_nn_x3<TN, false, F>(A, K, Yx, ldy, splits, st, C, ldc, rowsum, m, row0, 0, \
                                           m16, colinv, s, gate, gate_on)
  if (ldy % 512 == 0) DSVGD_X3_TN(4);
  if (ldy % 256 == 0) DSVGD_X3_TN(2);
  DSVGD_X3_TN(1);
#undef DSVGD_X3_TN
}

int nn_x3_gemm(bool exp_, const float* A, int64_t K, const __bf16* Yx, int64_t ldy, int splits,
               const dsvgd_select_state* st, float* C, int64_t ldc, float* rowsum, int64_t m,
               int64_t row0, hipStream_t s, int sym, int m16, const float* gate) {
  return nn_split_gemm<FmtX3>(exp_, A, K, Yx, ldy, splits, st, C, ldc, rowsum, m, row0, s, sym,
                              m16, nullptr, gate, 1);
}

int nn_h2_gemm(bool exp_, const float* A, int64_t K, const _Float16* Yh, int64_t ldy, int splits,
               const dsvgd_select_state* st, float* C, int64_t ldc, float* rowsum, int64_t m,
               int64_t row0, hipStream_t s, int sym, const float* colinv, const float* gate) {
  return nn_split_gemm<FmtH2>(exp_, A, K, Yh, ldy, splits, st, C, ldc, rowsum, m, row0, s, sym, 0,
                              colinv, gate, 0);
}


// phi[i][c] = inv_n (KS[i][c] + (2/h)(r_i xc[i][c] - KX[i][c])) [+ extra[i][c]];
// X[i][c] += step phi.  KY / rowsum hold `splits` split-K partials, summed
// here in slice order.  extra (nullable): the h * W2-gradient rows, added to
// phi before the step as in distsampler.py:196-200.
__global__ __launch_bounds__(256) void phi_finish_kernel(
    const float* __restrict__ KY, int64_t ldk, const float* __restrict__ rowsum, int splits,
    const float* __restrict__ Y, int64_t ldy, int64_t row0, int64_t m, int64_t d, int64_t dp,
    const dsvgd_select_state* __restrict__ st, float inv_n, float step,
    const float* __restrict__ extra, int64_t lde, float* __restrict__ phi, int64_t ldphi,
    float* __restrict__ X, int64_t ldx) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= m * d) return;
  const int64_t i = t / d, c = t % d;
  const float two_inv_h = 2.f * st->inv_h;
  const int64_t mp = roundup128(m);
  float kx = 0.f, ks = 0.f, r = 0.f;
  for (int z = 0; z < splits; ++z) {
    const float* ky = KY + (int64_t)z * m * ldk + i * ldk;
    kx += ky[c];
    ks += ky[dp + c];
    r += rowsum[(int64_t)z * mp + i];
  }
  const float* yi = Y + (row0 + i) * ldy;
  // + the self term k_ii (s_i + 2/h (x_i - x_i)) = s_i, excluded from phi_mm
  float p = inv_n * ((yi[dp + c] + ks) + two_inv_h * (r * yi[c] - kx));
  if (extra) p += extra[i * lde + c];
  if (phi) phi[i * ldphi + c] = p;
  if (X) X[i * ldx + c] += step * p;
}

// phi_finish_kernel with four consecutive columns per thread (16-byte loads
// and stores; every stride and base 16-byte aligned, d % 4 == 0): the same
// per-element arithmetic in the same order, so the same bits.
__global__ __launch_bounds__(256) void phi_finish4_kernel(
    const float* __restrict__ KY, int64_t ldk, const float* __restrict__ rowsum, int splits,
    const float* __restrict__ Y, int64_t ldy, int64_t row0, int64_t m, int64_t d4, int64_t dp,
    const dsvgd_select_state* __restrict__ st, float inv_n, float step,
    const float* __restrict__ extra, int64_t lde, float* __restrict__ phi, int64_t ldphi,
    float* __restrict__ X, int64_t ldx) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= m * d4) return;
  const int64_t i = t / d4, c = (t % d4) * 4;
  const float two_inv_h = 2.f * st->inv_h;
  const int64_t mp = roundup128(m);
  f32x4 kx = {0.f, 0.f, 0.f, 0.f}, ks = {0.f, 0.f, 0.f, 0.f};
  float r = 0.f;
  for (int z = 0; z < splits; ++z) {
    const float* ky = KY + (int64_t)z * m * ldk + i * ldk;
    kx += *reinterpret_cast<const f32x4*>(ky + c);
    ks += *reinterpret_cast<const f32x4*>(ky + dp + c);
    r += rowsum[(int64_t)z * mp + i];
  }
  const float* yi = Y + (row0 + i) * ldy;
  const f32x4 yx = *reinterpret_cast<const f32x4*>(yi + c);
  const f32x4 ys = *reinterpret_cast<const f32x4*>(yi + dp + c);
  const f32x4 ex = extra ? *reinterpret_cast<const f32x4*>(extra + i * lde + c)
                         : f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 p;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    // + the self term k_ii (s_i + 2/h (x_i - x_i)) = s_i, excluded from phi_mm
    float q = inv_n * ((ys[e] + ks[e]) + two_inv_h * (r * yx[e] - kx[e]));
    if (extra) q += ex[e];
    p[e] = q;
  }
  if (phi) *reinterpret_cast<f32x4*>(phi + i * ldphi + c) = p;
  if (X) {
    f32x4 x = *reinterpret_cast<const f32x4*>(X + i * ldx + c);
#pragma unroll
    for (int e = 0; e < 4; ++e) x[e] += step * p[e];
    *reinterpret_cast<f32x4*>(X + i * ldx + c) = x;
  }
}

// ---- split-K partials summed (dsvgd_phi_h2_transposed, the wide sweep) ---
// out[i][c] = sum_z P[z][i][c], out_rs[i] = sum_z rs[z][i] in a fixed order:
// a workgroup takes 256 / G float4 positions; its G thread groups (G = the
// slice count rounded up to a power of two, at most 16) sum the slices z =
// g, g + G, ... (independent loads in flight), then the G group sums are
// added in g order.  (One thread per position walking all the slices was
// latency-bound: 122 us for 256 slices of 64 x 512, r11d.)
// Slice z at P + z zs, its row sums at rs + z zrs; blockIdx.y = part: the
// inputs ps_in, the outputs ps_out floats after the previous part's.
__global__ __launch_bounds__(256) void partial_reduce_kernel(
    const float* __restrict__ P, int64_t ldp, const float* __restrict__ rs, int splits,
    int64_t rows, int64_t cols, float* __restrict__ out, int64_t ldo, float* __restrict__ out_rs,
    int G, int64_t zs, int64_t zrs, int64_t ps_in, int64_t ps_out) {
  __shared__ f32x4 red[256];
  const int per = 256 / G;
  const int q = threadIdx.x % per, g = threadIdx.x / per;
  const int64_t c4 = cols >> 2;
  P += blockIdx.y * ps_in;
  rs += blockIdx.y * ps_in;
  out += blockIdx.y * ps_out;
  out_rs += blockIdx.y * ps_out;
  const int64_t npos = rows * c4, nrs = (rows + 3) >> 2;
  const int64_t p = (int64_t)blockIdx.x * per + q;
  f32x4 a = {0.f, 0.f, 0.f, 0.f};
  if (p < npos) {
    const int64_t i = p / c4, c = (p % c4) * 4;
    for (int z = g; z < splits; z += G)
      a += *reinterpret_cast<const f32x4*>(P + (int64_t)z * zs + i * ldp + c);
  } else if (p < npos + nrs) {
    const int64_t i0 = (p - npos) * 4;
    for (int z = g; z < splits; z += G)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (i0 + e < rows) a[e] += rs[(int64_t)z * zrs + i0 + e];
  }
  red[g * per + q] = a;
  __syncthreads();
  if (g == 0) {
    f32x4 sum = red[q];
    for (int k = 1; k < G; ++k) sum += red[k * per + q];
    if (p < npos) {
      const int64_t i = p / c4, c = (p % c4) * 4;
      *reinterpret_cast<f32x4*>(out + i * ldo + c) = sum;
    } else if (p < npos + nrs) {
      const int64_t i0 = (p - npos) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (i0 + e < rows) out_rs[i0 + e] = sum[e];
    }
  }
}

// phi_finish over the own slices plus the partials of the pair-split layout
// (list order after the own slices: deterministic); gate != 0: the range
// guard's whole-row fallback wrote splits_fb own slices, the parts are skipped
constexpr int kMaxPhiParts = 16;
struct PhiPartsArg {
  int n;
  const float* ky[kMaxPhiParts];
  const float* rs[kMaxPhiParts];
  int64_t ldk[kMaxPhiParts], row_off[kMaxPhiParts], rows[kMaxPhiParts];
  int splits[kMaxPhiParts];
};

__global__ __launch_bounds__(256) void phi_finish_parts_kernel(
    const float* __restrict__ KY, int64_t ldk, const float* __restrict__ rowsum, int splits,
    const float* __restrict__ Y, int64_t ldy, int64_t row0, int64_t m, int64_t d, int64_t dp,
    const dsvgd_select_state* __restrict__ st, float inv_n, float step,
    const float* __restrict__ extra, int64_t lde, float* __restrict__ phi, int64_t ldphi,
    float* __restrict__ X, int64_t ldx, PhiPartsArg parts, const float* __restrict__ gate,
    int splits_fb) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= m * d) return;
  const int64_t i = t / d, c = t % d;
  const bool fb = gate && *gate != 0.f;
  const int ns = fb ? splits_fb : splits;
  const float two_inv_h = 2.f * st->inv_h;
  const int64_t mp = roundup128(m);
  float kx = 0.f, ks = 0.f, r = 0.f;
  for (int z = 0; z < ns; ++z) {
    const float* ky = KY + (int64_t)z * m * ldk + i * ldk;
    kx += ky[c];
    ks += ky[dp + c];
    r += rowsum[(int64_t)z * mp + i];
  }
  const int np = fb ? 0 : parts.n;
  for (int p = 0; p < np; ++p) {
    const int64_t li = i - parts.row_off[p];
    if (li < 0 || li >= parts.rows[p]) continue;
    const int64_t rows = parts.rows[p], lk = parts.ldk[p];
    for (int z = 0; z < parts.splits[p]; ++z) {
      const float* ky = parts.ky[p] + ((int64_t)z * rows + li) * lk;
      kx += ky[c];
      ks += ky[dp + c];
      r += parts.rs[p][(int64_t)z * roundup128(rows) + li];
    }
  }
  const float* yi = Y + (row0 + i) * ldy;
  float p = inv_n * ((yi[dp + c] + ks) + two_inv_h * (r * yi[c] - kx));
  if (extra) p += extra[i * lde + c];
  if (phi) phi[i * ldphi + c] = p;
  if (X) X[i * ldx + c] += step * p;
}

// d <= 64: phi from explicit differences, the reference's own pairwise form
//   phi_i = inv_n sum_j k_ij (s_j + (2/h)(x_i - x_j))
// (no r_i x_i - (K X)_i cancellation, which at small d and a narrow bandwidth
// exceeds the 1e-5 tolerance).  Block: 64 rows x 64 columns; thread (rq, cq)
// owns rows 4rq..+3 x columns 4cq..+3; j streams in chunks of 64 through LDS
// (K chunk transposed [j][i], x_j and s_j [j][c]).  VALU: 3 ops per (i,j,c).
constexpr int kPhiDirectMaxD = 64;

__global__ __launch_bounds__(256) void phi_direct_kernel(
    const float* __restrict__ D, int64_t n_pad, const float* __restrict__ Y, int64_t ldy,
    int64_t row0, int64_t m, int64_t n, int d, int64_t dp,
    const dsvgd_select_state* __restrict__ st, float inv_n, float step,
    const float* __restrict__ extra, int64_t lde, float* __restrict__ phi, int64_t ldphi,
    float* __restrict__ X, int64_t ldx, int64_t jchunk, float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float kT[64][64];
  __shared__ __attribute__((aligned(16))) float xs[64][64];
  __shared__ __attribute__((aligned(16))) float ss[64][64];
  const int t = threadIdx.x, rq = t >> 4, cq = t & 15;
  const int64_t i0 = (int64_t)blockIdx.x * 64;
  const float inv_h = st->inv_h;
  const float scale = -inv_h * kLog2e, g = 2.f * inv_h;
  float xi[4][4], acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int64_t i = i0 + 4 * rq + a;
      const int col = 4 * cq + c;
      xi[a][c] = (i < m && col < d) ? Y[(row0 + i) * ldy + col] : 0.f;
      acc[a][c] = 0.f;
    }
  // the j sum runs in chains of kChain columns added into `tot` (one long
  // fp32 chain over n ~ 16k terms costs ~5e-6 of max|phi|)
  constexpr int64_t kChain = 4096;
  float tot[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) tot[a][c] = 0.f;
  // blockIdx.y: split-J slice [jb, je) (part != null: write the raw sums)
  const int64_t jb = (int64_t)blockIdx.y * jchunk, je = min(n, jb + jchunk);
  for (int64_t j0 = jb; j0 < je; j0 += 64) {
    if ((j0 - jb) % kChain == 0 && j0 > jb) {
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          tot[a][c] += acc[a][c];
          acc[a][c] = 0.f;
        }
    }
    for (int e = t; e < 64 * 64; e += 256) {
      const int r = e >> 6, q = e & 63;  // kT[q][r]: row i0+r, column j0+q
      const int64_t i = i0 + r, j = j0 + q;
      kT[q][r] = (i < m && j < je) ? __builtin_amdgcn_exp2f(D[panel_off(i, j, n_pad)] * scale) : 0.f;
      const int64_t jr = j0 + r;
      xs[r][q] = (jr < je && q < d) ? Y[jr * ldy + q] : 0.f;
      ss[r][q] = (jr < je && q < d) ? Y[jr * ldy + dp + q] : 0.f;
    }
    __syncthreads();
    const int jn = (int)min((int64_t)64, je - j0);
    for (int q = 0; q < jn; ++q) {
      const f32x4 k4 = *reinterpret_cast<const f32x4*>(&kT[q][4 * rq]);
      const f32x4 x4 = *reinterpret_cast<const f32x4*>(&xs[q][4 * cq]);
      const f32x4 s4 = *reinterpret_cast<const f32x4*>(&ss[q][4 * cq]);
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[a][c] = fmaf(k4[a], fmaf(g, xi[a][c] - x4[c], s4[c]), acc[a][c]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[a][c] += tot[a][c];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int64_t i = i0 + 4 * rq + a;
      const int col = 4 * cq + c;
      if (i < m && col < d) {
        if (part) {
          part[((int64_t)blockIdx.y * m + i) * d + col] = acc[a][c];
          continue;
        }
        float p = inv_n * acc[a][c];
        if (extra) p += extra[i * lde + col];
        if (phi) phi[i * ldphi + col] = p;
        if (X) X[i * ldx + col] += step * p;
      }
    }
}

// split-J partial sums of phi_direct_kernel, added in slice order
__global__ __launch_bounds__(256) void phi_direct_finish_kernel(
    const float* __restrict__ part, int nsplit, int64_t m, int64_t d, float inv_n, float step,
    const float* __restrict__ extra, int64_t lde, float* __restrict__ phi, int64_t ldphi,
    float* __restrict__ X, int64_t ldx) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= m * d) return;
  const int64_t i = e / d, col = e % d;
  float a = 0.f;
  for (int z = 0; z < nsplit; ++z) a += part[(int64_t)z * m * d + e];
  float p = inv_n * a;
  if (extra) p += extra[i * lde + col];
  if (phi) phi[i * ldphi + col] = p;
  if (X) X[i * ldx + col] += step * p;
}

// red[g * dc + c] for g < G groups -> red[c] (c < dc): pairwise halving in
// a fixed order (deterministic; a serial walk over 256 groups on one thread
// cost ~8 us per chunk at d = 1).  Called by all 256 threads.
__device__ __forceinline__ void group_reduce(float* red, int dc, int G) {
  const int t = threadIdx.x;
  while (G > 1) {
    const int h = (G + 1) >> 1;
    if (t < (G - h) * dc) red[t] += red[t + h * dc];
    __syncthreads();
    G = h;
  }
}

// Gauss-Seidel row update (reference order, exact differences, no Gram):
// one block; j in chunks of 256 (one per thread) -> k_j in LDS; then the
// (column, j) sums are split over the block: for a column block of dc <= 256
// columns, G = 256/dc thread groups each take every G-th j, and the G
// partials per column are added in group order (deterministic).  At the
// reference's small d (1-3) that keeps the whole block busy instead of d
// threads walking every j.
__global__ __launch_bounds__(256) void phi_row_kernel(float* __restrict__ X, int64_t ldx,
                                                      const float* __restrict__ S, int64_t lds,
                                                      int64_t n, int64_t d, int64_t i,
                                                      const dsvgd_select_state* __restrict__ st,
                                                      float step,
                                                      const float* __restrict__ extra,
                                                      float* __restrict__ phi_out) {
  extern __shared__ __attribute__((aligned(16))) float dyn[];
  float* xi = dyn;            // d
  float* acc = dyn + d;       // d
  float* kb = dyn + 2 * d;    // 256
  float* red = kb + 256;      // 256
  const int t = threadIdx.x;
  const float inv_h = st->inv_h;
  const float g2 = 2.f * inv_h;
  for (int64_t c = t; c < d; c += 256) {
    xi[c] = X[i * ldx + c];
    acc[c] = 0.f;
  }
  __syncthreads();
  for (int64_t j0 = 0; j0 < n; j0 += 256) {
    const int64_t j = j0 + t;
    float k = 0.f;
    if (j < n) {
      float s2 = 0.f;
      for (int64_t c = 0; c < d; ++c) {
        const float df = X[j * ldx + c] - xi[c];
        s2 = fmaf(df, df, s2);
      }
      k = expf(-s2 * inv_h);
    }
    kb[t] = k;
    __syncthreads();
    const int nj = (int)min((int64_t)256, n - j0);
    for (int64_t c0 = 0; c0 < d; c0 += 256) {
      const int dc = (int)min((int64_t)256, d - c0);
      const int G = 256 / dc;
      float part = 0.f;
      if (t < dc * G) {
        const int64_t c = c0 + t % dc;
        const float x = xi[c];
        for (int q = t / dc; q < nj; q += G) {
          const int64_t jj = j0 + q;
          part = fmaf(kb[q], fmaf(g2, x - X[jj * ldx + c], S[jj * lds + c]), part);
        }
      }
      red[t] = part;
      __syncthreads();
      group_reduce(red, dc, G);
      if (t < dc) acc[c0 + t] += red[t];
      __syncthreads();
    }
  }
  const float inv_n = 1.f / (float)n;
  for (int64_t c = t; c < d; c += 256) {
    float p = inv_n * acc[c];
    if (extra) p += extra[c];
    if (phi_out) phi_out[c] = p;
    X[i * ldx + c] = xi[c] + step * p;
  }
}

// Gauss-Seidel row update at scale (n in the thousands and up): the j range
// is split over `blocks` workgroups -- one workgroup walking all n rows with
// per-thread row loops was ~1.2 ms per particle at n = 16384, d = 64.
// Workgroup b takes rows [b J, (b+1) J): phase 1 puts k_j of its rows in LDS
// (16 lanes per row, 16-byte loads, x_i from LDS), phase 2 sums
// k_j (s_j + (2/h)(x_i - x_j)) over them per column (column-coalesced reads,
// the phi_row_kernel column/group split) into partial[b][c].
// phi_row_finish_kernel adds the partials in block order (deterministic) and
// moves x_i.  VEC: ldx % 4 == 0 and a 16-byte aligned X.
template <bool VEC>
__global__ __launch_bounds__(256) void phi_row_part_kernel(const float* __restrict__ X,
                                                           int64_t ldx,
                                                           const float* __restrict__ S,
                                                           int64_t lds, int64_t n, int64_t d,
                                                           int64_t i, int64_t J,
                                                           const dsvgd_select_state* __restrict__ st,
                                                           float* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) float dyn[];
  float* xi = dyn;         // roundup(d, 4)
  float* red = dyn + ((d + 3) & ~(int64_t)3);  // 256
  float* kb = red + 256;   // J
  const int t = threadIdx.x;
  const float inv_h = st->inv_h;
  const float g2 = 2.f * inv_h;
  const int64_t j0 = (int64_t)blockIdx.x * J, j1 = min(n, j0 + J);
  for (int64_t c = t; c < ((d + 3) & ~(int64_t)3); c += 256) xi[c] = c < d ? X[i * ldx + c] : 0.f;
  __syncthreads();
  if (VEC) {
    const int l16 = t & 15;
    for (int64_t jb = j0; jb < j1; jb += 16) {  // block-uniform trip count
      const int64_t j = jb + (t >> 4);
      float s2 = 0.f;
      if (j < j1) {
        const float* xj = X + j * ldx;
        for (int64_t c = 4 * l16; c < d; c += 64) {
          const f32x4 a = *reinterpret_cast<const f32x4*>(xj + c);
          const f32x4 b = *reinterpret_cast<const f32x4*>(xi + c);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float df = c + e < d ? a[e] - b[e] : 0.f;
            s2 = fmaf(df, df, s2);
          }
        }
      }
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) s2 += __shfl_xor(s2, o, 64);
      if (j < j1 && l16 == 0) kb[j - j0] = expf(-s2 * inv_h);
    }
  } else {
    for (int64_t j = j0 + t; j < j1; j += 256) {
      float s2 = 0.f;
      for (int64_t c = 0; c < d; ++c) {
        const float df = X[j * ldx + c] - xi[c];
        s2 = fmaf(df, df, s2);
      }
      kb[j - j0] = expf(-s2 * inv_h);
    }
  }
  __syncthreads();
  const int nj = (int)(j1 - j0);
  for (int64_t c0 = 0; c0 < d; c0 += 256) {
    const int dc = (int)min((int64_t)256, d - c0);
    const int G = 256 / dc;
    float part = 0.f;
    if (t < dc * G) {
      const int64_t c = c0 + t % dc;
      const float x = xi[c];
      for (int q = t / dc; q < nj; q += G) {
        const int64_t jj = j0 + q;
        part = fmaf(kb[q], fmaf(g2, x - X[jj * ldx + c], S[jj * lds + c]), part);
      }
    }
    red[t] = part;
    __syncthreads();
    group_reduce(red, dc, G);
    if (t < dc) partial[(int64_t)blockIdx.x * d + c0 + t] = red[t];
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void phi_row_finish_kernel(float* __restrict__ X, int64_t ldx,
                                                             int64_t n, int64_t d, int64_t i,
                                                             const float* __restrict__ partial,
                                                             int64_t blocks, float step,
                                                             const float* __restrict__ extra,
                                                             float* __restrict__ phi_out) {
  // columns in chunks of dc <= 256; G = 256 / dc thread groups take every
  // G-th block's partial (loads in flight together, not one chained walk
  // over all blocks), then the group sums are added in group order
  __shared__ float red[256];
  const int t = threadIdx.x;
  const float inv_n = 1.f / (float)n;
  for (int64_t c0 = 0; c0 < d; c0 += 256) {
    const int dc = (int)min((int64_t)256, d - c0);
    const int G = 256 / dc;
    float a = 0.f;
    if (t < dc * G) {
      const int64_t c = c0 + t % dc;
      for (int64_t b = t / dc; b < blocks; b += G) a += partial[b * d + c];
    }
    red[t] = a;
    __syncthreads();
    group_reduce(red, dc, G);
    if (t < dc) {
      const int64_t c = c0 + t;
      float p = inv_n * red[t];
      if (extra) p += extra[c];
      if (phi_out) phi_out[c] = p;
      X[i * ldx + c] += step * p;
    }
    __syncthreads();
  }
}

// NN block shape: 128 rows x 128*TN columns, 8 waves (2 per SIMD, 128
// accumulators each); K-steps of 32 columns (two D panels per barrier,
// 160 KiB LDS, XOR-swizzled A image) when K allows, else 16.
template <int TN, int BJ>
int launch_nn_shape(bool exp_, const float* A, const float* B, int64_t ldb, int64_t K, int splits,
                    const dsvgd_select_state* st, float* C, int64_t ldc, float* rowsum, int64_t m,
                    int64_t cols, int64_t row0, hipStream_t s, const float* gate) {
  constexpr int WM = 2, TM = 2, BM = 32 * TM * WM;
  if (K % BJ != 0) return fail_arg("nn_kernel: K must be a multiple of the K-step");
  const int64_t kchunk = roundup((K + splits - 1) / splits, BJ);
  const dim3 grid(cols / (128 * TN), roundup(m, BM) / BM, splits);
  if (exp_)
    hipLaunchKernelGGL((nn_kernel<TN, true, WM, TM, BJ>), grid, dim3(256 * WM), 0, s, A, K, B, ldb,
                       K, kchunk, st, C, ldc, rowsum, m, row0, gate);
  else
    hipLaunchKernelGGL((nn_kernel<TN, false, WM, TM, BJ>), grid, dim3(256 * WM), 0, s, A, K, B, ldb,
                       K, kchunk, st, C, ldc, rowsum, m, row0, gate);
  return check_launch("nn_kernel");
}

template <int TN>
int launch_nn(bool exp_, const float* A, const float* B, int64_t ldb, int64_t K, int splits,
              const dsvgd_select_state* st, float* C, int64_t ldc, float* rowsum, int64_t m,
              int64_t cols, int64_t row0, hipStream_t s, const float* gate) {
  if (K % 32 == 0)  // split-K chunks are rounded to the K-step
    return launch_nn_shape<TN, 32>(exp_, A, B, ldb, K, splits, st, C, ldc, rowsum, m, cols, row0,
                                   s, gate);
  return launch_nn_shape<TN, 16>(exp_, A, B, ldb, K, splits, st, C, ldc, rowsum, m, cols, row0, s,
                                 gate);
}

// C[splits x m x cols] = f(A) B with A in panel layout (m_pad x K), B row-major K x cols.
// exp_: f = exp2(-inv_h log2e a) with the diagonal (column row0 + i) skipped.
int nn_gemm(bool exp_, const float* A, int64_t K, const float* B, int64_t ldb, int64_t cols,
            int splits, const dsvgd_select_state* st, float* C, int64_t ldc, float* rowsum,
            int64_t m, int64_t row0, hipStream_t s, const float* gate) {
  // buffer-resource loads: 32-bit byte offsets from a block's A row panel
  // (K columns x 128 rows) and from B's first row (K rows x ldb)
  if (K * ldb * (int64_t)sizeof(float) >= ((int64_t)1 << 31) ||
      K * 128 * (int64_t)sizeof(float) >= ((int64_t)1 << 31))
    return fail_arg("nn_kernel: K x ldb too large for 32-bit buffer offsets (split the columns)");
  if (cols % 512 == 0)
    return launch_nn<4>(exp_, A, B, ldb, K, splits, st, C, ldc, rowsum, m, cols, row0, s, gate);
  if (cols % 256 == 0)
    return launch_nn<2>(exp_, A, B, ldb, K, splits, st, C, ldc, rowsum, m, cols, row0, s, gate);
  return launch_nn<1>(exp_, A, B, ldb, K, splits, st, C, ldc, rowsum, m, cols, row0, s, gate);
}

// split-K slices: (1) enough for >= 2 blocks per CU (256 CUs) when the owned
// row block is small (S ranks), (2) at most kMaxChain columns per fp32
// accumulation chain.  (2) is precision: K.S is a coherent sum (|sum| grows
// linearly), so one n-long fma chain loses ~sqrt(n) eps |sum| -- 8.7e-6 of
// max|phi| at n = 65536, d = 256 on the round-1 engine (scripts/diag_precision.py);
// slices summed in slice order by phi_finish cut that.  FmtH2 at n = 65536:
// 5.2e-7 with 8192-long slices, 7.8e-7 with 16384 (shipped: half the
// partials to write and re-read, S = 1 step -1.7 %; profiles/r5g/).
// (kMaxChain: defined with g_phi_symrow above)

int64_t phi_splits(int64_t m, int64_t n, int64_t ldy) {
  const int64_t cols = ldy % 512 == 0 ? 512 : (ldy % 256 == 0 ? 256 : 128);
  const int64_t blocks = (roundup(m, 128) / 128) * (ldy / cols);
  const int64_t n_pad = roundup(n, 128);
  int64_t s = 1;
  while (blocks * s < 512 && n_pad / (2 * s) >= 1024) s *= 2;
  while (n_pad / s > kMaxChain && s < 64) s *= 2;
  // (the symmetric layout's hybrid gives each of its two launches half the
  // slices, so a chain reaches 2 kMaxChain there: 1.2e-6 phi error at n =
  // 65536; twice the slices cost 1.4 % of phi_mm, profiles/r6y)
  return s;
}

}  // namespace dsvgd

using namespace dsvgd;

extern "C" {

int64_t dsvgd_phi_splits(int64_t m, int64_t n, int64_t ldy) { return phi_splits(m, n, ldy); }

int64_t dsvgd_phi_splits_sym(int64_t n, int64_t ldy) {
  int64_t s = phi_splits(n, n, ldy);
  // only the one-launch form (phi_w1 DS 4: symrow on, TN = 4, i.e. ldy a
  // multiple of 512) takes the longer slices; the hybrid and the 8-wave
  // symmetric tile give each of their launches half the slices, so halving
  // them there would double their chains again
  if (!g_phi_symrow || ldy % 512 != 0) return s;
  // the one-launch form: its slices' chains may reach 2 kMaxChain (as each
  // launch of the hybrid's did), while the launch still fills the CUs twice
  const int64_t n_pad = roundup(n, 128), blocks = (n_pad / 128) * (ldy / 512);
  while (s > 2 && n_pad / (s / 2) <= 2 * kMaxChain && blocks * (s / 2) >= 512) s /= 2;
  return s;
}

int dsvgd_phi_set_gxd_w1(int on) {
  const int prev = g_gxd_w1;
  g_gxd_w1 = on ? 1 : 0;
  return prev;
}

int dsvgd_phi_set_xmap(int mask) {
  const int prev = g_phi_xmap;
  g_phi_xmap = mask & 7;
  return prev;
}

int dsvgd_phi_set_symrow(int on) {
  const int prev = g_phi_symrow;
  g_phi_symrow = on ? 1 : 0;
  return prev;
}

int dsvgd_phi_mm(const float* D, int64_t ldd, const float* Y, int64_t ldy, int64_t row0,
                 int64_t m, int64_t n, const dsvgd_select_state* st, int64_t splits, float* KY,
                 int64_t ldk, float* rowsum, void* stream) {
  DSVGD_REQUIRE(D && Y && st && KY && rowsum, "null pointer");
  DSVGD_REQUIRE(m > 0 && n > 0, "sizes");
  const int64_t n_pad = roundup(n, 128);
  DSVGD_REQUIRE(ldd == n_pad, "ldd must equal roundup(n,128) (panel layout)");
  DSVGD_REQUIRE(ldy % 128 == 0 && ldk >= ldy, "ldy must be a multiple of 128, ldk >= ldy");
  DSVGD_REQUIRE(((uintptr_t)Y & 15) == 0 && ((uintptr_t)D & 15) == 0, "16-byte alignment");
  DSVGD_REQUIRE(roundup(m, 128) / 128 <= 65535, "too many row tiles");
  DSVGD_REQUIRE(splits >= 1 && splits <= 1024, "splits must be in [1, 1024]");
  DSVGD_REQUIRE(row0 >= 0 && row0 + m <= n, "row block outside [0, n)");
  return nn_gemm(true, D, n_pad, Y, ldy, ldy, (int)splits, st, KY, ldk, rowsum, m, row0,
                 (hipStream_t)stream, nullptr);
}

int dsvgd_phi_mm_gated(const float* D, int64_t ldd, const float* Y, int64_t ldy, int64_t row0,
                       int64_t m, int64_t n, const dsvgd_select_state* st, int64_t splits,
                       float* KY, int64_t ldk, float* rowsum, const float* gate, void* stream) {
  DSVGD_REQUIRE(D && Y && st && KY && rowsum && gate, "null pointer");
  DSVGD_REQUIRE(m > 0 && n > 0, "sizes");
  const int64_t n_pad = roundup(n, 128);
  DSVGD_REQUIRE(ldd == n_pad, "ldd must equal roundup(n,128) (panel layout)");
  DSVGD_REQUIRE(ldy % 128 == 0 && ldk >= ldy, "ldy must be a multiple of 128, ldk >= ldy");
  DSVGD_REQUIRE(((uintptr_t)Y & 15) == 0 && ((uintptr_t)D & 15) == 0, "16-byte alignment");
  DSVGD_REQUIRE(roundup(m, 128) / 128 <= 65535, "too many row tiles");
  DSVGD_REQUIRE(splits >= 1 && splits <= 1024, "splits must be in [1, 1024]");
  DSVGD_REQUIRE(row0 >= 0 && row0 + m <= n, "row block outside [0, n)");
  return nn_gemm(true, D, n_pad, Y, ldy, ldy, (int)splits, st, KY, ldk, rowsum, m, row0,
                 (hipStream_t)stream, gate);
}

int64_t dsvgd_ysplit_bytes(int64_t rows, int64_t ldy) {
  return roundup(rows, kX3Step) * kX3Parts * ldy * 2;
}

int dsvgd_ysplit(const float* Y, int64_t ldy, int64_t rows, void* Yx, int swz, const float* gate,
                 void* stream) {
  DSVGD_REQUIRE(Y && Yx, "null pointer");
  DSVGD_REQUIRE(rows > 0 && rows % kX3Step == 0, "rows must be a positive multiple of 16");
  DSVGD_REQUIRE(ldy > 0 && ldy % 8 == 0, "ldy must be a multiple of 8");
  DSVGD_REQUIRE(((uintptr_t)Yx & 15) == 0, "16-byte alignment");
  const int64_t ksteps = rows / kX3Step, threads = ksteps * ldy;
  hipLaunchKernelGGL(ysplit_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, Y, ldy, ksteps, (__bf16*)Yx, swz, gate);
  return check_launch("ysplit");
}

int64_t dsvgd_rowsplit_bytes(int64_t rows_pad, int64_t kpad) {
  return roundup(kpad, kX3Step) * rows_pad * kX3Parts * 2;
}

int dsvgd_rowsplit(const float* A, int64_t lda, int64_t rows, int64_t cols, int64_t rows_pad,
                   int64_t kpad, void* img, int swz, void* stream) {
  DSVGD_REQUIRE(A && img, "null pointer");
  DSVGD_REQUIRE(rows >= 0 && cols >= 0 && rows <= rows_pad && lda >= cols, "sizes");
  DSVGD_REQUIRE(rows_pad > 0 && rows_pad % 16 == 0 && kpad > 0 && kpad % kX3Step == 0,
                "rows_pad and kpad must be positive multiples of 16");
  DSVGD_REQUIRE(((uintptr_t)img & 15) == 0, "16-byte alignment");
  const int64_t ksteps = kpad / kX3Step, threads = ksteps * rows_pad;
  hipLaunchKernelGGL(rowsplit_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, A, lda, rows, cols, rows_pad, ksteps, (__bf16*)img, swz);
  return check_launch("rowsplit");
}

int dsvgd_phi_mm_x3(const float* D, int64_t ldd, const void* Yx, int64_t ldy, int64_t row0,
                    int64_t m, int64_t n, const dsvgd_select_state* st, int64_t splits, float* KY,
                    int64_t ldk, float* rowsum, int sym, int m16, const float* gate,
                    void* stream) {
  DSVGD_REQUIRE(D && Yx && st && KY && rowsum, "null pointer");
  DSVGD_REQUIRE(m > 0 && n > 0, "sizes");
  const int64_t n_pad = roundup(n, 128);
  DSVGD_REQUIRE(ldd == n_pad, "ldd must equal roundup(n,128) (panel layout)");
  DSVGD_REQUIRE(ldy % 128 == 0 && ldk >= ldy, "ldy must be a multiple of 128, ldk >= ldy");
  DSVGD_REQUIRE(((uintptr_t)Yx & 15) == 0 && ((uintptr_t)D & 15) == 0, "16-byte alignment");
  DSVGD_REQUIRE(roundup(m, 128) / 128 <= 65535, "too many row tiles");
  DSVGD_REQUIRE(splits >= 1 && splits <= 1024, "splits must be in [1, 1024]");
  DSVGD_REQUIRE(row0 >= 0 && row0 + m <= n, "row block outside [0, n)");
  // buffer-resource loads: 32-bit byte offsets into the block's D panel row
  // and into Yx (K rows x 3 parts x ldy x 2 B)
  DSVGD_REQUIRE(n_pad * ldy * 6 < ((int64_t)1 << 31) && n_pad * 128 * 4 < ((int64_t)1 << 31),
                "n x ldy too large for 32-bit buffer offsets (use dsvgd_phi_mm)");
  DSVGD_REQUIRE(!sym || (m == n && row0 == 0), "sym: the symmetric layout needs m == n, row0 == 0");
  return nn_x3_gemm(true, D, n_pad, (const __bf16*)Yx, ldy, (int)splits, st, KY, ldk, rowsum, m,
                    row0, (hipStream_t)stream, sym, m16, gate);
}

int dsvgd_phi_mm_h2(const float* D, int64_t ldd, const void* Yh, int64_t ldy, int64_t row0,
                    int64_t m, int64_t n, const dsvgd_select_state* st, int64_t splits, float* KY,
                    int64_t ldk, float* rowsum, int sym, const float* colinv, const float* gate,
                    void* stream) {
  DSVGD_REQUIRE(D && Yh && st && KY && rowsum && colinv, "null pointer");
  DSVGD_REQUIRE(m > 0 && n > 0, "sizes");
  const int64_t n_pad = roundup(n, 128);
  DSVGD_REQUIRE(ldd == n_pad, "ldd must equal roundup(n,128) (panel layout)");
  DSVGD_REQUIRE(ldy % 128 == 0 && ldk >= ldy, "ldy must be a multiple of 128, ldk >= ldy");
  DSVGD_REQUIRE(((uintptr_t)Yh & 15) == 0 && ((uintptr_t)D & 15) == 0, "16-byte alignment");
  DSVGD_REQUIRE(roundup(m, 128) / 128 <= 65535, "too many row tiles");
  DSVGD_REQUIRE(splits >= 1 && splits <= 1024, "splits must be in [1, 1024]");
  DSVGD_REQUIRE(row0 >= 0 && row0 + m <= n, "row block outside [0, n)");
  DSVGD_REQUIRE(n_pad * ldy * 4 < ((int64_t)1 << 31) && n_pad * 128 * 4 < ((int64_t)1 << 31),
                "n x ldy too large for 32-bit buffer offsets (use dsvgd_phi_mm)");
  DSVGD_REQUIRE(!sym || (m == n && row0 == 0 && ldy % 256 == 0),
                "sym: the symmetric layout needs m == n, row0 == 0, ldy % 256 == 0");
  return nn_h2_gemm(true, D, n_pad, (const _Float16*)Yh, ldy, (int)splits, st, KY, ldk, rowsum, m,
                    row0, (hipStream_t)stream, sym, colinv, gate);
}

int dsvgd_phi_h2_window(const float* D, int64_t ldd, const void* Yh, int64_t ldy, int64_t row0,
                        int64_t m, int64_t n, int64_t col0, int64_t wlen,
                        const dsvgd_select_state* st, int64_t splits, float* KY, int64_t ldk,
                        float* rowsum, const float* colinv, const float* gate, int gate_on,
                        void* stream) {
  DSVGD_REQUIRE(D && Yh && st && KY && rowsum && colinv, "null pointer");
  const int64_t n_pad = roundup(n, 128);
  DSVGD_REQUIRE(ldd == n_pad, "ldd must equal roundup(n,128) (panel layout)");
  DSVGD_REQUIRE(m > 0 && row0 >= 0 && row0 + m <= n, "rows outside [0, n)");
  DSVGD_REQUIRE(ldy % 512 == 0 && ldk >= ldy, "ldy must be a multiple of 512, ldk >= ldy");
  DSVGD_REQUIRE(col0 >= 0 && col0 < n_pad && col0 % 16 == 0 && wlen > 0 && wlen <= n_pad &&
                    wlen % 16 == 0,
                "window: col0 in [0, n_pad), wlen in (0, n_pad], multiples of 16");
  DSVGD_REQUIRE(splits >= 1 && splits <= 1024, "splits must be in [1, 1024]");
  DSVGD_REQUIRE(n_pad * ldy * 4 < ((int64_t)1 << 31), "n x ldy too large for 32-bit offsets");
  DSVGD_REQUIRE(((uintptr_t)Yh & 15) == 0 && ((uintptr_t)D & 15) == 0, "16-byte alignment");
  const int64_t kchunk = roundup((wlen + splits - 1) / splits, (int64_t)PhiW1::BJ);
  const dim3 grid((unsigned)(ldy / PhiW1::BC), (unsigned)(roundup(m, 128) / 128), (unsigned)splits);
  launch_w1<0>(grid, (hipStream_t)stream, D, n_pad, (const _Float16*)Yh, ldy, wlen, kchunk, st, KY,
               ldk, rowsum, m, row0, 0, colinv, 0, gate, gate_on, (int)(col0 / PhiW1::BJ),
               (int)(n_pad / PhiW1::BJ), 0, xmap_ok(grid, 2));
  return check_launch("phi_w1_kernel(window)");
}

int dsvgd_phi_h2_transposed(const float* D, int64_t ldd, const void* Yh, int64_t ldy,
                            int64_t yrow0, int64_t krows, int64_t col0, int64_t mo, int64_t n,
                            const dsvgd_select_state* st, int64_t splits, float* P, int64_t ldp,
                            float* rs, const float* colinv, const float* gate, int gate_on,
                            void* stream) {
  DSVGD_REQUIRE(D && Yh && st && P && rs && colinv, "null pointer");
  const int64_t n_pad = roundup(n, 128);
  DSVGD_REQUIRE(ldd == n_pad, "ldd must equal roundup(n,128) (panel layout)");
  DSVGD_REQUIRE(ldy % 512 == 0 && ldp >= ldy, "ldy must be a multiple of 512, ldp >= ldy");
  DSVGD_REQUIRE(krows > 0 && krows % 16 == 0 && yrow0 >= 0 && yrow0 % 16 == 0 &&
                    yrow0 + krows <= n_pad,
                "the rectangle's rows: a multiple of 16 inside [0, n_pad)");
  DSVGD_REQUIRE(mo > 0 && col0 >= 0 && col0 % 128 == 0 && col0 + roundup(mo, 128) <= n_pad,
                "the rectangle's columns: 128-aligned inside [0, n_pad)");
  DSVGD_REQUIRE(splits >= 1 && splits <= 1024, "splits must be in [1, 1024]");
  DSVGD_REQUIRE(n_pad * ldy * 4 < ((int64_t)1 << 31), "n x ldy too large for 32-bit offsets");
  DSVGD_REQUIRE(((uintptr_t)Yh & 15) == 0 && ((uintptr_t)D & 15) == 0, "16-byte alignment");
  const int64_t kchunk = roundup((krows + splits - 1) / splits, (int64_t)PhiW1::BJ);
  const dim3 grid((unsigned)(ldy / PhiW1::BC), (unsigned)(roundup(mo, 128) / 128),
                  (unsigned)splits);
  launch_w1<3>(grid, (hipStream_t)stream, D, n_pad, (const _Float16*)Yh, ldy, krows, kchunk, st, P,
               ldp, rs, mo, (int64_t)0, 0, colinv, 0, gate, gate_on, (int)(yrow0 / PhiW1::BJ), 0,
               (int)(col0 / 128));
  return check_launch("phi_w1_kernel(transposed)");
}

int dsvgd_phi_h2_transposed_blocks(const float* D, int64_t ldd, const void* Yh, int64_t ldy,
                                   int64_t yrow0, int64_t m, int64_t first, int64_t nblocks,
                                   int64_t count, int64_t n, const dsvgd_select_state* st,
                                   float* P, int64_t ldp, int64_t pstride, const float* colinv,
                                   const float* gate, int gate_on, void* stream) {
  return dsvgd_phi_h2_transposed_blocks_split(D, ldd, Yh, ldy, yrow0, m, first, nblocks, count, 1,
                                              n, st, P, ldp, pstride, colinv, gate, gate_on,
                                              stream);
}

int dsvgd_phi_h2_transposed_blocks_split(const float* D, int64_t ldd, const void* Yh, int64_t ldy,
                                         int64_t yrow0, int64_t m, int64_t first, int64_t nblocks,
                                         int64_t count, int64_t zsplit, int64_t n,
                                         const dsvgd_select_state* st, float* P, int64_t ldp,
                                         int64_t pstride, const float* colinv, const float* gate,
                                         int gate_on, void* stream) {
  DSVGD_REQUIRE(D && Yh && st && P && colinv, "null pointer");
  const int64_t n_pad = roundup(n, 128);
  DSVGD_REQUIRE(ldd == n_pad, "ldd must equal roundup(n,128) (panel layout)");
  DSVGD_REQUIRE(ldy % 512 == 0 && ldp >= ldy, "ldy must be a multiple of 512, ldp >= ldy");
  DSVGD_REQUIRE(m > 0 && m % 128 == 0 && nblocks * m <= n_pad && count >= 1 &&
                    count <= nblocks && first >= 0 && first < nblocks,
                "blocks: m a multiple of 128, count <= nblocks, nblocks m <= n_pad");
  DSVGD_REQUIRE(yrow0 >= 0 && yrow0 % 16 == 0 && yrow0 + m <= n_pad, "the rectangle's rows");
  DSVGD_REQUIRE(pstride >= m * ldp + roundup(m, 128), "pstride: room for P and its row sums");
  DSVGD_REQUIRE(zsplit >= 1 && zsplit <= 64 && m % (16 * zsplit) == 0,
                "zsplit in [1, 64], m a multiple of 16 zsplit");
  DSVGD_REQUIRE(n_pad * ldy * 4 < ((int64_t)1 << 31), "n x ldy too large for 32-bit offsets");
  DSVGD_REQUIRE(((uintptr_t)Yh & 15) == 0 && ((uintptr_t)D & 15) == 0, "16-byte alignment");
  const int64_t per = m / 128;
  const dim3 grid((unsigned)(ldy / PhiW1::BC), (unsigned)(per * count), (unsigned)zsplit);
  // (tcol0 is unused by the batched form: 1 = its slices mapped to XCDs)
  launch_w1<3>(grid, (hipStream_t)stream, D, n_pad, (const _Float16*)Yh, ldy, m, m / zsplit, st, P, ldp,
               P + m * ldp, m, (int64_t)0, 0, colinv, 0, gate, gate_on, (int)(yrow0 / PhiW1::BJ), 0,
               xmap_ok(grid, 4), (int)per, (int)first, (int)nblocks, pstride);
  return check_launch("phi_w1_kernel(transposed blocks)");
}

int dsvgd_phi_partial_reduce_blocks(const float* P, int64_t ldp, int64_t pstride, int64_t zsplit,
                                    int64_t count, int64_t rows, int64_t cols, float* out,
                                    int64_t ldo, int64_t ostride, void* stream) {
  DSVGD_REQUIRE(P && out, "null pointer");
  DSVGD_REQUIRE(rows > 0 && cols > 0 && cols % 4 == 0 && ldp >= cols && ldo >= cols &&
                    ldp % 4 == 0 && ldo % 4 == 0,
                "sizes (cols, ldp, ldo multiples of 4)");
  DSVGD_REQUIRE(zsplit >= 1 && zsplit <= 1024 && count >= 1 && count <= 65535, "zsplit, count");
  DSVGD_REQUIRE(pstride >= rows * ldp + roundup(rows, 128) && ostride >= rows * ldo + rows &&
                    pstride % 4 == 0 && ostride % 4 == 0,
                "strides: room for a partial and its row sums");
  DSVGD_REQUIRE(((uintptr_t)P & 15) == 0 && ((uintptr_t)out & 15) == 0, "16-byte alignment");
  const int64_t positions = rows * (cols / 4) + (rows + 3) / 4;
  int G = 1;
  while (G < zsplit && G < 16) G *= 2;
  const int64_t per = 256 / G;
  hipLaunchKernelGGL(partial_reduce_kernel,
                     dim3((unsigned)((positions + per - 1) / per), (unsigned)count), dim3(256), 0,
                     (hipStream_t)stream, P, ldp, P + rows * ldp, (int)zsplit, rows, cols, out, ldo,
                     out + rows * ldo, G, count * pstride, count * pstride, pstride, ostride);
  return check_launch("partial_reduce(blocks)");
}

int dsvgd_phi_partial_reduce(const float* P, int64_t ldp, const float* rs, int64_t splits,
                             int64_t rows, int64_t cols, float* out, int64_t ldo, float* out_rs,
                             void* stream) {
  DSVGD_REQUIRE(P && rs && out && out_rs, "null pointer");
  DSVGD_REQUIRE(rows > 0 && cols > 0 && cols % 4 == 0 && ldp >= cols && ldo >= cols &&
                    ldp % 4 == 0 && ldo % 4 == 0,
                "sizes (cols, ldp, ldo multiples of 4)");
  DSVGD_REQUIRE(splits >= 1 && splits <= 1024, "splits must be in [1, 1024]");
  DSVGD_REQUIRE(((uintptr_t)P & 15) == 0 && ((uintptr_t)out & 15) == 0, "16-byte alignment");
  const int64_t positions = rows * (cols / 4) + (rows + 3) / 4;
  int G = 1;
  while (G < splits && G < 16) G *= 2;
  const int64_t per = 256 / G;
  hipLaunchKernelGGL(partial_reduce_kernel, dim3((unsigned)((positions + per - 1) / per)), dim3(256),
                     0, (hipStream_t)stream, P, ldp, rs, (int)splits, rows, cols, out, ldo, out_rs,
                     G, rows * ldp, roundup(rows, (int64_t)128), (int64_t)0, (int64_t)0);
  return check_launch("partial_reduce");
}

int dsvgd_phi_finish_parts(const float* KY, int64_t ldk, const float* rowsum, int64_t splits,
                           const float* Y, int64_t ldy, int64_t row0, int64_t m, int64_t d,
                           int64_t dp, const dsvgd_select_state* st, float inv_n, float step,
                           const float* extra, int64_t lde, float* phi, int64_t ldphi, float* X,
                           int64_t ldx, const dsvgd_phi_part* parts, int nparts,
                           const float* gate, int64_t splits_fb, void* stream) {
  DSVGD_REQUIRE(KY && rowsum && Y && st, "null pointer");
  DSVGD_REQUIRE(!extra || lde >= d, "lde");
  DSVGD_REQUIRE(splits >= 1 && splits <= 1024 && splits_fb >= 0 && splits_fb <= 1024,
                "splits must be in [1, 1024]");
  DSVGD_REQUIRE(m > 0 && d > 0 && dp >= d && ldk >= 2 * dp && ldy >= 2 * dp, "sizes");
  DSVGD_REQUIRE(!phi || ldphi >= d, "ldphi");
  DSVGD_REQUIRE(!X || ldx >= d, "ldx");
  DSVGD_REQUIRE(nparts >= 0 && nparts <= kMaxPhiParts && (nparts == 0 || parts),
                "at most 16 parts");
  PhiPartsArg pa{};
  pa.n = nparts;
  for (int p = 0; p < nparts; ++p) {
    const dsvgd_phi_part& q = parts[p];
    DSVGD_REQUIRE(q.ky && q.rs, "null part");
    DSVGD_REQUIRE(q.row_off >= 0 && q.rows > 0 && q.row_off + q.rows <= m && q.ldk >= 2 * dp &&
                      q.splits >= 1 && q.splits <= 1024,
                  "part rows inside the block, ldk >= 2 dp, splits in [1, 1024]");
    pa.ky[p] = q.ky;
    pa.rs[p] = q.rs;
    pa.ldk[p] = q.ldk;
    pa.row_off[p] = q.row_off;
    pa.rows[p] = q.rows;
    pa.splits[p] = (int)q.splits;
  }
  hipLaunchKernelGGL(phi_finish_parts_kernel, dim3((unsigned)((m * d + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, KY, ldk, rowsum, (int)splits, Y, ldy, row0, m, d, dp,
                     st, inv_n, step, extra, lde, phi, ldphi, X, ldx, pa, gate,
                     (int)(splits_fb ? splits_fb : splits));
  return check_launch("phi_finish_parts");
}

// A/B switch (default 1): dsvgd_phi_finish on four columns per thread where
// the layout allows (phi_finish4_kernel, the same bits)
static int g_phi_finish_vec = 1;
int dsvgd_phi_set_finish_vec(int on) {
  const int prev = g_phi_finish_vec;
  g_phi_finish_vec = on ? 1 : 0;
  return prev;
}

int dsvgd_phi_finish(const float* KY, int64_t ldk, const float* rowsum, int64_t splits,
                     const float* Y, int64_t ldy, int64_t row0, int64_t m, int64_t d, int64_t dp,
                     const dsvgd_select_state* st, float inv_n, float step, const float* extra,
                     int64_t lde, float* phi, int64_t ldphi, float* X, int64_t ldx,
                     void* stream) {
  DSVGD_REQUIRE(KY && rowsum && Y && st, "null pointer");
  DSVGD_REQUIRE(!extra || lde >= d, "lde");
  DSVGD_REQUIRE(splits >= 1 && splits <= 1024, "splits must be in [1, 1024]");
  DSVGD_REQUIRE(m > 0 && d > 0 && dp >= d && ldk >= 2 * dp && ldy >= 2 * dp, "sizes");
  DSVGD_REQUIRE(!phi || ldphi >= d, "ldphi");
  DSVGD_REQUIRE(!X || ldx >= d, "ldx");
  auto a16 = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
  if (g_phi_finish_vec && d % 4 == 0 && dp % 4 == 0 && ldk % 4 == 0 && ldy % 4 == 0 &&
      a16(KY) && a16(Y) && (!extra || (lde % 4 == 0 && a16(extra))) &&
      (!phi || (ldphi % 4 == 0 && a16(phi))) && (!X || (ldx % 4 == 0 && a16(X)))) {
    const int64_t d4 = d / 4;
    hipLaunchKernelGGL(phi_finish4_kernel, dim3((unsigned)((m * d4 + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, KY, ldk, rowsum, (int)splits, Y, ldy, row0, m, d4,
                       dp, st, inv_n, step, extra, lde, phi, ldphi, X, ldx);
    return check_launch("phi_finish4");
  }
  hipLaunchKernelGGL(phi_finish_kernel, dim3((m * d + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, KY, ldk, rowsum, (int)splits, Y, ldy, row0, m, d, dp,
                     st, inv_n, step, extra, lde, phi, ldphi, X, ldx);
  return check_launch("phi_finish");
}

int dsvgd_phi_direct(const float* D, int64_t ldd, const float* Y, int64_t ldy, int64_t row0,
                     int64_t m, int64_t n, int64_t d, const dsvgd_select_state* st, float inv_n,
                     float step, const float* extra, int64_t lde, float* phi, int64_t ldphi,
                     float* X, int64_t ldx, float* partial, int64_t partial_floats,
                     void* stream) {
  DSVGD_REQUIRE(D && Y && st, "null pointer");
  DSVGD_REQUIRE(!extra || lde >= d, "lde");
  DSVGD_REQUIRE(m > 0 && n > 0 && d > 0 && row0 >= 0, "sizes");
  DSVGD_REQUIRE(d <= kPhiDirectMaxD, "phi_direct supports d <= 64");
  const int64_t n_pad = roundup(n, 128), dp = roundup(d, 32);
  DSVGD_REQUIRE(ldd == n_pad, "ldd must equal roundup(n,128) (panel layout)");
  DSVGD_REQUIRE(ldy >= 2 * dp, "ldy");
  DSVGD_REQUIRE(!phi || ldphi >= d, "ldphi");
  DSVGD_REQUIRE(!X || ldx >= d, "ldx");
  DSVGD_REQUIRE(!partial || partial_floats >= 0, "partial_floats");
  // split J over blockIdx.y until ~512 blocks (a few row blocks alone leave
  // the chip idle at small n), as far as the partial buffer holds
  const int64_t rb = (m + 63) / 64;
  int64_t nsplit = 1;
  if (partial) {
    nsplit = std::min<int64_t>((512 + rb - 1) / rb, (n + 63) / 64);
    nsplit = std::min<int64_t>(nsplit, partial_floats / (m * d));
    nsplit = std::max<int64_t>(nsplit, 1);
  }
  const int64_t jchunk = roundup((n + nsplit - 1) / nsplit, 64);
  nsplit = (n + jchunk - 1) / jchunk;
  float* part = nsplit > 1 ? partial : nullptr;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(phi_direct_kernel, dim3((unsigned)rb, (unsigned)nsplit), dim3(256), 0, s, D,
                     n_pad, Y, ldy, row0, m, n, (int)d, dp, st, inv_n, step, extra, lde, phi, ldphi,
                     X, ldx, jchunk, part);
  int rc = check_launch("phi_direct");
  if (rc || !part) return rc;
  hipLaunchKernelGGL(phi_direct_finish_kernel, dim3((unsigned)((m * d + 255) / 256)), dim3(256), 0,
                     s, part, (int)nsplit, m, d, inv_n, step, extra, lde, phi, ldphi, X, ldx);
  return check_launch("phi_direct_finish");
}

int dsvgd_phi_row(float* X, int64_t ldx, const float* S, int64_t lds, int64_t n_int, int64_t d,
                  int64_t i, const dsvgd_select_state* st, float step, const float* extra,
                  float* phi_out, void* stream) {
  DSVGD_REQUIRE(X && S && st, "null pointer");
  DSVGD_REQUIRE(n_int > 0 && d > 0 && i >= 0 && i < n_int && ldx >= d && lds >= d, "sizes");
  DSVGD_REQUIRE(d <= 7936, "phi_row supports d <= 7936 (64 KiB LDS)");
  const size_t shm = (size_t)(2 * d + 512) * sizeof(float);
  hipLaunchKernelGGL(phi_row_kernel, dim3(1), dim3(256), shm, (hipStream_t)stream, X, ldx, S, lds,
                     n_int, d, i, st, step, extra, phi_out);
  return check_launch("phi_row");
}

int64_t dsvgd_phi_row_blocks(int64_t n, int64_t d) {
  // one workgroup while it has few rows to walk (the reference's small n);
  // else ~64+ rows per workgroup, at most 256 workgroups
  if (n < 2048 || d > 4096) return 1;
  return std::min<int64_t>(256, (n + 63) / 64);
}

int dsvgd_phi_row_split(float* X, int64_t ldx, const float* S, int64_t lds, int64_t n, int64_t d,
                        int64_t i, const dsvgd_select_state* st, float step, const float* extra,
                        float* phi_out, float* partial, int64_t blocks, void* stream) {
  DSVGD_REQUIRE(X && S && st && partial, "null pointer");
  DSVGD_REQUIRE(n > 0 && d > 0 && ldx >= d && lds >= d && i >= 0 && i < n, "sizes");
  DSVGD_REQUIRE(blocks >= 1 && blocks <= 65535, "blocks must be in [1, 65535]");
  DSVGD_REQUIRE(d <= 4096, "d <= 4096 (x_i is staged in LDS)");
  const int64_t J = (n + blocks - 1) / blocks;
  const size_t shm = (size_t)(((d + 3) & ~(int64_t)3) + 256 + J) * sizeof(float);
  DSVGD_REQUIRE(shm <= 64 * 1024, "rows per workgroup exceed the LDS budget (use more blocks)");
  hipStream_t s = (hipStream_t)stream;
  if (ldx % 4 == 0 && ((uintptr_t)X & 15) == 0)
    hipLaunchKernelGGL(phi_row_part_kernel<true>, dim3((unsigned)blocks), dim3(256), shm, s, X, ldx,
                       S, lds, n, d, i, J, st, partial);
  else
    hipLaunchKernelGGL(phi_row_part_kernel<false>, dim3((unsigned)blocks), dim3(256), shm, s, X,
                       ldx, S, lds, n, d, i, J, st, partial);
  int rc = check_launch("phi_row_part");
  if (rc) return rc;
  hipLaunchKernelGGL(phi_row_finish_kernel, dim3(1), dim3(256), 0, s, X, ldx, n, d, i, partial,
                     blocks, step, extra, phi_out);
  return check_launch("phi_row_finish");
}

}  // extern "C"
