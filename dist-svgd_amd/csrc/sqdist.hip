// sqdist.hip -- pairwise squared distances D_ij = ||x_i - x_j||^2 in the panel
// layout, plus the per-entry accounting of the exact median select.
//
// d > 64: Gram form on MFMA (v_mfma_f32_32x32x2_f32) over centred particles,
//   upper-triangle tiles only for a square block (mirror stored).  Roofline per
//   128x128 tile: 2*128*128*dp flop vs 64 KiB written -> MFMA-bound for dp >= 64.
// d <= 64: explicit differences on the VALU (torch.dist semantics).
#include <cmath>

#include "gemm_tiles.hpp"
#include "select.hpp"

namespace dsvgd {

using GramTile = NTTile<2, 2, 2, 2>;  // 128 x 128 block, 4 waves of 64 x 64

// Upper-triangle tile pair (bi <= bj) of linear block id b over T x T tiles.
__device__ __forceinline__ void tri_decode(int64_t b, int T, int& bi, int& bj) {
  const double A = (double)T + 0.5;
  int x = (int)(A - sqrt(A * A - 2.0 * (double)b));
  auto off = [&](int r) { return (int64_t)r * T - (int64_t)r * (r - 1) / 2; };
  while (x > 0 && off(x) > b) --x;
  while (x + 1 < T && off(x + 1) <= b) ++x;
  bi = x;
  bj = x + (int)(b - off(x));
}

// Rows [row0, row0+m) of Y against rows [0,n).  SYM (m == n, row0 == 0): only
// tiles bi <= bj, the off-diagonal ones stored twice (tile + transpose) and
// accounted with weight 2.
template <bool SYM>
__global__ __launch_bounds__(256) void sqdist_kernel(const float* __restrict__ Y, int64_t ldy,
                                                     const float* __restrict__ norms, int64_t row0,
                                                     int64_t m, int64_t n, int64_t n_pad, int dp,
                                                     float* __restrict__ D, int smode,
                                                     dsvgd_select_state* __restrict__ st,
                                                     float* __restrict__ cand) {
  __shared__ __attribute__((aligned(16))) float smem[GramTile::kSmemFloats];
  __shared__ uint32_t shist[DSVGD_RADIX_BINS];
  __shared__ float snorm[GramTile::BM + GramTile::BN];

  int bi, bj;
  if (SYM) {
    tri_decode(blockIdx.x, (int)(n_pad / 128), bi, bj);
  } else {
    bi = blockIdx.y;
    bj = blockIdx.x;
  }
  const bool mirror = SYM && bi != bj;
  const int64_t i0 = (int64_t)bi * GramTile::BM;  // within the owned block
  const int64_t j0 = (int64_t)bj * GramTile::BN;
  if (smode == kSelHist)
    for (int b = threadIdx.x; b < DSVGD_RADIX_BINS; b += 256) shist[b] = 0u;

  GramTile tile;
  tile.run(Y + (row0 + i0) * ldy, ldy, Y + j0 * ldy, ldy, dp, smem);

  for (int t = threadIdx.x; t < GramTile::BM + GramTile::BN; t += 256)
    snorm[t] = t < GramTile::BM ? norms[row0 + i0 + t] : norms[j0 + t - GramTile::BM];
  __syncthreads();

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w >> 1, wn = w & 1;
  float v[64];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      const int cl = wn * 64 + ni * 32 + (lane & 31);
      const int64_t gj = j0 + cl;
      const float nj = snorm[GramTile::BM + cl];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rl = wm * 64 + mi * 32 + c_row(r, lane);
        const int64_t gi = i0 + rl;
        float x;
        if (gi < m && gj < n)
          x = (row0 + gi == gj) ? 0.f : fmaxf(0.f, (snorm[rl] + nj) - 2.f * tile.acc[mi][ni][r]);
        else
          x = INFINITY;
        v[(mi * 2 + ni) * 16 + r] = x;
        D[panel_off(gi, gj, n_pad)] = x;
      }
      if (mirror) {  // D[j][i]: 4 consecutive i per register quad -> 16-byte stores
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int64_t ci = i0 + wm * 64 + mi * 32 + 8 * q + 4 * (lane >> 5);
          const float* p = &v[(mi * 2 + ni) * 16 + 4 * q];
          *reinterpret_cast<f32x4*>(D + panel_off(gj, ci, n_pad)) = f32x4{p[0], p[1], p[2], p[3]};
        }
      }
    }
  const uint32_t weight = mirror ? 2u : 1u;
  if (smode == kSelHist) {
    hist_account(v, weight, shist);
    __syncthreads();
    flush_block_hist(shist, st);
  } else if (smode == kSelBracket) {
    bracket_account(v, weight, st, cand);
  }
}

// d <= 64: D_ij = sum_c (y_ic - y_jc)^2 from explicit differences on the VALU
// (what torch.dist(x, y)**2 computes per pair at experiments/logreg.py:61):
// no ||x||^2 - 2x.y cancellation, which at small d and a narrow median
// bandwidth costs more than the 1e-5 phi tolerance.  128 x 128 tile per block,
// 8 x 8 outputs per thread, both operand tiles transposed in LDS.
constexpr int kDirectMaxD = 64;

__global__ __launch_bounds__(256) void sqdist_direct_kernel(const float* __restrict__ Y,
                                                            int64_t ldy, int64_t row0, int64_t m,
                                                            int64_t n, int64_t n_pad, int d,
                                                            float* __restrict__ D, int smode,
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
  float v[64];
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    const int64_t gi = i0 + ty * 8 + a;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const int64_t gj = j0 + tx * 8 + b;
      v[a * 8 + b] = (gi < m && gj < n) ? acc[a][b] : INFINITY;
    }
    float* dst = D + panel_off(gi, j0 + tx * 8, n_pad);
    const float* p = &v[a * 8];
    *reinterpret_cast<f32x4*>(dst) = f32x4{p[0], p[1], p[2], p[3]};
    *reinterpret_cast<f32x4*>(dst + 4) = f32x4{p[4], p[5], p[6], p[7]};
  }
  if (smode == kSelHist) {
    hist_account(v, 1u, shist);
    __syncthreads();
    flush_block_hist(shist, st);
  } else if (smode == kSelBracket) {
    bracket_account(v, 1u, st, cand);
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
  if (d <= kDirectMaxD) {
    hipLaunchKernelGGL(sqdist_direct_kernel, dim3(n_pad / 128, m_pad / 128), dim3(256), 0, s, Y,
                       ldy, row0, m, n, n_pad, (int)d, D, select_mode, st, cand);
    return check_launch("sqdist_direct");
  }
  if (m == n && row0 == 0) {
    const int64_t T = n_pad / 128;
    hipLaunchKernelGGL((sqdist_kernel<true>), dim3(T * (T + 1) / 2), dim3(256), 0, s, Y, ldy,
                       norms, row0, m, n, n_pad, (int)dp, D, select_mode, st, cand);
  } else {
    hipLaunchKernelGGL((sqdist_kernel<false>), dim3(n_pad / 128, m_pad / 128), dim3(256), 0, s, Y,
                       ldy, norms, row0, m, n, n_pad, (int)dp, D, select_mode, st, cand);
  }
  return check_launch("sqdist");
}

}  // extern "C"
