// gs.hip -- the reference's Gauss-Seidel sweep (dsvgd/sampler.py:64-68,
// dsvgd/distsampler.py:194-200) in blocks of kGsB rows.
//
// Row i of a sweep moves with phi_i computed from the CURRENT particles:
// rows before i already moved, rows from i on not yet.  For a block of rows
// [r0, r0 + B):
//
//   P_i  = sum_{all j} t(x_i, x_j, s_j)        (the particles as the block starts)
//   phi_i = (P_i + sum_{r0 <= j < i} [t(x_i, x_j', s_j') - t(x_i, x_j, s_j)]) / n
//
// t(x, y, s) = k(x, y) (s + (2/h)(x - y)), k = exp(-|x - y|^2 / h), x_j' / s_j'
// the moved particle and its refreshed score.  P for the whole block is one
// wide pass over all n rows (gs_part_kernel: every CU busy, exact
// differences, split-J partials); only the in-block corrections are
// sequential (gs_sweep_kernel: one workgroup walks the B rows, the block's
// old and new rows in LDS, one barrier-separated row at a time).  The score
// refresh of a moved particle (the reference re-evaluates logp per pair, so
// later rows see it) is fused for the elementwise targets.  Same terms as the
// per-row path (dsvgd_phi_row_split), in a different summation order.
#include <algorithm>
#include <cmath>

#include "common.hpp"

namespace dsvgd {

constexpr int kGsB = 64;      // rows per block
constexpr int kGsMaxD = 64;   // features (one thread column group of 4 per 4 features)
constexpr int64_t kGsChain = 4096;

// part[z][i][c] = sum_{j in [z J, (z+1) J)} t(x_{r0+i}, x_j, s_j)[c] (raw
// sums, not / n), i < B, c < d.  Block z: the B x d outputs as 64 x 64,
// thread (rq, cq) rows 4 rq .. +3 x columns 4 cq .. +3; j in chunks of 64
// staged in LDS -- transposed copies for the distances (conflict-free f32x4
// reads along j / i), row copies for the accumulation.
__global__ __launch_bounds__(256) void gs_part_kernel(const float* __restrict__ X, int64_t ldx,
                                                      const float* __restrict__ S, int64_t lds,
                                                      int64_t n, int d, int64_t r0, int B,
                                                      const dsvgd_select_state* __restrict__ st,
                                                      int64_t jchunk, float* __restrict__ part) {
  // [c][i], [c][j]; pitch 68: the column-order staging writes 4-way instead
  // of 64-way bank conflicts, rows stay 16-byte aligned for the f32x4 reads
  __shared__ __attribute__((aligned(16))) float xiT[kGsMaxD][68];
  __shared__ __attribute__((aligned(16))) float xjT[kGsMaxD][68];
  __shared__ __attribute__((aligned(16))) float xj[64][kGsMaxD];   // [j][c]
  __shared__ __attribute__((aligned(16))) float sj[64][kGsMaxD];   // [j][c]
  __shared__ __attribute__((aligned(16))) float kT[64][64];        // [j][i]
  const int t = threadIdx.x, rq = t >> 4, cq = t & 15;
  const float inv_h = st->inv_h, g = 2.f * inv_h, scale = -inv_h * kLog2e;
  for (int e = t; e < 64 * kGsMaxD; e += 256) {
    const int i = e / kGsMaxD, c = e % kGsMaxD;
    xiT[c][i] = (i < B && c < d) ? X[(r0 + i) * ldx + c] : 0.f;
  }
  __syncthreads();
  float xr[4][4], acc[4][4], tot[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      xr[a][c] = xiT[4 * cq + c][4 * rq + a];
      acc[a][c] = 0.f;
      tot[a][c] = 0.f;
    }
  const int64_t jb = (int64_t)blockIdx.x * jchunk, je = min(n, jb + jchunk);
  for (int64_t j0 = jb; j0 < je; j0 += 64) {
    if ((j0 - jb) % kGsChain == 0 && j0 > jb) {
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          tot[a][c] += acc[a][c];
          acc[a][c] = 0.f;
        }
    }
    const int jn = (int)min((int64_t)64, je - j0);
    for (int e = t; e < 64 * kGsMaxD; e += 256) {
      const int r = e / kGsMaxD, c = e % kGsMaxD;
      const bool ok = r < jn && c < d;
      const float x = ok ? X[(j0 + r) * ldx + c] : 0.f;
      xj[r][c] = x;
      xjT[c][r] = x;
      sj[r][c] = ok ? S[(j0 + r) * lds + c] : 0.f;
    }
    __syncthreads();
    // k for rows 4 rq .. +3 x j 4 cq .. +3 (exact differences)
    float dd[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) dd[a][b] = 0.f;
    for (int c = 0; c < d; ++c) {
      const f32x4 xa = *reinterpret_cast<const f32x4*>(&xiT[c][4 * rq]);
      const f32x4 xb = *reinterpret_cast<const f32x4*>(&xjT[c][4 * cq]);
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const float df = xa[a] - xb[b];
          dd[a][b] = fmaf(df, df, dd[a][b]);
        }
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b)
        kT[4 * cq + b][4 * rq + a] =
            (4 * rq + a < B && 4 * cq + b < jn) ? __builtin_amdgcn_exp2f(dd[a][b] * scale) : 0.f;
    __syncthreads();
    for (int q = 0; q < jn; ++q) {
      const f32x4 k4 = *reinterpret_cast<const f32x4*>(&kT[q][4 * rq]);
      const f32x4 x4 = *reinterpret_cast<const f32x4*>(&xj[q][4 * cq]);
      const f32x4 s4 = *reinterpret_cast<const f32x4*>(&sj[q][4 * cq]);
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[a][c] = fmaf(k4[a], fmaf(g, xr[a][c] - x4[c], s4[c]), acc[a][c]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int i = 4 * rq + a, col = 4 * cq + c;
      if (i < B && col < d) part[((int64_t)blockIdx.x * B + i) * d + col] = tot[a][c] + acc[a][c];
    }
}

// The block's rows in order, one workgroup.  LDS: the block's old rows and
// scores, the moved rows and refreshed scores, k(x_i, x_j) of the old pairs
// (all at the start), P (the partials summed in slice order).
// score_kind: 0 scores frozen (exchanged scores, or the caller refreshes),
// 1 Gaussian s = scale * (-lam (x - mu)), 2 the 1-D two-component mixture of
// experiments/gmm.py per coordinate (csrc/prep.hip score_gmm_kernel).
constexpr int kGsLd = kGsMaxD + 1;  // row pitch: lanes reading one column of many rows spread over banks

__device__ __forceinline__ float gs_score(int kind, float x, float mu, float lam, float sc) {
  if (kind == 1) return sc * (-lam * (x - mu));
  const float a = -0.5f * (x + 2.f) * (x + 2.f), b = -0.5f * (x - 2.f) * (x - 2.f);
  const float m = fmaxf(a, b);
  const float ea = __expf(a - m), eb = __expf(b - m);
  return sc * (-(ea * (x + 2.f) + eb * (x - 2.f)) / (ea + eb));
}

__global__ __launch_bounds__(256) void gs_sweep_kernel(
    float* __restrict__ X, int64_t ldx, float* __restrict__ S, int64_t lds, int64_t n, int d,
    int64_t r0, int B, const dsvgd_select_state* __restrict__ st, float step,
    const float* __restrict__ part, int nsplit, const float* __restrict__ extra, int64_t lde,
    float* __restrict__ phi_out, int64_t ldphi, int score_kind, const float* __restrict__ mu,
    const float* __restrict__ lam, float score_scale) {
  __shared__ float xo[kGsB][kGsLd], so[kGsB][kGsLd], xn[kGsB][kGsLd], sn[kGsB][kGsLd];
  __shared__ float P[kGsB][kGsMaxD];
  __shared__ float ko[kGsB][kGsB + 1];  // k(x_i, x_j), both as the block starts
  __shared__ float kn[kGsB];            // k(x_i, x_j') of the row in progress
  __shared__ float red[4][kGsMaxD];
  const int t = threadIdx.x;
  const float inv_h = st->inv_h, g = 2.f * inv_h, scale = -inv_h * kLog2e;
  const float inv_n = 1.f / (float)n;
  for (int e = t; e < B * d; e += 256) {
    const int i = e / d, c = e % d;
    xo[i][c] = X[(r0 + i) * ldx + c];
    so[i][c] = S[(r0 + i) * lds + c];
    float p = 0.f;
    for (int z = 0; z < nsplit; ++z) p += part[((int64_t)z * B + i) * d + c];  // slice order
    P[i][c] = p;
  }
  __syncthreads();
  // k of the old pairs (j < i), exact differences
  for (int e = t; e < B * B; e += 256) {
    const int i = e / B, j = e % B;
    if (j >= i) continue;
    float s2 = 0.f;
    for (int c = 0; c < d; ++c) {
      const float df = xo[i][c] - xo[j][c];
      s2 = fmaf(df, df, s2);
    }
    ko[i][j] = __builtin_amdgcn_exp2f(s2 * scale);
  }
  __syncthreads();
  // distances: lane quad (j = t >> 2, quarter q4 = t & 3 of the columns);
  // accumulation: column cg = t % 64 of group gg = t / 64, over j = gg, gg + 4, ...
  const int jq = t >> 2, q4 = t & 3;
  const int dq = (d + 3) / 4;
  const int G = 256 / kGsMaxD;  // 4 groups of (up to) 64 columns
  const int cg = t % kGsMaxD, gg = t / kGsMaxD;
  for (int i = 0; i < B; ++i) {
    // k(x_i, x_j') for the rows already moved in this block
    if (jq < i) {
      float s2 = 0.f;
      for (int c = q4 * dq; c < min(d, (q4 + 1) * dq); ++c) {
        const float df = xo[i][c] - xn[jq][c];
        s2 = fmaf(df, df, s2);
      }
      s2 += __shfl_xor(s2, 1, 64);
      s2 += __shfl_xor(s2, 2, 64);
      if (q4 == 0) kn[jq] = __builtin_amdgcn_exp2f(s2 * scale);
    }
    __syncthreads();
    // sum over j < i of t(x_i, x_j', s_j') - t(x_i, x_j, s_j), group gg: j = gg, gg + G, ...
    float a = 0.f;
    if (cg < d) {
      const float xi = xo[i][cg];
      for (int j = gg; j < i; j += G)
        a += kn[j] * fmaf(g, xi - xn[j][cg], sn[j][cg]) - ko[i][j] * fmaf(g, xi - xo[j][cg], so[j][cg]);
    }
    red[gg][cg] = a;
    __syncthreads();
    if (t < d) {
      const float corr = ((red[0][t] + red[1][t]) + red[2][t]) + red[3][t];
      float p = inv_n * (P[i][t] + corr);
      if (extra) p += extra[(int64_t)i * lde + t];
      if (phi_out) phi_out[(int64_t)i * ldphi + t] = p;
      const float x = xo[i][t] + step * p;
      xn[i][t] = x;
      X[(r0 + i) * ldx + t] = x;
      float s = so[i][t];
      if (score_kind != 0) {
        s = gs_score(score_kind, x, mu ? mu[t] : 0.f, lam ? lam[t] : 0.f, score_scale);
        S[(r0 + i) * lds + t] = s;
      }
      sn[i][t] = s;
    }
    __syncthreads();
  }
}

}  // namespace dsvgd

using namespace dsvgd;

extern "C" {

int64_t dsvgd_gs_block_rows(void) { return kGsB; }

int64_t dsvgd_gs_splits(int64_t n) {
  // about 512 workgroups over the j range, at least 64 rows each
  const int64_t s = std::min<int64_t>(512, (n + 63) / 64);
  return s < 1 ? 1 : s;
}

int dsvgd_gs_block_part(const float* X, int64_t ldx, const float* S, int64_t lds, int64_t n,
                        int64_t d, int64_t r0, int64_t B, const dsvgd_select_state* st,
                        float* partial, int64_t nsplit, void* stream) {
  DSVGD_REQUIRE(X && S && st && partial, "null pointer");
  DSVGD_REQUIRE(n > 0 && d > 0 && d <= kGsMaxD && ldx >= d && lds >= d, "sizes (d <= 64)");
  DSVGD_REQUIRE(B > 0 && B <= kGsB && r0 >= 0 && r0 + B <= n, "block rows");
  DSVGD_REQUIRE(nsplit >= 1 && nsplit <= 65535, "nsplit");
  const int64_t jchunk = roundup((n + nsplit - 1) / nsplit, 64);
  hipLaunchKernelGGL(gs_part_kernel, dim3((unsigned)nsplit), dim3(256), 0, (hipStream_t)stream, X,
                     ldx, S, lds, n, (int)d, r0, (int)B, st, jchunk, partial);
  return check_launch("gs_part");
}

int dsvgd_gs_block_sweep(float* X, int64_t ldx, float* S, int64_t lds, int64_t n, int64_t d,
                         int64_t r0, int64_t B, const dsvgd_select_state* st, float step,
                         const float* partial, int64_t nsplit, const float* extra, int64_t lde,
                         float* phi_out, int64_t ldphi, int score_kind, const float* mu,
                         const float* lam, float score_scale, void* stream) {
  DSVGD_REQUIRE(X && S && st && partial, "null pointer");
  DSVGD_REQUIRE(n > 0 && d > 0 && d <= kGsMaxD && ldx >= d && lds >= d, "sizes (d <= 64)");
  DSVGD_REQUIRE(B > 0 && B <= kGsB && r0 >= 0 && r0 + B <= n, "block rows");
  DSVGD_REQUIRE(nsplit >= 1, "nsplit");
  DSVGD_REQUIRE(score_kind >= 0 && score_kind <= 2, "score_kind must be 0, 1 or 2");
  DSVGD_REQUIRE(score_kind != 1 || (mu && lam), "Gaussian scores need mu and lam");
  DSVGD_REQUIRE(!extra || lde >= d, "lde");
  DSVGD_REQUIRE(!phi_out || ldphi >= d, "ldphi");
  hipLaunchKernelGGL(gs_sweep_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, X, ldx, S, lds,
                     n, (int)d, r0, (int)B, st, step, partial, (int)nsplit, extra, lde, phi_out,
                     ldphi, score_kind, mu, lam, score_scale);
  return check_launch("gs_sweep");
}

}  // extern "C"
