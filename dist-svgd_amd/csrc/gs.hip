// gs.hip -- the reference's Gauss-Seidel sweep (dsvgd/sampler.py:64-68,
// dsvgd/distsampler.py:194-200) in blocks of kGsB rows.
//
// Row i of a sweep moves with phi_i computed from the CURRENT particles:
// rows before i already moved, rows from i on not yet.  For a block of rows
// [r0, r0 + B):
//
//   Q_i  = sum_{j outside [r0, r0 + i)} t(x_i, x_j, s_j)   (as the block starts)
//   phi_i = (Q_i + sum_{r0 <= j < r0 + i} t(x_i, x_j', s_j')) / n
//
// t(x, y, s) = k(x, y) (s + (2/h)(x - y)), k = exp(-|x - y|^2 / h), x_j' / s_j'
// the moved particle and its refreshed score.  Q for the whole block is one
// wide pass over all n rows (gs_part_kernel: every CU busy, exact
// differences, split-J partials, the block's own earlier rows masked out)
// plus a slice reduction (gs_reduce_kernel, fixed order); only the sums over
// the rows moved in this block are sequential (gs_sweep_kernel: ONE wave walks
// the B rows -- lane j for the distances to the moved rows, lane c for the
// columns -- with no barrier between rows: one wave's LDS accesses execute in
// order).  The score refresh of a moved particle (the reference re-evaluates
// logp per pair, so later rows see it) is fused for the elementwise targets.
// Same terms as the per-row path (dsvgd_phi_row_split), in a different
// summation order.
#include <algorithm>
#include <cmath>

#include "common.hpp"
#include "gemm_tiles.hpp"

namespace dsvgd {

constexpr int kGsB = 64;      // rows per block
// few slices (small n, small d): the sweep sums them itself (one launch less
// per block); otherwise gs_reduce_kernel does, over many workgroups
constexpr int64_t kGsFoldMax = 16384;  // B d nsplit values summed in the sweep
__host__ __device__ inline bool gs_fold(int64_t B, int64_t d, int64_t nsplit) {
  return B * d * nsplit <= kGsFoldMax;
}
constexpr int kGsMaxD = 64;   // features (one thread column group of 4 per 4 features)
constexpr int64_t kGsChain = 4096;

// part[z][i][c] = sum_{j in [z J, (z+1) J), j outside [r0, r0 + i)}
// t(x_{r0+i}, x_j, s_j)[c] (raw sums, not / n), i < B, c < d.  Block z: the B x d outputs as 64 x 64,
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
    // pairs with the block's own earlier rows (r0 <= j < r0 + i) are left to
    // the sweep, which uses the moved rows there
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int64_t jr = j0 + 4 * cq + b - r0;
        const bool moved = jr >= 0 && jr < 4 * rq + a;
        kT[4 * cq + b][4 * rq + a] = (4 * rq + a < B && 4 * cq + b < jn && !moved)
                                         ? __builtin_amdgcn_exp2f(dd[a][b] * scale)
                                         : 0.f;
      }
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

// Q = the slices of gs_part summed in slice order (z = w, w + 4, ... per
// wave, then the four wave sums in a fixed tree), written over slice 0.
// Element e = 64 blockIdx.x + lane; each element is read and written by one
// workgroup only, so the in-place write after the barrier is safe.
__global__ __launch_bounds__(256) void gs_reduce_kernel(float* __restrict__ part, int64_t elems,
                                                        int nsplit) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t e = (int64_t)blockIdx.x * 64 + lane;
  float s = 0.f;
  if (e < elems) {
    int z = w;
    for (; z + 28 < nsplit; z += 32) {  // 8 loads in flight
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(int64_t)(z + 4 * u) * elems + e];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; z < nsplit; z += 4) s += part[(int64_t)z * elems + e];
  }
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && e < elems) part[e] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

// The block's rows in order, by ONE wave (the other three only help load).
// LDS: the block's old rows, the moved rows and their scores, Q.  Per row i:
// lane j < i: k(x_i, x_j') (exact differences, 16-byte reads along the
// features); lane c: sum_{j < i} k_j (s_j' + g (x_i - x_j')) with k_j read
// from lane j (v_readlane), then phi_i, the move and the score refresh.
// score_kind: 0 scores frozen (exchanged scores, or the caller refreshes),
// 1 Gaussian s = scale * (-lam (x - mu)), 2 the 1-D two-component mixture of
// experiments/gmm.py per coordinate (csrc/prep.hip score_gmm_kernel).
constexpr int kGsLd = kGsMaxD + 4;  // row pitch (floats): 16-byte rows, 4 banks apart

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
    const float* __restrict__ Q, int nsum, const float* __restrict__ extra, int64_t lde,
    float* __restrict__ phi_out, int64_t ldphi, int score_kind, const float* __restrict__ mu,
    const float* __restrict__ lam, float score_scale) {
  // xo: old rows (zero past d, so the 16-byte distance reads need no mask)
  __shared__ __attribute__((aligned(16))) float xo[kGsB][kGsLd];
  __shared__ __attribute__((aligned(16))) float xn[kGsB][kGsLd];
  __shared__ float sn[kGsB][kGsLd];
  __shared__ float q[kGsB][kGsMaxD];
  const int t = threadIdx.x;
  const float inv_h = st->inv_h, g = 2.f * inv_h, scale = -inv_h * kLog2e;
  const float inv_n = 1.f / (float)n;
  for (int e = t; e < kGsB * kGsLd; e += 256) {
    const int i = e / kGsLd, c = e % kGsLd;
    const bool ok = i < B && c < d;
    xo[i][c] = ok ? X[(r0 + i) * ldx + c] : 0.f;
    xn[i][c] = 0.f;
    if (i < B && c < d) {
      float v = 0.f;
      for (int z = 0; z < nsum; ++z) v += Q[((int64_t)z * B + i) * d + c];  // slice order
      q[i][c] = v;
    }
  }
  __syncthreads();
  if (t >= 64) return;
  const int lane = t;
  const int d4 = (d + 3) >> 2;
  const float mu_c = (score_kind == 1 && lane < d) ? mu[lane] : 0.f;
  const float lam_c = (score_kind == 1 && lane < d) ? lam[lane] : 0.f;
  for (int i = 0; i < B; ++i) {
    // k(x_i, x_j') of the rows already moved: lane j
    // (both loops are LDS-latency chains: unrolled so the reads of several
    // iterations are in flight together, two partial sums each)
    float s2a = 0.f, s2b = 0.f;
#pragma unroll 4
    for (int c4 = 0; c4 < d4; ++c4) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(&xo[i][4 * c4]);
      const f32x4 b = *reinterpret_cast<const f32x4*>(&xn[lane][4 * c4]);
      const float d0 = a[0] - b[0], d1 = a[1] - b[1], d2 = a[2] - b[2], d3 = a[3] - b[3];
      s2a = fmaf(d0, d0, fmaf(d2, d2, s2a));
      s2b = fmaf(d1, d1, fmaf(d3, d3, s2b));
    }
    const float kj = lane < i ? __builtin_amdgcn_exp2f((s2a + s2b) * scale) : 0.f;
    // lane c: the moved rows' terms
    const int c = lane < d ? lane : 0;
    const float xi = xo[i][c];
    float acc0 = 0.f, acc1 = 0.f;
    int j = 0;
    for (; j + 8 <= i; j += 8) {
      float xv[8], sv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        xv[u] = xn[j + u][c];
        sv[u] = sn[j + u][c];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float k = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, kj), j + u));
        const float tv = k * fmaf(g, xi - xv[u], sv[u]);
        if (u & 1) acc1 += tv; else acc0 += tv;
      }
    }
    for (; j < i; ++j) {
      const float k = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, kj), j));
      acc0 = fmaf(k, fmaf(g, xi - xn[j][c], sn[j][c]), acc0);
    }
    const float acc = acc0 + acc1;
    if (lane < d) {
      float p = inv_n * (q[i][c] + acc);
      if (extra) p += extra[(int64_t)i * lde + c];
      if (phi_out) phi_out[(int64_t)i * ldphi + c] = p;
      const float x = xi + step * p;
      X[(r0 + i) * ldx + c] = x;
      float s = S[(r0 + i) * lds + c];
      if (score_kind != 0) {
        s = gs_score(score_kind, x, mu_c, lam_c, score_scale);
        S[(r0 + i) * lds + c] = s;
      }
      xn[i][c] = x;
      sn[i][c] = s;
    }
    // the next row reads row i's LDS writes: one wave's LDS accesses run in
    // order; keep the compiler from moving them
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

// ---- d > 64: the wide blocked sweep (engine.sequential_sweep) -----------
// The block's wide pass runs on the exact f32 MFMA engines of the Jacobi
// step (dsvgd_sqdist over the centred rows Y = [X - c | S], then
// dsvgd_phi_mm over all n columns with the block's own earlier rows masked
// to +inf here, then dsvgd_phi_partial_reduce): Q = [K Xc | K S] and r = K 1
// of the rows [r0, r0 + B) against every row not moved before them in the
// block.  The walk (gsw_sweep_kernel) then moves the B rows in order with one
// workgroup: per row the distances to the rows already moved (all 256
// threads, a quarter of the features each), their kernel values, and per
// column the moved rows' terms k_j w_j, w_j = s_j' - (2/h)(x_j' - c).  LDS
// holds the moved rows (centred x' and w) and the old row being moved, so B
// d <= kGswLds.
constexpr int kGswLds = 16384;   // floats per LDS array (64 KiB): B = min(64, kGswLds / dp)
constexpr int kGswLdsR = 10240;  // refreshed scores: three arrays (x', w, s') of 40 KiB
constexpr int kGswMaxD = 1024;

__host__ __device__ inline int gsw_rows(int64_t dp, bool refreshed) {
  const int64_t b = (refreshed ? kGswLdsR : kGswLds) / dp;
  return (int)(b >= kGsB ? kGsB : b);
}

// D[i][r0 + j] = +inf for j < i < B (panel layout, row i of the block's D):
// the pairs the walk takes with the moved rows
__global__ void gs_mask_kernel(float* __restrict__ D, int64_t ldd, int64_t r0, int B) {
  const int i = blockIdx.x;
  for (int j = threadIdx.x; j < i && i < B; j += blockDim.x) {
    const int64_t col = r0 + j;
    D[((int64_t)(i >> 7) * (ldd >> 4) + (col >> 4)) * kPanelElems + (i & 127) * 16 + (col & 15)] =
        INFINITY;
  }
}

// D[i][c0 + j] = +inf for i < B, j < nc: the pipelined wide sweep's pass of
// group g + 1 runs while group g walks, so it leaves group g's columns out
// (dsvgd_gsw_group_corr adds them at their moved positions afterwards)
__global__ void gs_mask_cols_kernel(float* __restrict__ D, int64_t ldd, int64_t c0, int64_t nc) {
  const int i = blockIdx.x;
  for (int64_t j = threadIdx.x; j < nc; j += blockDim.x) {
    const int64_t col = c0 + j;
    D[((int64_t)(i >> 7) * (ldd >> 4) + (col >> 4)) * kPanelElems + (i & 127) * 16 + (col & 15)] =
        INFINITY;
  }
}

// test hook: one wave holds the stream for ns nanoseconds (s_memrealtime:
// 100 MHz), so that work queued on another stream is in flight when the
// kernels behind it start (the pipelined sweep's forced-overlap test)
__global__ void debug_spin_kernel(int64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) < ticks) __builtin_amdgcn_s_sleep(8);
}

// The grouped wide sweep's correction: the wide pass of a group of blocks
// left every pair (i, j) with j < i inside the group out (dsvgd_gs_mask over
// the group), so once a block has walked, the group's later rows [r0, r0 +
// nr) (not moved yet) gain its pB rows [p0, p0 + pB) at their moved
// positions: Q = [K Xc | K S] += k_ij (x_j' - c | s_j'), Qr += k_ij, k_ij =
// exp(-|x_i - x_j'|^2 / h) by explicit differences (the walk's own form).
// One workgroup per row i: wave w forms k_ij for j = w, w + 4, ... (lanes
// over the features, a fixed butterfly), then thread t adds the j terms to
// columns t, t + 256, ... in j order (deterministic).
__global__ __launch_bounds__(256) void gsw_group_corr_kernel(
    const float* __restrict__ X, int64_t ldx, const float* __restrict__ S, int64_t lds,
    const float* __restrict__ center, int64_t d, int64_t dp, int64_t r0, int64_t p0, int pB,
    const dsvgd_select_state* __restrict__ st, float* __restrict__ Q, int64_t ldq,
    float* __restrict__ Qr) {
  __shared__ float xi[kGswMaxD];
  __shared__ float kv[2 * kGsB];   // up to two blocks of earlier rows (a group)
  const int i = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
  const float scale = -st->inv_h * kLog2e;
  for (int64_t c = t; c < d; c += 256) xi[c] = X[(r0 + i) * ldx + c];
  __syncthreads();
  if (d <= 256) {
    // the same sums in the same order with every load of a loop issued
    // before its first use (the general loops below wait on one L2 round
    // trip per moved row: 28 us per 64-row correction at config D, r13ag);
    // the earlier rows in halves of 64
    float xv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) xv[k] = lane + 64 * k < d ? xi[lane + 64 * k] : 0.f;
    for (int hb = 0; hb < pB; hb += kGsB) {
      float xr[16][4];
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) {
        const int j = hb + w + 4 * jj;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int c = lane + 64 * k;
          xr[jj][k] = (j < pB && c < d) ? X[(p0 + j) * ldx + c] : xv[k];
        }
      }
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) {
        const int j = hb + w + 4 * jj;
        float a = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float df = xv[k] - xr[jj][k];
          a = fmaf(df, df, a);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
        if (lane == 0 && j < pB) kv[j] = __builtin_amdgcn_exp2f(a * scale);
      }
    }
    __syncthreads();
    float* q = Q + (int64_t)i * ldq;
    const int c = t;
    if (c < d) {
      const float cc = center[c];
      float qx = 0.f, qs = 0.f;
      for (int hb = 0; hb < pB; hb += kGsB) {
        float xa[kGsB], sa[kGsB];
#pragma unroll
        for (int j = 0; j < kGsB; ++j) {
          xa[j] = hb + j < pB ? X[(p0 + hb + j) * ldx + c] : 0.f;
          sa[j] = hb + j < pB ? S[(p0 + hb + j) * lds + c] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < kGsB; ++j) {
          if (hb + j < pB) {   // (not break: the loop must unroll)
            const float k = kv[hb + j];
            qx = fmaf(k, xa[j] - cc, qx);
            qs = fmaf(k, sa[j], qs);
          }
        }
      }
      q[c] += qx;
      q[dp + c] += qs;
    }
    if (t == 0) {
      float r = 0.f;
      for (int j = 0; j < pB; ++j) r += kv[j];
      Qr[i] += r;
    }
    return;
  }
  for (int j = w; j < pB; j += 4) {
    const float* xj = X + (p0 + j) * ldx;
    float a = 0.f;
    for (int64_t c = lane; c < d; c += 64) {
      const float df = xi[c] - xj[c];
      a = fmaf(df, df, a);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
    if (lane == 0) kv[j] = __builtin_amdgcn_exp2f(a * scale);
  }
  __syncthreads();
  float* q = Q + (int64_t)i * ldq;
  for (int64_t c = t; c < d; c += 256) {
    const float cc = center[c];
    float qx = 0.f, qs = 0.f;
    for (int j = 0; j < pB; ++j) {
      const float k = kv[j];
      qx = fmaf(k, X[(p0 + j) * ldx + c] - cc, qx);
      qs = fmaf(k, S[(p0 + j) * lds + c], qs);
    }
    q[c] += qx;
    q[dp + c] += qs;
  }
  if (t == 0) {
    float r = 0.f;
    for (int j = 0; j < pB; ++j) r += kv[j];
    Qr[i] += r;
  }
}

// One workgroup of 256 threads walks rows [r0, r0 + B).  Q: [K Xc | K S] of
// the wide pass (ldq >= 2 dp), Qr its row sums; Y: [X - c | S] (rewritten for
// the moved rows, with norms[], at the block's end), centre c = the Y
// packing centre.
// Per row two barriers: (1) after the distance partials, (2) after the moved
// row's LDS writes.  Every wave forms the row's kernel values itself (lane j:
// k(x_i, x_j'), its moved-row sum by a wave reduction) and the column loop
// broadcasts them with v_readlane.  The next row's global operands (Q, Qr,
// its old x and s, the extra row) are loaded one row ahead into registers,
// and NO global store is issued inside the row loop (X, S, Y and the norms
// of the moved rows go out from LDS after it): vmcnt counts loads and stores
// in order, so a store of row i made the loop-head wait for row i + 1's
// operands also wait for it (~2.7 us per row, r11e).  phi_out (tests only) is
// the one in-loop store.
constexpr int kGswCols = kGswMaxD / 256;  // columns per thread
// LDS hand-offs only: wait for this wave's LDS operations, then s_barrier.
// No global location the walk writes is read inside it by another thread.
__device__ __forceinline__ void gsw_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

constexpr int kGswCoef = 4096;            // logreg refresh: the waves' partials [4][dp]

// The logistic regression score of the moved row x' (logreg_small_kernel's
// terms: s_0 = -a + p/2 - a/2 |w|^2, s_w = sum_q t_q sigma(-t_q xd_q . w) xd_q
// - a w, times scale) in ONE pass over the rank's nd data rows: every wave
// holds w in the dwordx4 lane layout (lane: w[256 v + 4 lane .. + 3]), takes
// R = 16 / NV rows per batch (one dwordx4 load per row and 256 features,
// the next batch in flight while this one is reduced: 32 loads per wave),
// forms z_q by an interleaved wave reduction, and adds t_q sigma(-t_q z_q)
// xd_q into register partials from the SAME loaded values; the four waves'
// partials meet in LDS.  A single workgroup streams the data at the rate
// its loads in flight allow (~128 KiB), so rows are 16-byte aligned
// (ldxd % 4 == 0, the caller's padded copy).
template <int NV>
__device__ __forceinline__ void gsw_logreg_refresh(
    const float* xr, float cla, const float (&cw)[kGswMaxD / 64], const float* __restrict__ xd,
    int64_t ldxd, const float* __restrict__ td, int nd, float* red, int dp, float scale, int d,
    float* snrow, float* wnrow, float g2, const float (&cen)[kGswCols]) {
  constexpr int R = 16 / NV;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int p = d - 1;
  const float a = expf(xr[0] + cla);
  float wv[NV][4], g[NV][4];
  float w2 = 0.f;
#pragma unroll
  for (int v = 0; v < NV; ++v)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = 256 * v + 4 * lane + k;
      wv[v][k] = c < p ? xr[1 + c] + cw[4 * v + k] : 0.f;
      w2 = fmaf(wv[v][k], wv[v][k], w2);
      g[v][k] = 0.f;
    }
  for (int o = 32; o > 0; o >>= 1) w2 += __shfl_xor(w2, o, 64);
  // wave w's batches: rows [4 R it + R w, + R), it = 0, 1, ...
  const int nb = (nd + 4 * R - 1) / (4 * R);
  f32x4 buf[2][R][NV];
  float tb[2][R];
  auto load = [&](f32x4 (&bb)[R][NV], float (&tt)[R], int it) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int q = min(4 * R * it + R * w + r, nd - 1);
      const float* xq = xd + (int64_t)q * ldxd + 4 * lane;
#pragma unroll
      for (int v = 0; v < NV; ++v)
        bb[r][v] = (256 * v + 4 * lane < p) ? *reinterpret_cast<const f32x4*>(xq + 256 * v)
                                            : f32x4{0.f, 0.f, 0.f, 0.f};
      tt[r] = td[q];
    }
  };
  auto use = [&](const f32x4 (&bb)[R][NV], const float (&tt)[R], int it) {
    float z[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        s0 = fmaf(bb[r][v][0], wv[v][0], fmaf(bb[r][v][2], wv[v][2], s0));
        s1 = fmaf(bb[r][v][1], wv[v][1], fmaf(bb[r][v][3], wv[v][3], s1));
      }
      z[r] = s0 + s1;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
#pragma unroll
      for (int r = 0; r < R; ++r) z[r] += __shfl_xor(z[r], o, 64);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const bool ok = 4 * R * it + R * w + r < nd;
      const float cf = ok ? tt[r] / (1.f + expf(tt[r] * z[r])) : 0.f;
#pragma unroll
      for (int v = 0; v < NV; ++v)
#pragma unroll
        for (int k = 0; k < 4; ++k) g[v][k] = fmaf(cf, bb[r][v][k], g[v][k]);
    }
  };
  if (nb > 0) load(buf[0], tb[0], 0);
  for (int it = 0; it < nb; it += 2) {
    if (it + 1 < nb) load(buf[1], tb[1], it + 1);
    use(buf[0], tb[0], it);
    if (it + 1 >= nb) break;
    if (it + 2 < nb) load(buf[0], tb[0], it + 2);
    use(buf[1], tb[1], it + 1);
  }
#pragma unroll
  for (int v = 0; v < NV; ++v)
    if (256 * v + 4 * lane < p)
      *reinterpret_cast<f32x4*>(red + w * dp + 256 * v + 4 * lane) =
          f32x4{g[v][0], g[v][1], g[v][2], g[v][3]};
  gsw_barrier();
#pragma unroll
  for (int u = 0; u < kGswCols; ++u) {
    const int c = t + 256 * u;
    if (c >= d) continue;
    float sv;
    if (c == 0) {
      sv = scale * (-a + 0.5f * (float)p - 0.5f * a * w2);
    } else {
      const float gs = (red[c - 1] + red[dp + c - 1]) + (red[2 * dp + c - 1] + red[3 * dp + c - 1]);
      sv = scale * (gs - a * (xr[c] + cen[u]));
    }
    snrow[c] = sv;
    wnrow[c] = sv - g2 * xr[c];
  }
}


template <bool LOGREG>  // score_kind 3 (its refresh's registers stay out of the others' walk)
__global__ __launch_bounds__(256) void gsw_sweep_kernel(
    float* __restrict__ X, int64_t ldx, float* __restrict__ S, int64_t lds, float* __restrict__ Y,
    int64_t ldy, float* __restrict__ norms, const float* __restrict__ center, int64_t n, int d,
    int dp, int64_t r0, int B, const dsvgd_select_state* __restrict__ st, float step,
    const float* __restrict__ Q, int64_t ldq, const float* __restrict__ Qr,
    const float* __restrict__ extra, int64_t lde, float* __restrict__ phi_out, int64_t ldphi,
    int score_kind, const float* __restrict__ mu, const float* __restrict__ lam,
    float score_scale, const float* __restrict__ xd, int64_t ldxd, const float* __restrict__ td,
    int nd, int dbg) {
  extern __shared__ __attribute__((aligned(16))) float gsw_smem[];
  const bool refreshed = score_kind != 0;
  const int pitch = dp + 4;                       // 16-byte rows, 4 banks apart
  // xn row j: the old row (centred) until row j moves, then the moved one
  float* xn = gsw_smem;                           // [B][pitch]
  float* wn = xn + (int64_t)B * pitch;            // [B][dp]: w_j = s_j' - g (x_j' - c)
  float* sn = wn + (int64_t)B * dp;               // [B][dp]: their scores (refreshed only)
  float* part = sn + (refreshed ? (int64_t)B * dp : 0);  // [4][64] partial distances
  float* red = part + 256;                        // [js][dp] the column loop's j-group sums
  float* redr = red + 1024;                       // [js] their kernel sums
  float* coef = redr + 16;                        // [kGswCoef] logreg: the waves' partials
  // dp % 256 == 0: the column loop over f32x4 column quads, the moved rows
  // split over js = 1024 / dp wave groups (wave-uniform j: v_readlane)
  const int nq = dp >> 2;
  const bool quad = (dp & 255) == 0;
  const int js = quad ? 1024 / dp : 1;
  const int qd = (int)threadIdx.x % nq, jq = (int)threadIdx.x / nq;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const float inv_h = st->inv_h, g = 2.f * inv_h, scale = -inv_h * kLog2e;
  const float inv_n = 1.f / (float)n;
  const int q4 = dp >> 2;                         // features per quarter (dp % 32 == 0)
  // the block's old rows (Y's centred half, zero past d) into xn: the walk's
  // only global loads are then the next row's operands, one row ahead
  for (int e = t; e < B * (dp >> 2); e += 256) {
    const int i = e / (dp >> 2), c4 = (e % (dp >> 2)) << 2;
    *reinterpret_cast<f32x4*>(xn + i * pitch + c4) =
        *reinterpret_cast<const f32x4*>(Y + (r0 + i) * ldy + c4);
  }
  // per-thread columns c = t + 256 u, u < kGswCols, and the next row's operands
  float cen[kGswCols], mu_c[kGswCols], lam_c[kGswCols];
  float nq_x[kGswCols], nq_s[kGswCols], n_so[kGswCols], n_ex[kGswCols];
  float nqr = 0.f;
  auto prefetch = [&](int i) {  // row i's operands (i < B)
    const int64_t gi = r0 + i;
#pragma unroll
    for (int u = 0; u < kGswCols; ++u) {
      const int c = t + 256 * u;
      const bool ok = c < d;
      nq_x[u] = ok ? Q[i * ldq + c] : 0.f;
      nq_s[u] = ok ? Q[i * ldq + dp + c] : 0.f;
      n_so[u] = ok ? Y[gi * ldy + dp + c] : 0.f;
      n_ex[u] = (ok && extra) ? extra[(int64_t)i * lde + c] : 0.f;
    }
    nqr = Qr[i];
  };
#pragma unroll
  for (int u = 0; u < kGswCols; ++u) {
    const int c = t + 256 * u;
    cen[u] = c < d ? center[c] : 0.f;
    mu_c[u] = (score_kind == 1 && c < d) ? mu[c] : 0.f;
    lam_c[u] = (score_kind == 1 && c < d) ? lam[c] : 0.f;
  }
  // logreg (score_kind 3): the centre of log alpha and of this lane's
  // weights w[c], c = 256 v + 4 lane + k
  const float cla = LOGREG ? center[0] : 0.f;
  float cw[kGswMaxD / 64];   // w[256 v + 4 lane + k] at cw[4 v + k]
#pragma unroll
  for (int v = 0; v < kGswMaxD / 256; ++v)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = 256 * v + 4 * lane + k;
      cw[4 * v + k] = (LOGREG && c + 1 < d) ? center[1 + c] : 0.f;
    }
  prefetch(0);
  __syncthreads();
  for (int i = 0; i < B; ++i) {
    float q_x[kGswCols], q_s[kGswCols], s_o[kGswCols], ex[kGswCols];
#pragma unroll
    for (int u = 0; u < kGswCols; ++u) {
      q_x[u] = nq_x[u];
      q_s[u] = nq_s[u];
      s_o[u] = n_so[u];
      ex[u] = n_ex[u];
    }
    const float qr = nqr;
    if (i + 1 < B && !(dbg & 1)) prefetch(i + 1);
    const float* xoi = xn + i * pitch;   // row i, still the old one
    // (a) distances of the old row i to the moved rows j < i: thread (j =
    // lane, quarter w) over features [w q4, (w + 1) q4)
    {
      float sa = 0.f, sb = 0.f;
      if (lane < i && !(dbg & 2)) {
        const float* pa = xoi + w * q4;
        const float* pb = xn + lane * pitch + w * q4;
        auto acc4 = [&](const f32x4& va, const f32x4& vb) {
          const float d0 = va[0] - vb[0], d1 = va[1] - vb[1], d2 = va[2] - vb[2], d3 = va[3] - vb[3];
          sa = fmaf(d0, d0, fmaf(d2, d2, sa));
          sb = fmaf(d1, d1, fmaf(d3, d3, sb));
        };
        int c = 0;
        for (; c + 16 <= q4; c += 16) {  // eight 16-byte LDS reads in flight
          f32x4 va[4], vb[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            va[r] = *reinterpret_cast<const f32x4*>(pa + c + 4 * r);
            vb[r] = *reinterpret_cast<const f32x4*>(pb + c + 4 * r);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) acc4(va[r], vb[r]);
        }
        for (; c < q4; c += 4)
          acc4(*reinterpret_cast<const f32x4*>(pa + c), *reinterpret_cast<const f32x4*>(pb + c));
      }
      part[w * 64 + lane] = sa + sb;
    }
    gsw_barrier();                                                          // (1)
    // every wave: lane j's k(x_i, x_j') and the moved rows' kernel sum
    const float dd = (part[lane] + part[64 + lane]) + (part[128 + lane] + part[192 + lane]);
    const int kb = __builtin_bit_cast(int, lane < i ? __builtin_amdgcn_exp2f(dd * scale) : 0.f);
    float rm = 0.f;   // sum_{j<i} k_j, summed along the column loop's broadcasts
    // (b) per column: sum_{j<i} k_j w_j (k_j broadcast by v_readlane), eight
    // moved rows' LDS reads in flight at a time
    float acc[kGswCols][2];
#pragma unroll
    for (int u = 0; u < kGswCols; ++u) acc[u][0] = acc[u][1] = 0.f;
    const int iw = (dbg & 4) ? 0 : i;   // (timing probe: no column loop)
    if (quad) {
      // thread (quad qd, group jq): sum_{j = jq mod js, j < i} k_j w_j[4 qd .. +3]
      f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
      float rp = 0.f;
      if (jq < js) {
        const float* wq = wn + 4 * qd;
        int j = jq;
        for (; j + 7 * js < iw; j += 8 * js) {
          float kk[8];
          f32x4 wv8[8];
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            kk[r] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(kb, j + r * js));
            wv8[r] = *reinterpret_cast<const f32x4*>(wq + (j + r * js) * dp);
          }
          rp += ((kk[0] + kk[1]) + (kk[2] + kk[3])) + ((kk[4] + kk[5]) + (kk[6] + kk[7]));
#pragma unroll
          for (int r = 0; r < 8; r += 2) {
            a0 += kk[r] * wv8[r];
            a1 += kk[r + 1] * wv8[r + 1];
          }
        }
        for (; j < iw; j += js) {
          const float k0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(kb, j));
          rp += k0;
          a0 += k0 * *reinterpret_cast<const f32x4*>(wq + j * dp);
        }
        *reinterpret_cast<f32x4*>(red + jq * dp + 4 * qd) = a0 + a1;
        if (qd == 0) redr[jq] = rp;
      }
      gsw_barrier();                                                        // (1b)
#pragma unroll
      for (int u = 0; u < kGswCols; ++u) {
        const int c = t + 256 * u;
        if (c >= d) continue;
        float sacc = 0.f;
        for (int q = 0; q < js; ++q) sacc += red[q * dp + c];
        acc[u][0] = sacc;
      }
      for (int q = 0; q < js; ++q) rm += redr[q];
    } else {
    int j = 0;
    for (; j + 8 <= iw; j += 8) {
      float kk[8];
#pragma unroll
      for (int r = 0; r < 8; ++r)
        kk[r] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(kb, j + r));
      rm += ((kk[0] + kk[1]) + (kk[2] + kk[3])) + ((kk[4] + kk[5]) + (kk[6] + kk[7]));
#pragma unroll
      for (int u = 0; u < kGswCols; ++u) {
        const int c = t + 256 * u;
        if (256 * u >= d) break;   // (uniform) no column of this u anywhere
        if (c >= d) continue;
        float wv8[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) wv8[r] = wn[(j + r) * dp + c];
#pragma unroll
        for (int r = 0; r < 8; ++r) acc[u][r & 1] = fmaf(kk[r], wv8[r], acc[u][r & 1]);
      }
    }
    for (; j < iw; ++j) {
      const float k0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(kb, j));
      rm += k0;
#pragma unroll
      for (int u = 0; u < kGswCols; ++u) {
        const int c = t + 256 * u;
        if (256 * u >= d) break;
        if (c >= d) continue;
        acc[u][0] = fmaf(k0, wn[j * dp + c], acc[u][0]);
      }
    }
    }
    float xc_o[kGswCols];   // row i's old values (this thread's columns)
#pragma unroll
    for (int u = 0; u < kGswCols; ++u) {
      const int c = t + 256 * u;
      xc_o[u] = c < d ? xoi[c] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kGswCols; ++u) {
      const int c = t + 256 * u;
      if (c >= d) continue;
      // sum_{j<i} k_j (s_j' + g (x_i - x_j')) = sum k_j w_j + g x_i sum k_j
      // (centred); + the self term s_i (the wide pass skipped the diagonal)
      // + the wide pass's terms
      const float rtot = qr + rm;
      float p = inv_n * (((q_s[u] + s_o[u]) - g * q_x[u]) + (acc[u][0] + acc[u][1]) +
                         g * (rtot * xc_o[u]));
      p += ex[u];
      if (phi_out) phi_out[(int64_t)i * ldphi + c] = p;
      const float x = (xc_o[u] + cen[u]) + step * p;
      const float xc = x - cen[u];
      xn[i * pitch + c] = xc;
      if (!LOGREG) {
        float sv = s_o[u];
        if (score_kind == 1 || score_kind == 2) {
          sv = gs_score(score_kind, x, mu_c[u], lam_c[u], score_scale);
          sn[i * dp + c] = sv;
        }
        wn[i * dp + c] = sv - g * xc;
      }
    }
    gsw_barrier();                                                          // (2)
    if (LOGREG) {
      // the moved row's logreg score on the rank's data, in one pass over it
      const float* xr = xn + i * pitch;
      const int nv4 = (d - 1 + 255) >> 8;   // 256-feature groups (1 .. 4)
      if (nv4 == 1)
        gsw_logreg_refresh<1>(xr, cla, cw, xd, ldxd, td, nd, coef, dp, score_scale, d,
                              sn + i * dp, wn + i * dp, g, cen);
      else if (nv4 == 2)
        gsw_logreg_refresh<2>(xr, cla, cw, xd, ldxd, td, nd, coef, dp, score_scale, d,
                              sn + i * dp, wn + i * dp, g, cen);
      else if (nv4 == 3)
        gsw_logreg_refresh<3>(xr, cla, cw, xd, ldxd, td, nd, coef, dp, score_scale, d,
                              sn + i * dp, wn + i * dp, g, cen);
      else
        gsw_logreg_refresh<4>(xr, cla, cw, xd, ldxd, td, nd, coef, dp, score_scale, d,
                              sn + i * dp, wn + i * dp, g, cen);
      // sn[i] / wn[i] are read after the next row's barrier (1); the
      // partials' LDS is rewritten only after it
    }
  }
  // the moved rows out: X (= the centred row + c), Y's row x' - c and its
  // norm |x' - c|^2 (the later blocks' distances), and with refreshed scores
  // S and Y's score half (frozen scores: both unchanged)
  for (int i = 0; i < B; ++i) {
    const int64_t gi = r0 + i;
#pragma unroll
    for (int u = 0; u < kGswCols; ++u) {
      const int c = t + 256 * u;
      if (c >= d) continue;
      const float xc = xn[i * pitch + c];
      X[gi * ldx + c] = xc + cen[u];
      Y[gi * ldy + c] = xc;
      if (refreshed) {
        const float sv = sn[i * dp + c];
        S[gi * lds + c] = sv;
        Y[gi * ldy + dp + c] = sv;
      }
    }
  }
  {  // norms: four threads per row, a quarter of the features each (zero past d)
    const int i = t >> 2, qq = t & 3;
    float s2a = 0.f, s2b = 0.f;
    if (i < B) {
      const float* pr = xn + i * pitch + qq * q4;
      for (int c = 0; c < q4; c += 4) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(pr + c);
        s2a = fmaf(v[0], v[0], fmaf(v[2], v[2], s2a));
        s2b = fmaf(v[1], v[1], fmaf(v[3], v[3], s2b));
      }
    }
    float s2 = s2a + s2b;
    s2 += __shfl_xor(s2, 1, 64);
    s2 += __shfl_xor(s2, 2, 64);
    if (i < B && qq == 0) norms[r0 + i] = s2;
  }
}

// ---- the incremental walk (dp <= 256, elementwise or frozen scores) -------
// The same terms as gsw_sweep_kernel with the work per row moved OFF the
// row-to-row path: when row j moves, every later row i of the block gets its
// pair term at once -- k_ij = k(x_i, x_j') (x_i still the old row) into its
// row sum, and k_ij w_j into its column accumulators -- so row i's phi is
// ready when its turn comes (no distance phase, no column loop of its own).
// Per row two barriers:
//   A  thread c (column c): phi_j[c] from the wide pass's Q, the row's own
//      accumulator and row sum, the move, w_j[c] = s_j'[c] - g (x_j'[c] - cen);
//      the moved row into LDS;                                        (1)
//   B  wave w, lane (r, q): row i = 16 w + r, features [64 q, 64 q + 64) of
//      the old row in registers against the moved row from LDS, summed over
//      the quad (DPP); k_ij for i > j into LDS at slot i - j - 1, the row sum
//      r_i += k_ij;                                                   (2)
//   C  thread c: acc[m] = acc[m + 1] + k_{j+1+m, j} w_j[c], m = 0 .. 62 --
//      accumulator m belongs to row j + 1 + m, so the next row's is acc[0]
//      (static register indices, no select chain).
// Sums run over j in order (acc, r) and over the features in a fixed
// order; the results differ from the four-wave walk's in rounding only.
constexpr int kGsiMaxDp = 256;
// CPT columns per thread (roundup(d, 32) <= 256 CPT): phase B's rows get 4 CPT
// lanes of 64 features each, so a wave holds 16 / CPT rows and a block at
// most 64 / CPT (the host falls back to the four-wave walk above that).
template <int CPT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gsw_inc_kernel(
    float* __restrict__ X, int64_t ldx, float* __restrict__ S, int64_t lds, float* __restrict__ Y,
    int64_t ldy, float* __restrict__ norms, const float* __restrict__ center, int64_t n, int d,
    int dp, int64_t r0, int B, const dsvgd_select_state* __restrict__ st, float step,
    const float* __restrict__ Q, int64_t ldq, const float* __restrict__ Qr,
    const float* __restrict__ extra, int64_t lde, float* __restrict__ phi_out, int64_t ldphi,
    int score_kind, const float* __restrict__ mu, const float* __restrict__ lam,
    float score_scale) {
  constexpr int DPW = kGsiMaxDp * CPT;            // features a row carries in LDS
  constexpr int LPR = 4 * CPT;                    // phase B lanes per row
  constexpr int RPW = 64 / LPR;                   // rows per wave
  constexpr int BMAX = 4 * RPW;                   // rows per block
  extern __shared__ __attribute__((aligned(16))) float gsw_smem[];
  const bool refreshed = score_kind != 0;
  const int pitch = DPW + 4;                      // zero past dp: phase B reads DPW features
  float* xn = gsw_smem;                           // [B][pitch]: old rows, moved ones once moved
  float* sn = xn + (int64_t)B * pitch;            // [B][dp] refreshed scores
  float* kb = sn + (refreshed ? (int64_t)B * dp : 0);  // [64] k_{j+1+m, j}
  float* rb = kb + 64;                            // [64] row sums over the moved rows
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int rr = lane / LPR, qq = lane % LPR;     // phase B: row RPW w + rr, features 64 qq ..
  const int ib = RPW * w + rr;
  const float inv_h = st->inv_h, g = 2.f * inv_h, scale = -inv_h * kLog2e;
  const float inv_n = 1.f / (float)n;
  for (int e = t; e < B * (DPW >> 2); e += 256) {
    const int i = e / (DPW >> 2), c4 = (e % (DPW >> 2)) << 2;
    *reinterpret_cast<f32x4*>(xn + i * pitch + c4) =
        c4 < dp ? *reinterpret_cast<const f32x4*>(Y + (r0 + i) * ldy + c4)
                : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if (t < 64) rb[t] = 0.f;
  // phase B's old row in registers (zero past dp and for rows >= B)
  f32x4 xo[16];
#pragma unroll
  for (int f = 0; f < 16; ++f) {
    const int cc = 64 * qq + 4 * f;
    xo[f] = (ib < B && cc < dp) ? *reinterpret_cast<const f32x4*>(Y + (r0 + ib) * ldy + cc)
                                : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  // phase A / C columns c = t + 256 u
  float cen[CPT], mu_c[CPT], lam_c[CPT];
#pragma unroll
  for (int u = 0; u < CPT; ++u) {
    const int c = t + 256 * u;
    cen[u] = c < d ? center[c] : 0.f;
    mu_c[u] = (score_kind == 1 && c < d) ? mu[c] : 0.f;
    lam_c[u] = (score_kind == 1 && c < d) ? lam[c] : 0.f;
  }
  float nq_x[CPT], nq_s[CPT], n_so[CPT], n_ex[CPT], nqr = 0.f;
  auto prefetch = [&](int i) {
    const int64_t gi = r0 + i;
#pragma unroll
    for (int u = 0; u < CPT; ++u) {
      const int c = t + 256 * u;
      const bool ok = c < d;
      nq_x[u] = ok ? Q[i * ldq + c] : 0.f;
      nq_s[u] = ok ? Q[i * ldq + dp + c] : 0.f;
      n_so[u] = ok ? Y[gi * ldy + dp + c] : 0.f;
      n_ex[u] = (ok && extra) ? extra[(int64_t)i * lde + c] : 0.f;
    }
    nqr = Qr[i];
  };
  float acc[BMAX][CPT];
#pragma unroll
  for (int m = 0; m < BMAX; ++m)
#pragma unroll
    for (int u = 0; u < CPT; ++u) acc[m][u] = 0.f;
  float rsum = 0.f;   // phase B lanes: row ib's sum over the moved rows
  prefetch(0);
  __syncthreads();
  for (int j = 0; j < B; ++j) {
    // ---- A: row j's phi and move (columns t + 256 u) ----
    float q_x[CPT], q_s[CPT], s_o[CPT], ex[CPT];
#pragma unroll
    for (int u = 0; u < CPT; ++u) {
      q_x[u] = nq_x[u];
      q_s[u] = nq_s[u];
      s_o[u] = n_so[u];
      ex[u] = n_ex[u];
    }
    const float qr = nqr;
    if (j + 1 < B) prefetch(j + 1);
    const float rj = rb[j];
    float wj[CPT];
#pragma unroll
    for (int u = 0; u < CPT; ++u) {
      const int c = t + 256 * u;
      const float xc_o = xn[j * pitch + c];   // (zero past dp)
      wj[u] = 0.f;
      if (c < d) {
        float p = inv_n * (((q_s[u] + s_o[u]) - g * q_x[u]) + acc[0][u] + g * ((qr + rj) * xc_o));
        p += ex[u];
        if (phi_out) phi_out[(int64_t)j * ldphi + c] = p;
        const float x = (xc_o + cen[u]) + step * p;
        const float xc = x - cen[u];
        xn[j * pitch + c] = xc;
        float sv = s_o[u];
        if (score_kind == 1 || score_kind == 2) {
          sv = gs_score(score_kind, x, mu_c[u], lam_c[u], score_scale);
          sn[j * dp + c] = sv;
        }
        wj[u] = sv - g * xc;
      }
    }
    gsw_barrier();                                                          // (1)
    // ---- B: k(x_i, x_j') for the later rows i of this wave ----
    {
      const float* pm = xn + j * pitch + 64 * qq;   // (zero past dp: pitch covers DPW)
      // feature pairs on the packed fp32 VALU, one v_pk_add + one v_pk_fma per
      // two features (inline: the compiler's own packing added a v_mov per value)
      f32x2 da = {0.f, 0.f}, dbv = {0.f, 0.f};
#pragma unroll
      for (int f = 0; f < 16; ++f) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(pm + 4 * f);
        const f32x2 x01 = {xo[f][0], xo[f][1]}, x23 = {xo[f][2], xo[f][3]};
        const f32x2 v01 = {v[0], v[1]}, v23 = {v[2], v[3]};
        f32x2 d01, d23;
        asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(d01) : "v"(x01), "v"(v01));
        asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(d23) : "v"(x23), "v"(v23));
        asm("v_pk_fma_f32 %0, %1, %1, %0" : "+v"(da) : "v"(d01));
        asm("v_pk_fma_f32 %0, %1, %1, %0" : "+v"(dbv) : "v"(d23));
      }
      float dd = (da.x + dbv.x) + (da.y + dbv.y);
      // the row's LPR lanes summed (every lane ends with the total)
      if constexpr (LPR == 16) {   // one DPP row: rotations by 8, then 4
        dd += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                                            0, __builtin_bit_cast(int, dd), 0x128, 0xF, 0xF, false));
        dd += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                                            0, __builtin_bit_cast(int, dd), 0x124, 0xF, 0xF, false));
      } else if constexpr (LPR == 8) {
        dd += __shfl_xor(dd, 4, 64);
      }
      dd += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                                          0, __builtin_bit_cast(int, dd), 0xB1, 0xF, 0xF, false));
      dd += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                                          0, __builtin_bit_cast(int, dd), 0x4E, 0xF, 0xF, false));
      const bool later = ib > j && ib < B;
      const float k = later ? __builtin_amdgcn_exp2f(dd * scale) : 0.f;
      rsum += k;
      if (qq == 0 && ib > j) {
        kb[ib - j - 1] = k;
        rb[ib] = rsum;
      }
    }
    gsw_barrier();                                                          // (2)
    // ---- C: the later rows' accumulators gain k_ij w_j, shifted by one ----
#pragma unroll
    for (int m4 = 0; m4 < BMAX / 4; ++m4) {
      const f32x4 kv = *reinterpret_cast<const f32x4*>(kb + 4 * m4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = 4 * m4 + e;
        // (inline: the compiler paired these shifted FMAs on the packed VALU
        // at the cost of ~1.5 v_mov per value)
#pragma unroll
        for (int u = 0; u < CPT; ++u)
          if (m < BMAX - 1)
            asm("v_fma_f32 %0, %1, %2, %3" : "=v"(acc[m][u]) : "v"(kv[e]), "v"(wj[u]), "v"(acc[m + 1][u]));
      }
    }
#pragma unroll
    for (int u = 0; u < CPT; ++u) acc[BMAX - 1][u] = 0.f;
  }
  __syncthreads();
  for (int i = 0; i < B; ++i) {
    const int64_t gi = r0 + i;
#pragma unroll
    for (int u = 0; u < CPT; ++u) {
      const int c = t + 256 * u;
      if (c >= d) continue;
      const float xc = xn[i * pitch + c];
      X[gi * ldx + c] = xc + cen[u];
      Y[gi * ldy + c] = xc;
      if (refreshed) {
        const float sv = sn[i * dp + c];
        S[gi * lds + c] = sv;
        Y[gi * ldy + dp + c] = sv;
      }
    }
  }
  {  // norms: four threads per row, a quarter of the features each (zero past d)
    const int i = t >> 2, q4i = t & 3, q4 = dp >> 2;
    float s2a = 0.f, s2b = 0.f;
    if (i < B) {
      const float* pr = xn + i * pitch + q4i * q4;
      for (int cc = 0; cc < q4; cc += 4) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(pr + cc);
        s2a = fmaf(v[0], v[0], fmaf(v[2], v[2], s2a));
        s2b = fmaf(v[1], v[1], fmaf(v[3], v[3], s2b));
      }
    }
    float s2 = s2a + s2b;
    s2 += __shfl_xor(s2, 1, 64);
    s2 += __shfl_xor(s2, 2, 64);
    if (i < B && q4i == 0) norms[r0 + i] = s2;
  }
}

// the incremental walk for the shapes it covers (A/B switch dsvgd_gsw_set_inc)
static int g_gsw_inc = 1;

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
  const int rc = check_launch("gs_part");
  if (rc || nsplit == 1 || gs_fold(B, d, nsplit)) return rc;
  const int64_t elems = B * d;
  hipLaunchKernelGGL(gs_reduce_kernel, dim3((unsigned)((elems + 63) / 64)), dim3(256), 0,
                     (hipStream_t)stream, partial, elems, (int)nsplit);
  return check_launch("gs_reduce");
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
                     n, (int)d, r0, (int)B, st, step, partial, gs_fold(B, d, nsplit) ? (int)nsplit : 1,
                     extra, lde, phi_out,
                     ldphi, score_kind, mu, lam, score_scale);
  return check_launch("gs_sweep");
}

static int& gsw_debug_mask() {
  static int m = 0;
  return m;
}

int dsvgd_gsw_debug(int mask) {
  const int old = gsw_debug_mask();
  gsw_debug_mask() = mask;
  return old;
}

int dsvgd_gsw_set_inc(int on) {
  const int prev = g_gsw_inc;
  g_gsw_inc = on ? 1 : 0;
  return prev;
}

int64_t dsvgd_gsw_block_rows(int64_t d, int score_kind) {
  if (d <= 0 || d > kGswMaxD) return 0;
  return gsw_rows(roundup(d, 32), score_kind != 0);
}

int dsvgd_gs_mask(float* D, int64_t ldd, int64_t r0, int64_t B, void* stream) {
  DSVGD_REQUIRE(D, "null pointer");
  DSVGD_REQUIRE(B > 0 && B <= 1024 && r0 >= 0 && r0 + B <= ldd && ldd % 128 == 0, "sizes");
  hipLaunchKernelGGL(gs_mask_kernel, dim3((unsigned)B), dim3(256), 0, (hipStream_t)stream, D, ldd,
                     r0, (int)B);
  return check_launch("gs_mask");
}

int dsvgd_gs_mask_cols(float* D, int64_t ldd, int64_t B, int64_t c0, int64_t nc, void* stream) {
  DSVGD_REQUIRE(D, "null pointer");
  DSVGD_REQUIRE(B > 0 && B <= 1024 && c0 >= 0 && nc > 0 && c0 + nc <= ldd && ldd % 128 == 0,
                "sizes");
  hipLaunchKernelGGL(gs_mask_cols_kernel, dim3((unsigned)B), dim3(256), 0, (hipStream_t)stream, D,
                     ldd, c0, nc);
  return check_launch("gs_mask_cols");
}

int dsvgd_debug_spin(int64_t ns, void* stream) {
  DSVGD_REQUIRE(ns >= 0 && ns <= 1000000000, "0 <= ns <= 1 s");
  hipLaunchKernelGGL(debug_spin_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, ns / 10);
  return check_launch("debug_spin");
}

int dsvgd_gsw_group_corr(const float* X, int64_t ldx, const float* S, int64_t lds,
                         const float* center, int64_t n, int64_t d, int64_t r0, int64_t nr,
                         int64_t p0, int64_t pB, const dsvgd_select_state* st, float* Q,
                         int64_t ldq, float* Qr, void* stream) {
  DSVGD_REQUIRE(X && S && center && st && Q && Qr, "null pointer");
  const int64_t dp = roundup(d, 32);
  DSVGD_REQUIRE(n > 0 && d > 0 && d <= kGswMaxD && ldx >= d && lds >= d && ldq >= 2 * dp,
                "sizes (d <= 1024, ldq >= 2 roundup(d, 32))");
  DSVGD_REQUIRE(nr > 0 && nr <= 65535 && r0 >= 0 && r0 + nr <= n && pB > 0 &&
                    pB <= 2 * kGsB && p0 >= 0 && p0 + pB <= r0,
                "rows: the later rows [r0, r0 + nr) after at most 128 rows [p0, p0 + pB)");
  hipLaunchKernelGGL(gsw_group_corr_kernel, dim3((unsigned)nr), dim3(256), 0, (hipStream_t)stream,
                     X, ldx, S, lds, center, d, dp, r0, p0, (int)pB, st, Q, ldq, Qr);
  return check_launch("gsw_group_corr");
}

int dsvgd_gsw_block_sweep(float* X, int64_t ldx, float* S, int64_t lds, float* Y, int64_t ldy,
                          float* norms, const float* center, int64_t n, int64_t d, int64_t r0,
                          int64_t B, const dsvgd_select_state* st, float step, const float* Q,
                          int64_t ldq, const float* Qr, const float* extra, int64_t lde,
                          float* phi_out, int64_t ldphi, int score_kind, const float* mu,
                          const float* lam, float score_scale, const float* xd, int64_t ldxd,
                          const float* td, int64_t nd, void* stream) {
  DSVGD_REQUIRE(X && S && Y && norms && center && st && Q && Qr, "null pointer");
  const int64_t dp = roundup(d, 32);
  DSVGD_REQUIRE(n > 0 && d > 0 && d <= kGswMaxD && ldx >= d && lds >= d && ldy >= 2 * dp &&
                    ldq >= 2 * dp,
                "sizes (d <= 1024, ldy and ldq >= 2 roundup(d, 32))");
  DSVGD_REQUIRE(B > 0 && B <= gsw_rows(dp, score_kind != 0) && r0 >= 0 && r0 + B <= n,
                "block rows (dsvgd_gsw_block_rows(d, score_kind))");
  DSVGD_REQUIRE(score_kind >= 0 && score_kind <= 3, "score_kind must be 0, 1, 2 or 3");
  DSVGD_REQUIRE(score_kind != 1 || (mu && lam), "Gaussian scores need mu and lam");
  DSVGD_REQUIRE(score_kind != 3 || (xd && td && d >= 2 && ldxd >= d - 1 && nd > 0 &&
                                    nd < ((int64_t)1 << 31)),
                "logreg scores need the data (nd rows of d - 1 features) and the labels");
  DSVGD_REQUIRE(score_kind != 3 || (ldxd % 4 == 0 && ((uintptr_t)xd & 15) == 0),
                "logreg data rows must be 16-byte aligned (ldxd % 4 == 0)");
  DSVGD_REQUIRE(!extra || lde >= d, "lde");
  DSVGD_REQUIRE(!phi_out || ldphi >= d, "ldphi");
  const int cpt = dp <= kGsiMaxDp ? 1 : (dp <= 2 * kGsiMaxDp ? 2 : 4);
  // the incremental walk (roundup(d, 32) <= 1024 at 1 / 2 / 4 columns per
  // thread, B <= 64 / cpt rows); when its LDS cannot be reserved the
  // four-wave walk below runs the block instead (slower, same results)
  const size_t smem_i = sizeof(float) * ((size_t)B * (kGsiMaxDp * cpt + 4) +
                                         (score_kind != 0 ? (size_t)B * dp : 0) + 128);
  const void* fn_i = cpt == 1   ? reinterpret_cast<const void*>(&gsw_inc_kernel<1>)
                     : cpt == 2 ? reinterpret_cast<const void*>(&gsw_inc_kernel<2>)
                                : reinterpret_cast<const void*>(&gsw_inc_kernel<4>);
  if (g_gsw_inc && score_kind != 3 && B <= 64 / cpt && !(gsw_debug_mask() & 7) &&
      hipFuncSetAttribute(fn_i, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem_i) ==
          hipSuccess) {
#define DSVGD_GSI(C)                                                                              \
  hipLaunchKernelGGL(gsw_inc_kernel<C>, dim3(1), dim3(256), smem_i, (hipStream_t)stream, X, ldx, S, \
                     lds, Y, ldy, norms, center, n, (int)d, (int)dp, r0, (int)B, st, step, Q, ldq,  \
                     Qr, extra, lde, phi_out, ldphi, score_kind, mu, lam, score_scale)
    if (cpt == 1)
      DSVGD_GSI(1);
    else if (cpt == 2)
      DSVGD_GSI(2);
    else
      DSVGD_GSI(4);
#undef DSVGD_GSI
    return check_launch("gsw_inc");
  }
  const size_t smem =
      sizeof(float) * ((size_t)B * (dp + 4) + (size_t)B * dp * (score_kind != 0 ? 2 : 1) + 256 +
                       1024 + 16 + (score_kind == 3 ? kGswCoef : 0));
  const void* fn = score_kind == 3 ? reinterpret_cast<const void*>(&gsw_sweep_kernel<true>)
                                    : reinterpret_cast<const void*>(&gsw_sweep_kernel<false>);
  if (hipFuncSetAttribute(fn,
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem) != hipSuccess)
    return fail_arg("gsw_sweep: cannot reserve the walk's LDS");
  if (score_kind == 3)
    hipLaunchKernelGGL(gsw_sweep_kernel<true>, dim3(1), dim3(256), smem, (hipStream_t)stream, X, ldx, S,
                     lds, Y, ldy, norms, center, n, (int)d, (int)dp, r0, (int)B, st, step, Q, ldq,
                     Qr, extra, lde, phi_out, ldphi, score_kind, mu, lam, score_scale, xd, ldxd,
                     td, (int)(score_kind == 3 ? nd : 0), gsw_debug_mask());
  else
    hipLaunchKernelGGL(gsw_sweep_kernel<false>, dim3(1), dim3(256), smem, (hipStream_t)stream, X, ldx, S,
                     lds, Y, ldy, norms, center, n, (int)d, (int)dp, r0, (int)B, st, step, Q, ldq,
                     Qr, extra, lde, phi_out, ldphi, score_kind, mu, lam, score_scale, xd, ldxd,
                     td, (int)(score_kind == 3 ? nd : 0), gsw_debug_mask());
  return check_launch("gsw_sweep");
}

}  // extern "C"
