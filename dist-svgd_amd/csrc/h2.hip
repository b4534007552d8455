// h2.hip -- operand preparation of the FmtH2 split engine (gemm_x3.hpp):
// power-of-two scales and the two-part fp16 images.
//
// An operand v is fed to the fp16 MFMA as s v = v0 + v1 (v0 = f16(s v),
// v1 = f16(s v - v0)), s a power of two that puts the operand's largest
// magnitude in [2^14, 2^15): per COLUMN for the B operand of the NN engine
// (phi_mm's Y = [Xc | S], logreg's Xd) -- a column's scale divides out of the
// same output column -- and per TENSOR for the row images of the NT engine
// (the Gram's Xc, logreg's W and Xd), whose scales divide out of every entry.
// HBM passes, O(rows x cols): ~0.1 ms at n = 65536, d = 256.
#include <cmath>

#include "common.hpp"
#include "gemm_x3.hpp"

namespace dsvgd {

constexpr int kScaleRows = 512;  // rows per partial-max block
constexpr float kH2Range = 65536.f;  // 2^16: FmtH2's window

// partial[b][c] = max |A[r][c]| over rows r of block b, as the bit pattern of
// |v| (unsigned order: finite < inf < NaN, so a NaN or inf is carried through)
// -- 64-column stripes, 4 row groups of 64 lanes, four loads in flight per lane.

__global__ __launch_bounds__(256) void colmax_partial_kernel(const float* __restrict__ A,
                                                             int64_t lda, int64_t rows,
                                                             int64_t cols,
                                                             uint32_t* __restrict__ partial) {
  __shared__ uint32_t red[4][64];
  const int64_t c = (int64_t)blockIdx.y * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * kScaleRows, r1 = min(r0 + kScaleRows, rows);
  uint32_t m0 = 0u, m1 = 0u, m2 = 0u, m3 = 0u;
  if (c < cols) {
    int64_t r = r0 + rg;
    for (; r + 12 < r1; r += 16) {
      m0 = max(m0, abs_bits(A[r * lda + c]));
      m1 = max(m1, abs_bits(A[(r + 4) * lda + c]));
      m2 = max(m2, abs_bits(A[(r + 8) * lda + c]));
      m3 = max(m3, abs_bits(A[(r + 12) * lda + c]));
    }
    for (; r < r1; r += 4) m0 = max(m0, abs_bits(A[r * lda + c]));
  }
  red[rg][threadIdx.x & 63] = max(max(m0, m1), max(m2, m3));
  __syncthreads();
  if (rg == 0 && c < cols)
    partial[(int64_t)blockIdx.x * cols + c] =
        max(max(red[0][threadIdx.x], red[1][threadIdx.x]),
            max(red[2][threadIdx.x], red[3][threadIdx.x]));
}

// the range statistics of the unfused path (d > 1024, no pack maxima):
// rng[0 | 1] = largest |entry| of the half [0, dp) | [dp, cols), rng[2 | 3] =
// the smallest nonzero row max of that half (bit patterns; one wave per row,
// one atomic per wave and statistic -- vector-memory atomics on 4 words)
__global__ void rowrange_init_kernel(uint32_t* __restrict__ rng) {
  if (threadIdx.x < 4) rng[threadIdx.x] = threadIdx.x < 2 ? 0u : 0x7F800000u;
}

__global__ __launch_bounds__(256) void rowrange_kernel(const float* __restrict__ A, int64_t lda,
                                                       int64_t rows, int64_t cols, int64_t dp,
                                                       uint32_t* __restrict__ rng) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= rows) return;
  uint32_t mx = 0u, ms = 0u;
  for (int64_t c = lane; c < cols; c += 64) {
    const uint32_t v = abs_bits(A[i * lda + c]);
    if (c < dp) mx = max(mx, v);
    else ms = max(ms, v);
  }
  for (int o = 32; o > 0; o >>= 1) {
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
    ms = max(ms, (uint32_t)__shfl_xor((int)ms, o));
  }
  if (lane == 0) {
    atomicMax(&rng[0], mx);
    atomicMax(&rng[1], ms);
    if (mx) atomicMin(&rng[2], mx);
    if (ms) atomicMin(&rng[3], ms);
  }
}

// one block: out[c] = s_c, out[cols + c] = 1 / s_c; out[2 cols] = t = the
// smallest s_c over the nonzero finite columns (1 if any column is not
// finite, or none is nonzero), out[2 cols + 1] = 1 / t; out[2 cols + 2] =
// the range guard from rng (as scales_h2_kernel's; 0 without rng)
__global__ __launch_bounds__(256) void colscale_final_kernel(const uint32_t* __restrict__ partial,
                                                             int64_t nb, int64_t cols,
                                                             float* __restrict__ out,
                                                             const uint32_t* __restrict__ rng,
                                                             int both) {
  __shared__ float red[256];
  __shared__ int bad[256];
  float tmin = INFINITY;
  int nonfinite = 0;
  for (int64_t c = threadIdx.x; c < cols; c += 256) {
    // eight independent chains: the loads are in flight together
    uint32_t mq[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
    int64_t b = 0;
    for (; b + 8 <= nb; b += 8)
#pragma unroll
      for (int q = 0; q < 8; ++q) mq[q] = max(mq[q], partial[(b + q) * cols + c]);
    for (; b < nb; ++b) mq[0] = max(mq[0], partial[b * cols + c]);
    uint32_t mb = 0u;
#pragma unroll
    for (int q = 0; q < 8; ++q) mb = max(mb, mq[q]);
    const float m = __uint_as_float(mb);
    const float s = pow2_scale(m);
    out[c] = s;
    out[cols + c] = 1.f / s;
    if (!isfinite(m)) nonfinite = 1;
    else if (m > 0.f) tmin = fminf(tmin, s);
  }
  red[threadIdx.x] = tmin;
  bad[threadIdx.x] = nonfinite;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      red[threadIdx.x] = fminf(red[threadIdx.x], red[threadIdx.x + o]);
      bad[threadIdx.x] |= bad[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float t = (bad[0] || !isfinite(red[0])) ? 1.f : red[0];
    out[2 * cols] = t;
    out[2 * cols + 1] = 1.f / t;
    float guard = 0.f;
    if (rng) {
      const bool gx_wide = __uint_as_float(rng[0]) > kH2Range * __uint_as_float(rng[2]);
      const bool gs_wide = __uint_as_float(rng[1]) > kH2Range * __uint_as_float(rng[3]);
      guard = (gx_wide || (both && gs_wide)) ? 1.f : 0.f;
    }
    out[2 * cols + 2] = guard;
  }
}

// the scales of dsvgd_h2_colscale's layout from pack_h2's maxima, over the
// first `cols` columns (cols == dp: the X half; cols == ldy: all of Y,
// phi_mm's B image).  16 columns x 16 row groups per block; t =
// pow2_scale(the largest magnitude over those columns) -- the smallest
// nonzero column scale, since pow2_scale is monotone, and 1 when it is 0 or
// not finite -- from gmax, by every block's lane group 0 (block 0 writes it),
// and the RANGE GUARD out[2 cols + 2]: 1 when a half of Y in those columns
// has its largest magnitude more than kH2Range times its smallest nonzero
// row max (some particle's row then sits below FmtH2's 2^-16 window of its
// column's scale), else 0.
constexpr int kScaleCols = 16;

__global__ __launch_bounds__(256) void scales_h2_kernel(const uint32_t* __restrict__ partial,
                                                        const uint32_t* __restrict__ gmax,
                                                        int64_t nb, int64_t ldp, int64_t cols,
                                                        int64_t dp, float* __restrict__ out) {
  __shared__ uint32_t red[16][kScaleCols];
  __shared__ uint32_t gred[4][4];
  const int cl = threadIdx.x & (kScaleCols - 1), rg = threadIdx.x / kScaleCols;
  const int64_t c = (int64_t)blockIdx.x * kScaleCols + cl;
  uint32_t m0 = 0u, m1 = 0u, m2 = 0u, m3 = 0u;
  if (c < cols) {
    int64_t b = rg;
    for (; b + 48 < nb; b += 64) {
      m0 = max(m0, partial[b * ldp + c]);
      m1 = max(m1, partial[(b + 16) * ldp + c]);
      m2 = max(m2, partial[(b + 32) * ldp + c]);
      m3 = max(m3, partial[(b + 48) * ldp + c]);
    }
    for (; b < nb; b += 16) m0 = max(m0, partial[b * ldp + c]);
  }
  red[rg][cl] = max(max(m0, m1), max(m2, m3));
  __syncthreads();
  if (rg == 0 && c < cols) {
    uint32_t mb = 0u;
#pragma unroll
    for (int q = 0; q < 16; ++q) mb = max(mb, red[q][cl]);
    const float s = pow2_scale(__uint_as_float(mb));
    out[c] = s;
    out[cols + c] = 1.f / s;
  }
  if (blockIdx.x == 0) {
    // gmax[4b + h]: largest |entry| of half h; gmax[4b + 2 + h]: smallest
    // nonzero row max of half h (h = 0: [0, dp), h = 1: the rest of the row)
    uint32_t gx = 0u, gs = 0u, rx = 0x7F800000u, rs = 0x7F800000u;
    for (int64_t b = threadIdx.x; b < nb; b += 256) {
      gx = max(gx, gmax[4 * b]);
      gs = max(gs, gmax[4 * b + 1]);
      rx = min(rx, gmax[4 * b + 2]);
      rs = min(rs, gmax[4 * b + 3]);
    }
    for (int o = 32; o > 0; o >>= 1) {
      gx = max(gx, (uint32_t)__shfl_xor((int)gx, o));
      gs = max(gs, (uint32_t)__shfl_xor((int)gs, o));
      rx = min(rx, (uint32_t)__shfl_xor((int)rx, o));
      rs = min(rs, (uint32_t)__shfl_xor((int)rs, o));
    }
    if ((threadIdx.x & 63) == 0) {
      gred[threadIdx.x >> 6][0] = gx;
      gred[threadIdx.x >> 6][1] = gs;
      gred[threadIdx.x >> 6][2] = rx;
      gred[threadIdx.x >> 6][3] = rs;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t g[4];
#pragma unroll
      for (int h = 0; h < 4; ++h)
        g[h] = h < 2 ? max(max(gred[0][h], gred[1][h]), max(gred[2][h], gred[3][h]))
                     : min(min(gred[0][h], gred[1][h]), min(gred[2][h], gred[3][h]));
      const bool both = cols > dp;
      const float t = pow2_scale(__uint_as_float(both ? max(g[0], g[1]) : g[0]));
      out[2 * cols] = t;
      out[2 * cols + 1] = 1.f / t;
      const bool gx_wide = __uint_as_float(g[0]) > kH2Range * __uint_as_float(g[2]);
      const bool gs_wide = __uint_as_float(g[1]) > kH2Range * __uint_as_float(g[3]);
      out[2 * cols + 2] = (gx_wide || (both && gs_wide)) ? 1.f : 0.f;
    }
  }
}

// rscale[i] = pow2_scale(max_c |A[i][c]|) and rinv[i] = 1 / rscale[i] for
// rows i < rows (1 for a zero / non-finite row; rows_pad > rows: 1): the
// per-row scales of an NT row image (the Gram's, logreg's W) -- one wave per row.
__global__ __launch_bounds__(256) void rowscale_h2_kernel(const float* __restrict__ A,
                                                          int64_t lda, int64_t rows, int64_t cols,
                                                          int64_t rows_pad,
                                                          float* __restrict__ rscale,
                                                          float* __restrict__ rinv) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= rows_pad) return;
  uint32_t m = 0u;
  if (i < rows)
    for (int64_t c = lane; c < cols; c += 64) m = max(m, abs_bits(A[i * lda + c]));
  for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
  if (lane == 0) {
    const float s = pow2_scale(__uint_as_float(m));
    rscale[i] = s;
    if (rinv) rinv[i] = pow2_inv(s);
  }
}

// Yh[kstep][part][column][16 k] = the two fp16 parts of s_c Y[16 kstep + k][c]
// (16-B halves swapped on columns with bit 3 set: the 32x32x16 image)
__global__ __launch_bounds__(256) void ysplit_h2_kernel(const float* __restrict__ Y, int64_t ldy,
                                                        int64_t ksteps,
                                                        const float* __restrict__ colscale,
                                                        _Float16* __restrict__ Yh) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= ksteps * ldy) return;
  const int64_t kb = t / ldy, c = t % ldy;
  const float sc = colscale[c];
  f16x8 s[2][2];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    _Float16 v[2];
    split_fmt<FmtH2>(sc * Y[(kb * 16 + k) * ldy + c], v);
    s[0][k >> 3][k & 7] = v[0];
    s[1][k >> 3][k & 7] = v[1];
  }
  const int sw = (int)((c >> 3) & 1);
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    _Float16* dst = Yh + ((kb * 2 + p) * ldy + c) * 16;
    *reinterpret_cast<f16x8*>(dst + 8 * sw) = s[p][0];
    *reinterpret_cast<f16x8*>(dst + 8 * (sw ^ 1)) = s[p][1];
  }
}

// img[kstep][part][row][16 k] = the two fp16 parts of t A[row][16 kstep + k]
// (t = *tscale; zero outside rows x cols; halves swapped on rows with bit 3 set)
// OFF >= 0: lda % 4 == 0 and A sits OFF floats past a 16-byte boundary (e.g.
// logreg's W = X[:, 1:], OFF = 1): a thread's 16 values come in as 16-byte
// loads of the aligned window around them (four, or five when OFF > 0; each
// load's 16-byte chunk holds an element of the row, so it stays inside
// mapped memory) -- scalar loads would touch 64 rows' lines per
// wave-instruction, 16 times over.  OFF < 0: element loads (any layout).
// RS: tscale is per ROW (tscale[i], rows < rows_pad), else one tensor scale.
template <int OFF, bool RS = false>
__global__ __launch_bounds__(256) void rowsplit_h2_kernel(const float* __restrict__ A,
                                                          int64_t lda, int64_t rows, int64_t cols,
                                                          int64_t rows_pad, int64_t ksteps,
                                                          const float* __restrict__ tscale,
                                                          _Float16* __restrict__ img,
                                                          int64_t row_begin = 0,
                                                          int64_t nrows = -1) {
  // rows [row_begin, row_begin + nrows) of the image (default: all rows_pad)
  const int64_t nr = nrows < 0 ? rows_pad : nrows;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= ksteps * nr) return;
  const int64_t kb = t / nr, i = row_begin + t % nr;
  const float sc = RS ? (i < rows ? tscale[i] : 1.f) : *tscale;
  float a[16];
  if (OFF >= 0 && i < rows && kb * 16 + 16 <= cols) {
    constexpr int kOff = OFF < 0 ? 0 : OFF;
    constexpr int kLoads = kOff ? 5 : 4;
    const f32x4* src = reinterpret_cast<const f32x4*>(A + i * lda + kb * 16 - kOff);
    float win[4 * kLoads];
#pragma unroll
    for (int q = 0; q < kLoads; ++q) {
      const f32x4 v = src[q];
#pragma unroll
      for (int e = 0; e < 4; ++e) win[4 * q + e] = v[e];
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) a[k] = win[k + kOff];
  } else {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int64_t c = kb * 16 + k;
      a[k] = (i < rows && c < cols) ? A[i * lda + c] : 0.f;
    }
  }
  f16x8 s[2][2];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    _Float16 v[2];
    split_fmt<FmtH2>(sc * a[k], v);
    s[0][k >> 3][k & 7] = v[0];
    s[1][k >> 3][k & 7] = v[1];
  }
  const int sw = (int)((i >> 3) & 1);
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    _Float16* dst = img + ((kb * 2 + p) * rows_pad + i) * 16;
    *reinterpret_cast<f16x8*>(dst + 8 * sw) = s[p][0];
    *reinterpret_cast<f16x8*>(dst + 8 * (sw ^ 1)) = s[p][1];
  }
}

// rowscale_h2_kernel and rowsplit_h2_kernel<*, true> in one pass (the
// logreg W image, rebuilt every step): one wave per row takes the row's
// largest magnitude, its power-of-two scale (rscale, rinv), then splits the
// row -- the second read hits the L1 / L2 lines the first one brought in.
// Per 256-column chunk lane l holds K-step 16 q + l / 4, values 4 (l & 3) ..
// +3: one 8-byte store per part into the row's 32-byte slot (halves swapped
// on rows with bit 3 set, as rowsplit_h2_kernel).  Same bits as the two
// kernels (same maxima, scales and splits).
__global__ __launch_bounds__(256) void rowimage_h2_kernel(const float* __restrict__ A,
                                                          int64_t lda, int64_t rows, int64_t cols,
                                                          int64_t rows_pad, int64_t ksteps,
                                                          float* __restrict__ rscale,
                                                          float* __restrict__ rinv,
                                                          _Float16* __restrict__ img) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= rows_pad) return;
  const float* row = A + i * lda;
  const int sw = (int)((i >> 3) & 1);
  const int k0 = 4 * (lane & 3);
  const int pos = (k0 < 8 ? 8 * sw : 8 * (sw ^ 1)) + (k0 & 7);
  if (ksteps <= 16) {
    // one K-step per lane (kb = lane / 4: columns 4 lane .. 4 lane + 3): the
    // row read once, every load before the maximum's reduction (the same
    // maximum, scale and splits)
    const int64_t kb = lane >> 2;
    float a[4];
    uint32_t m = 0u;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t c = kb * 16 + k0 + e;
      a[e] = (kb < ksteps && i < rows && c < cols) ? row[c] : 0.f;
      m = max(m, abs_bits(a[e]));
    }
    for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
    const float sc = pow2_scale(__uint_as_float(m));
    if (lane == 0) {
      rscale[i] = sc;
      rinv[i] = pow2_inv(sc);
    }
    if (kb >= ksteps) return;
    f16x4 h[2];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      _Float16 v[2];
      split_fmt<FmtH2>(sc * a[e], v);
      h[0][e] = v[0];
      h[1][e] = v[1];
    }
#pragma unroll
    for (int p = 0; p < 2; ++p)
      *reinterpret_cast<f16x4*>(img + ((kb * 2 + p) * rows_pad + i) * 16 + pos) = h[p];
    return;
  }
  uint32_t m = 0u;
  if (i < rows)
    for (int64_t c = lane; c < cols; c += 64) m = max(m, abs_bits(row[c]));
  for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
  const float sc = pow2_scale(__uint_as_float(m));
  if (lane == 0) {
    rscale[i] = sc;
    rinv[i] = pow2_inv(sc);
  }
  for (int64_t kb = lane >> 2; kb < ksteps; kb += 16) {
    f16x4 h[2];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t c = kb * 16 + k0 + e;
      const float a = (i < rows && c < cols) ? row[c] : 0.f;
      _Float16 v[2];
      split_fmt<FmtH2>(sc * a, v);
      h[0][e] = v[0];
      h[1][e] = v[1];
    }
#pragma unroll
    for (int p = 0; p < 2; ++p)
      *reinterpret_cast<f16x4*>(img + ((kb * 2 + p) * rows_pad + i) * 16 + pos) = h[p];
  }
}

// the partial maxima, then 4 words of range statistics (dsvgd_h2_colscale_guarded)
size_t h2_colscale_ws_floats(int64_t rows, int64_t cols) {
  return (size_t)((rows + kScaleRows - 1) / kScaleRows) * (size_t)(cols < 1 ? 1 : cols) + 4;
}

// dp > 0: also the range guard of the halves [0, dp) and [dp, cols) (a
// second pass over A's rows: the unfused path only)
int h2_colscale(const float* A, int64_t lda, int64_t rows, int64_t cols, int64_t dp, float* ws,
                float* out, hipStream_t s) {
  const int64_t nb = (rows + kScaleRows - 1) / kScaleRows;
  uint32_t* part = reinterpret_cast<uint32_t*>(ws);
  uint32_t* rng = dp > 0 ? part + nb * cols : nullptr;
  hipLaunchKernelGGL(colmax_partial_kernel, dim3((unsigned)nb, (unsigned)((cols + 63) / 64)),
                     dim3(256), 0, s, A, lda, rows, cols, part);
  int rc = check_launch("colmax_partial");
  if (rc) return rc;
  if (rng) {
    hipLaunchKernelGGL(rowrange_init_kernel, dim3(1), dim3(64), 0, s, rng);
    hipLaunchKernelGGL(rowrange_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, A, lda,
                       rows, cols, dp, rng);
    if ((rc = check_launch("rowrange"))) return rc;
  }
  hipLaunchKernelGGL(colscale_final_kernel, dim3(1), dim3(256), 0, s, part, nb, cols, out, rng,
                     (int)(cols > dp));
  return check_launch("colscale_final");
}

int h2_ysplit(const float* Y, int64_t ldy, int64_t rows, const float* colscale, void* Yh,
              hipStream_t s) {
  const int64_t ksteps = rows / kX3Step, threads = ksteps * ldy;
  hipLaunchKernelGGL(ysplit_h2_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, Y,
                     ldy, ksteps, colscale, (_Float16*)Yh);
  return check_launch("ysplit_h2");
}

template <bool RS>
static int h2_rowsplit_t(const float* A, int64_t lda, int64_t rows, int64_t cols, int64_t rows_pad,
                         int64_t kpad, const float* tscale, void* img, hipStream_t s) {
  const int64_t ksteps = kpad / kX3Step, threads = ksteps * rows_pad;
  const dim3 grid((unsigned)((threads + 255) / 256));
  const int off = ((uintptr_t)A & 3) == 0 && lda % 4 == 0 ? (int)(((uintptr_t)A >> 2) & 3) : -1;
#define DSVGD_ROWSPLIT_H2(O)                                                                  \
  hipLaunchKernelGGL((rowsplit_h2_kernel<O, RS>), grid, dim3(256), 0, s, A, lda, rows, cols,   \
                     rows_pad, ksteps, tscale, (_Float16*)img)
  switch (off) {
    case 0: DSVGD_ROWSPLIT_H2(0); break;
    case 1: DSVGD_ROWSPLIT_H2(1); break;
    case 2: DSVGD_ROWSPLIT_H2(2); break;
    case 3: DSVGD_ROWSPLIT_H2(3); break;
    default: DSVGD_ROWSPLIT_H2(-1); break;
  }
#undef DSVGD_ROWSPLIT_H2
  return check_launch("rowsplit_h2");
}

int h2_rowsplit(const float* A, int64_t lda, int64_t rows, int64_t cols, int64_t rows_pad,
                int64_t kpad, const float* tscale, void* img, hipStream_t s) {
  return h2_rowsplit_t<false>(A, lda, rows, cols, rows_pad, kpad, tscale, img, s);
}

int h2_rowsplit_rows(const float* A, int64_t lda, int64_t rows, int64_t cols, int64_t rows_pad,
                     int64_t kpad, const float* rscale, void* img, hipStream_t s) {
  return h2_rowsplit_t<true>(A, lda, rows, cols, rows_pad, kpad, rscale, img, s);
}

// rows [row_begin, row_begin + nrows) of the per-row-scaled image only (the
// wide Gauss-Seidel sweep re-splits the rows a block moved); element loads
int h2_rowsplit_rows_range(const float* A, int64_t lda, int64_t rows, int64_t cols,
                           int64_t rows_pad, int64_t kpad, const float* rscale, void* img,
                           int64_t row_begin, int64_t nrows, hipStream_t s) {
  const int64_t ksteps = kpad / kX3Step, threads = ksteps * nrows;
  hipLaunchKernelGGL((rowsplit_h2_kernel<-1, true>), dim3((unsigned)((threads + 255) / 256)),
                     dim3(256), 0, s, A, lda, rows, cols, rows_pad, ksteps, rscale,
                     (_Float16*)img, row_begin, nrows);
  return check_launch("rowsplit_h2(range)");
}

int h2_rowimage(const float* A, int64_t lda, int64_t rows, int64_t cols, int64_t rows_pad,
                int64_t kpad, float* rscale, float* rinv, void* img, hipStream_t s) {
  hipLaunchKernelGGL(rowimage_h2_kernel, dim3((unsigned)((rows_pad + 3) / 4)), dim3(256), 0, s, A,
                     lda, rows, cols, rows_pad, kpad / kX3Step, rscale, rinv, (_Float16*)img);
  return check_launch("rowimage_h2");
}

int h2_rowscale(const float* A, int64_t lda, int64_t rows, int64_t cols, int64_t rows_pad,
                float* rscale, float* rinv, hipStream_t s) {
  hipLaunchKernelGGL(rowscale_h2_kernel, dim3((unsigned)((rows_pad + 3) / 4)), dim3(256), 0, s, A,
                     lda, rows, cols, rows_pad, rscale, rinv);
  return check_launch("rowscale_h2");
}

}  // namespace dsvgd

using namespace dsvgd;

extern "C" {

size_t dsvgd_h2_colscale_workspace_floats(int64_t rows, int64_t cols) {
  return h2_colscale_ws_floats(rows, cols);
}

int dsvgd_h2_colscale(const float* A, int64_t lda, int64_t rows, int64_t cols, float* ws,
                      float* scale, void* stream) {
  DSVGD_REQUIRE(A && ws && scale, "null pointer");
  DSVGD_REQUIRE(rows > 0 && cols > 0 && lda >= cols, "sizes");
  return h2_colscale(A, lda, rows, cols, 0, ws, scale, (hipStream_t)stream);
}

int dsvgd_h2_colscale_guarded(const float* A, int64_t lda, int64_t rows, int64_t cols, int64_t dp,
                              float* ws, float* scale, void* stream) {
  DSVGD_REQUIRE(A && ws && scale, "null pointer");
  DSVGD_REQUIRE(rows > 0 && cols > 0 && lda >= cols && dp > 0 && dp <= cols, "sizes");
  return h2_colscale(A, lda, rows, cols, dp, ws, scale, (hipStream_t)stream);
}

int dsvgd_h2_scales(const uint32_t* partial, const uint32_t* gmax, int64_t nb, int64_t ldy,
                    int64_t cols, int64_t dp, float* scale, void* stream) {
  DSVGD_REQUIRE(partial && gmax && scale, "null pointer");
  DSVGD_REQUIRE(nb > 0 && dp > 0 && (cols == dp || cols == ldy) && ldy >= 2 * dp,
                "cols must be dp (the X half) or ldy (all of Y)");
  hipLaunchKernelGGL(scales_h2_kernel, dim3((unsigned)((cols + kScaleCols - 1) / kScaleCols)),
                     dim3(256), 0, (hipStream_t)stream, partial, gmax, nb, ldy, cols, dp, scale);
  return check_launch("scales_h2");
}

int64_t dsvgd_h2_image_bytes(int64_t rows, int64_t cols) {
  return roundup(rows, kX3Step) * roundup(cols, kX3Step) * 2 * 2;
}

int dsvgd_h2_ysplit(const float* Y, int64_t ldy, int64_t rows, const float* colscale, void* Yh,
                    void* stream) {
  DSVGD_REQUIRE(Y && colscale && Yh, "null pointer");
  DSVGD_REQUIRE(rows > 0 && rows % kX3Step == 0, "rows must be a positive multiple of 16");
  DSVGD_REQUIRE(ldy > 0 && ldy % 16 == 0, "ldy must be a multiple of 16");
  DSVGD_REQUIRE(((uintptr_t)Yh & 15) == 0, "16-byte alignment");
  return h2_ysplit(Y, ldy, rows, colscale, Yh, (hipStream_t)stream);
}

int dsvgd_h2_rowsplit(const float* A, int64_t lda, int64_t rows, int64_t cols, int64_t rows_pad,
                      int64_t kpad, const float* tscale, void* img, void* stream) {
  DSVGD_REQUIRE(A && tscale && img, "null pointer");
  DSVGD_REQUIRE(rows >= 0 && cols >= 0 && rows <= rows_pad && lda >= cols, "sizes");
  DSVGD_REQUIRE(rows_pad > 0 && rows_pad % 16 == 0 && kpad > 0 && kpad % kX3Step == 0,
                "rows_pad and kpad must be positive multiples of 16");
  DSVGD_REQUIRE(((uintptr_t)img & 15) == 0, "16-byte alignment");
  return h2_rowsplit(A, lda, rows, cols, rows_pad, kpad, tscale, img, (hipStream_t)stream);
}

int dsvgd_h2_rowsplit_rows(const float* A, int64_t lda, int64_t rows, int64_t cols,
                           int64_t rows_pad, int64_t kpad, const float* rscale, void* img,
                           void* stream) {
  DSVGD_REQUIRE(A && rscale && img, "null pointer");
  DSVGD_REQUIRE(rows >= 0 && cols >= 0 && rows <= rows_pad && lda >= cols, "sizes");
  DSVGD_REQUIRE(rows_pad > 0 && rows_pad % 16 == 0 && kpad > 0 && kpad % kX3Step == 0,
                "rows_pad and kpad must be positive multiples of 16");
  DSVGD_REQUIRE(((uintptr_t)img & 15) == 0, "16-byte alignment");
  return h2_rowsplit_rows(A, lda, rows, cols, rows_pad, kpad, rscale, img, (hipStream_t)stream);
}

int dsvgd_h2_rowsplit_rows_range(const float* A, int64_t lda, int64_t rows, int64_t cols,
                                 int64_t rows_pad, int64_t kpad, const float* rscale, void* img,
                                 int64_t row_begin, int64_t nrows, void* stream) {
  DSVGD_REQUIRE(A && rscale && img, "null pointer");
  DSVGD_REQUIRE(rows >= 0 && cols >= 0 && rows <= rows_pad && lda >= cols, "sizes");
  DSVGD_REQUIRE(rows_pad > 0 && rows_pad % 16 == 0 && kpad > 0 && kpad % kX3Step == 0,
                "rows_pad and kpad must be positive multiples of 16");
  DSVGD_REQUIRE(row_begin >= 0 && nrows > 0 && row_begin + nrows <= rows_pad, "row range");
  DSVGD_REQUIRE(((uintptr_t)img & 15) == 0, "16-byte alignment");
  return h2_rowsplit_rows_range(A, lda, rows, cols, rows_pad, kpad, rscale, img, row_begin, nrows,
                                (hipStream_t)stream);
}

int dsvgd_h2_rowscale(const float* A, int64_t lda, int64_t rows, int64_t cols, int64_t rows_pad,
                      float* rscale, float* rinv, void* stream) {
  DSVGD_REQUIRE(A && rscale, "null pointer");
  DSVGD_REQUIRE(rows >= 0 && cols > 0 && rows <= rows_pad && lda >= cols, "sizes");
  return h2_rowscale(A, lda, rows, cols, rows_pad, rscale, rinv, (hipStream_t)stream);
}

int dsvgd_h2_rowimage(const float* A, int64_t lda, int64_t rows, int64_t cols, int64_t rows_pad,
                      int64_t kpad, float* rscale, float* rinv, void* img, void* stream) {
  DSVGD_REQUIRE(A && rscale && rinv && img, "null pointer");
  DSVGD_REQUIRE(rows >= 0 && cols > 0 && rows <= rows_pad && lda >= cols && kpad >= cols, "sizes");
  DSVGD_REQUIRE(rows_pad > 0 && rows_pad % 16 == 0 && kpad % kX3Step == 0,
                "rows_pad and kpad must be positive multiples of 16");
  DSVGD_REQUIRE(((uintptr_t)img & 15) == 0, "16-byte alignment");
  return h2_rowimage(A, lda, rows, cols, rows_pad, kpad, rscale, rinv, img, (hipStream_t)stream);
}

}  // extern "C"
