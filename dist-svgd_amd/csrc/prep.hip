// prep.hip -- ABI meta, error plumbing, particle preparation (mean, pack),
// elementwise target scores.  Bandwidth: HBM (all O(n d) streams).
#include <cstdarg>
#include <cmath>

#include "common.hpp"

namespace dsvgd {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int fail_arg(const char* what) {
  set_error("invalid argument: %s", what);
  return DSVGD_E_ARG;
}

int check_launch(const char* kernel) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s launch failed: %s", kernel, hipGetErrorString(e));
    return DSVGD_E_LAUNCH;
  }
  return DSVGD_OK;
}

// Grid of a persistent kernel: resident blocks per CU (occupancy of `fn` at
// `threads` threads, no dynamic LDS) x CUs, a multiple of the 8 XCDs.
// Cached per (kernel, device).
// CUs a persistent launch leaves free (dsvgd_set_cu_reserve): the pipelined
// Gauss-Seidel sweep's side-stream passes leave room for the walk beside them
static int g_cu_reserve = 0;
int set_cu_reserve(int cus) {
  const int prev = g_cu_reserve;
  g_cu_reserve = cus < 0 ? 0 : cus;
  return prev;
}

int persistent_blocks(const void* fn, int* blocks, int threads) {
  struct Entry { const void* fn; int dev; int per_cu, cus; };
  static thread_local Entry cache[16];
  static thread_local int ncache = 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    set_error("hipGetDevice failed");
    return DSVGD_E_LAUNCH;
  }
  int per_cu = 0, cus = 0;
  bool hit = false;
  for (int i = 0; i < ncache && !hit; ++i)
    if (cache[i].fn == fn && cache[i].dev == dev) {
      per_cu = cache[i].per_cu;
      cus = cache[i].cus;
      hit = true;
    }
  if (!hit) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, threads, 0) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
      set_error("occupancy query failed");
      return DSVGD_E_LAUNCH;
    }
    if (ncache < 16) cache[ncache++] = Entry{fn, dev, per_cu, cus};
  }
  const int use = cus - g_cu_reserve >= 8 ? cus - g_cu_reserve : 8;
  int b = (per_cu < 1 ? 1 : per_cu) * use;
  b = b >= 8 ? b / 8 * 8 : 8;
  *blocks = b;
  return DSVGD_OK;
}

// ---------------------------------------------------------------- mean ----
// Deterministic two-level column sum: block b sums rows [b*R, (b+1)*R) of a
// 64-column stripe into partial[b][c]; the second kernel sums the partials in
// block order.  (Float atomics would make the centring -- and so the median
// bits -- vary from run to run.)
constexpr int kMeanRows = 512;

__global__ __launch_bounds__(256) void colsum_partial_kernel(const float* __restrict__ X,
                                                             int64_t ldx, int64_t n, int64_t d,
                                                             float* __restrict__ partial) {
  __shared__ float red[4][64];
  const int c = blockIdx.y * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;  // 4 row groups
  const int64_t r0 = (int64_t)blockIdx.x * kMeanRows;
  const int64_t r1 = min(r0 + kMeanRows, n);
  // four independent chains per lane: four row loads in flight, not one
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (c < d) {
    int64_t r = r0 + rg;
    for (; r + 12 < r1; r += 16) {
      a0 += X[r * ldx + c];
      a1 += X[(r + 4) * ldx + c];
      a2 += X[(r + 8) * ldx + c];
      a3 += X[(r + 12) * ldx + c];
    }
    for (; r < r1; r += 4) a0 += X[r * ldx + c];
  }
  red[rg][threadIdx.x & 63] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (rg == 0 && c < d)
    partial[(int64_t)blockIdx.x * d + c] =
        ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x];
}

// 64 columns per block; the 4 waves split the partial rows, 4 chains each
__global__ __launch_bounds__(256) void colsum_final_kernel(const float* __restrict__ partial,
                                                           int64_t nb, int64_t n, int64_t d,
                                                           float* __restrict__ mean) {
  __shared__ float red[4][64];
  const int64_t c = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const int w = threadIdx.x >> 6;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (c < d) {
    int64_t b = w;
    for (; b + 12 < nb; b += 16) {
      a0 += partial[b * d + c];
      a1 += partial[(b + 4) * d + c];
      a2 += partial[(b + 8) * d + c];
      a3 += partial[(b + 12) * d + c];
    }
    for (; b < nb; b += 4) a0 += partial[b * d + c];
  }
  red[w][threadIdx.x & 63] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (w == 0 && c < d)
    mean[c] = (((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) +
               red[3][threadIdx.x]) / (float)n;
}

// --------------------------------------------------------------- center ----
// center[c] = the lower median of column c over m = min(n, kCenterRows) evenly
// spaced rows (row (k n) / m, k < m): a robust centre for the Gram form.
// Centering is exact algebra for phi (translation invariant) and D; what it
// changes is the conditioning of |x|^2 + |y|^2 - 2 x.y and of r x - K X,
// whose fp32 cancellation grows with the particles' distance from the centre.
// The mean moves by (outlier) / n when one particle diverges, and every
// other particle then sits that far from it (a particle 2^16 spreads away
// costs the mean-centred Gram ~3e-4 of phi in fp32); the median of a sample
// stays inside the bulk.  One block per column: the sample is bitonic-sorted
// in LDS (deterministic, no data-dependent control flow).
constexpr int kCenterRows = 1024;

__global__ __launch_bounds__(256) void colcenter_kernel(const float* __restrict__ X, int64_t ldx,
                                                        int64_t n, float* __restrict__ center) {
  __shared__ float v[kCenterRows];
  const int64_t c = blockIdx.x;
  const int m = (int)min(n, (int64_t)kCenterRows);
  for (int k = threadIdx.x; k < kCenterRows; k += 256)
    v[k] = k < m ? X[((int64_t)k * n / m) * ldx + c] : INFINITY;
  __syncthreads();
  for (int size = 2; size <= kCenterRows; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < kCenterRows / 2; t += 256) {
        const int i = 2 * t - (t & (stride - 1)), j = i + stride;
        const float a = v[i], b = v[j];
        if ((a > b) == ((i & size) == 0)) {
          v[i] = b;
          v[j] = a;
        }
      }
      __syncthreads();
    }
  if (threadIdx.x == 0) center[c] = v[(m - 1) / 2];
}

// ---------------------------------------------------------------- pack ----
// Y[j] = [X[j]-mean (dp cols) | scale*S[j] (dp cols) | 0], norms[j] =
// |X[j]-mean|^2, rows j >= n zero; with partial != nullptr also the FmtH2
// statistics of what it writes (h2.hip), so the scales need no second pass
// over Y: partial[b][c] = max |Y[r][c]| over block b's rows
// (pack_rows_per_block), and per block four words (kPackStats) gmax[4b + h]
// = the largest |entry| of half h (0: the X half [0, dp), 1: the S half),
// gmax[4b + 2 + h] = the smallest NONZERO row max of half h over the block's
// rows < n (+inf if none) -- the FmtH2 range guard's input.  rsc != nullptr
// (with X): rsc[j] = the power-of-two FmtH2 scale of row j's X half (its
// largest magnitude -> [2^14, 2^15), 1 for a zero row or a row >= n), the
// per-row scales of the Gram's row image.  X == nullptr: the S half of rows
// < n only (its columns' partials and the S words of gmax).  One wave per
// row, 16-byte accesses: a lane owns 4 adjacent columns of each 256-column
// pass (dp % 32 == 0, so a lane's 4 never straddle the X / S boundary).
constexpr int kPackQ = 8;  // 256-column passes per row: ldy <= 2048
constexpr int kPackStats = 4;
// rows per block: 64 (16 per wave) from ~64K rows, down to 4 (one per wave)
// below ~4K -- a small pack is latency-bound, its waves must not loop
__host__ __device__ inline int64_t pack_rows_per_block(int64_t rows_pad) {
  int64_t r = 4;
  while (r < 64 && rows_pad / (2 * r) >= 1024) r *= 2;
  return r;
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
  return v;
}

// VX / VS: 16-byte loads of X / S rows (aligned, ld % 4 == 0); NQ: the
// 256-column passes ldy needs (<= kPackQ: registers for those only)
template <bool VX, bool VS, int NQ>
__global__ __launch_bounds__(256) void pack_kernel(
    const float* __restrict__ X, int64_t ldx, const float* __restrict__ S, int64_t lds,
    float scale, const float* __restrict__ mean, int64_t n, int64_t d, int64_t rows_pad,
    int64_t dp, float* __restrict__ Y, int64_t ldy, float* __restrict__ norms,
    uint32_t* __restrict__ partial, uint32_t* __restrict__ gmax, float* __restrict__ rsc) {
  extern __shared__ uint32_t red[];  // [4 waves][ldy]
  __shared__ uint32_t gred[4][kPackStats];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t rpb = pack_rows_per_block(rows_pad);
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  const int64_t r1 = min(r0 + rpb, rows_pad);
  // the columns this launch owns -- both: the whole row, pad columns zero;
  // X alone: all but the S half (written by the pack of the scores that
  // follows, or not read); S alone: the S half only
  auto owns = [&](int64_t c) {
    const bool sh = c >= dp && c < 2 * dp;
    return X ? (S != nullptr || !sh) : sh;
  };
  uint32_t mx[NQ][4];
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int e = 0; e < 4; ++e) mx[q][e] = 0u;
  uint32_t rminx = 0x7F800000u, rmins = 0x7F800000u;  // +inf
  // row j's 16-byte pieces (zero past n / outside the halves read)
  auto load_row = [&](int64_t j, f32x4 (&v)[NQ]) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int64_t c = 4 * lane + 256 * q;
      v[q] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (c >= ldy || j >= n) continue;
      if (c < dp) {
        if (!X) continue;
        if (VX && c + 4 <= d) {
          v[q] = *reinterpret_cast<const f32x4*>(X + j * ldx + c) -
                 *reinterpret_cast<const f32x4*>(mean + c);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (c + e < d) v[q][e] = X[j * ldx + c + e] - mean[c + e];
        }
      } else if (c < 2 * dp && S != nullptr) {
        const int64_t cs = c - dp;
        if (VS && cs + 4 <= d) {
          v[q] = scale * *reinterpret_cast<const f32x4*>(S + j * lds + cs);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (cs + e < d) v[q][e] = scale * S[j * lds + cs + e];
        }
      }
    }
  };
  auto store_row = [&](int64_t j, const f32x4 (&v)[NQ]) {
    float nrm = 0.f;
    uint32_t rx = 0u, rs = 0u;  // this row's largest |entry| per half
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int64_t c = 4 * lane + 256 * q;
      if (c >= ldy || !owns(c)) continue;
      *reinterpret_cast<f32x4*>(Y + j * ldy + c) = v[q];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t a = abs_bits(v[q][e]);
        mx[q][e] = max(mx[q][e], a);
        if (c < dp) {
          nrm = fmaf(v[q][e], v[q][e], nrm);
          rx = max(rx, a);
        } else {
          rs = max(rs, a);
        }
      }
    }
    if (X) {
      nrm = warp_sum(nrm);
      if (lane == 0) norms[j] = nrm;
    }
    if (partial != nullptr || rsc != nullptr) {
      rx = wave_max_u32(rx);
      rs = wave_max_u32(rs);
      if (j < n) {
        if (rx != 0u) rminx = min(rminx, rx);
        if (rs != 0u) rmins = min(rmins, rs);
      }
      if (X && rsc && lane == 0) rsc[j] = pow2_scale(j < n ? __uint_as_float(rx) : 0.f);
    }
  };
  // two rows in flight per wave: the next row's loads are issued before this
  // row's reductions (one row at a time left each wave waiting out a full
  // HBM latency per row: ~2 TB/s)
  f32x4 va[NQ], vb[NQ];
  int64_t j = r0 + w;
  if (j < r1) load_row(j, va);
  for (; j < r1; j += 8) {
    const int64_t j2 = j + 4;
    if (j2 < r1) load_row(j2, vb);
    store_row(j, va);
    if (j2 >= r1) break;
    if (j2 + 4 < r1) load_row(j2 + 4, va);
    store_row(j2, vb);
  }
  if (partial == nullptr) return;
  uint32_t gx = 0u, gs = 0u;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int64_t c = 4 * lane + 256 * q;
    if (c >= ldy) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      red[w * ldy + c + e] = mx[q][e];
      if (c < dp) gx = max(gx, mx[q][e]);
      else gs = max(gs, mx[q][e]);
    }
  }
  gx = wave_max_u32(gx);
  gs = wave_max_u32(gs);
  if (lane == 0) {
    gred[w][0] = gx;
    gred[w][1] = gs;
    gred[w][2] = rminx;
    gred[w][3] = rmins;
  }
  __syncthreads();
  for (int64_t c = threadIdx.x; c < ldy; c += 256)
    if (owns(c))
      partial[(int64_t)blockIdx.x * ldy + c] =
          max(max(red[c], red[ldy + c]), max(red[2 * ldy + c], red[3 * ldy + c]));
  // X half: words 0, 2; S half: words 1, 3 (pack(NULL, S) leaves the X words)
  if (threadIdx.x < kPackStats && (X || (threadIdx.x & 1))) {
    const int h = threadIdx.x;
    const uint32_t v = h < 2 ? max(max(gred[0][h], gred[1][h]), max(gred[2][h], gred[3][h]))
                             : min(min(gred[0][h], gred[1][h]), min(gred[2][h], gred[3][h]));
    gmax[kPackStats * blockIdx.x + h] = v;
  }
}

// ldy > 256 kPackQ (d > 1024): one wave per row, element accesses, no maxima: Y[j] = [X[j]-mean (dp cols) | scale*S[j] (dp cols) | 0],
// norms[j] = |X[j]-mean|^2.  Rows j >= n are zero.
__global__ __launch_bounds__(256) void pack_wide_kernel(const float* __restrict__ X, int64_t ldx,
                                                   const float* __restrict__ S, int64_t lds,
                                                   float scale, const float* __restrict__ mean,
                                                   int64_t n, int64_t d, int64_t rows_pad,
                                                   int64_t dp, float* __restrict__ Y, int64_t ldy,
                                                   float* __restrict__ norms) {
  const int lane = threadIdx.x & 63;
  const int64_t j = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j >= rows_pad) return;
  float* y = Y + j * ldy;
  if (X == nullptr) {  // scores only: the S half of rows < n
    if (j < n)
      for (int64_t c = lane; c < d; c += 64) y[dp + c] = scale * S[j * lds + c];
    return;
  }
  float nrm = 0.f;
  if (j < n) {
    for (int64_t c = lane; c < ldy; c += 64) {
      float v = 0.f;
      if (c < d) {
        v = X[j * ldx + c] - mean[c];
        nrm = fmaf(v, v, nrm);
      } else if (c >= dp && c < dp + d && S != nullptr) {
        v = scale * S[j * lds + (c - dp)];
      }
      y[c] = v;
    }
  } else {
    for (int64_t c = lane; c < ldy; c += 64) y[c] = 0.f;
  }
  nrm = warp_sum(nrm);
  if (lane == 0) norms[j] = nrm;
}

// -------------------------------------------------------------- scores ----
__global__ __launch_bounds__(256) void score_gaussian_kernel(const float* __restrict__ X,
                                                             int64_t ldx, int64_t n, int64_t d,
                                                             const float* __restrict__ mu,
                                                             const float* __restrict__ lam,
                                                             float scale, float* __restrict__ S,
                                                             int64_t lds) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n * d) return;
  const int64_t j = t / d, c = t % d;
  S[j * lds + c] = scale * (-lam[c] * (X[j * ldx + c] - mu[c]));
}

// d/dx log(1/3 N(x;-2,1) + 1/3 N(x;2,1)) = -(w1 (x+2) + w2 (x-2)),  with
// (w1, w2) the softmax of (-(x+2)^2/2, -(x-2)^2/2): stable for any x.
__global__ __launch_bounds__(256) void score_gmm_kernel(const float* __restrict__ X, int64_t ldx,
                                                        int64_t n, int64_t d, float scale,
                                                        float* __restrict__ S, int64_t lds) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n * d) return;
  const int64_t j = t / d, c = t % d;
  const float x = X[j * ldx + c];
  const float a = -0.5f * (x + 2.f) * (x + 2.f), b = -0.5f * (x - 2.f) * (x - 2.f);
  const float m = fmaxf(a, b);
  const float ea = __expf(a - m), eb = __expf(b - m);
  const float s = -(ea * (x + 2.f) + eb * (x - 2.f)) / (ea + eb);
  S[j * lds + c] = scale * s;
}

__global__ void set_bandwidth_kernel(dsvgd_select_state* st, float h) {
  st->h = h;
  st->inv_h = 1.f / h;
  st->median = NAN;
}

}  // namespace dsvgd

using namespace dsvgd;

extern "C" {

int dsvgd_abi_version(void) { return DSVGD_ABI_VERSION; }
const char* dsvgd_last_error(void) { return g_err; }
size_t dsvgd_select_state_bytes(void) { return sizeof(dsvgd_select_state); }
int64_t dsvgd_pad128(int64_t n) { return roundup(n < 1 ? 1 : n, 128); }
int64_t dsvgd_dp(int64_t d) { return roundup(d < 1 ? 1 : d, 32); }
int64_t dsvgd_ldy(int64_t dp) {
  // phi column tile: 128 (2dp<=128), 256 (<=256), else multiples of 512
  const int64_t w = 2 * dp;
  if (w <= 128) return 128;
  if (w <= 256) return 256;
  return roundup(w, 512);
}

size_t dsvgd_colmean_workspace_floats(int64_t n, int64_t d) {
  return (size_t)((n + kMeanRows - 1) / kMeanRows) * (size_t)d;
}

int dsvgd_colmean(const float* X, int64_t ldx, int64_t n, int64_t d, float* partial, float* mean,
                  void* stream) {
  DSVGD_REQUIRE(X && partial && mean, "null pointer");
  DSVGD_REQUIRE(n > 0 && d > 0 && ldx >= d, "sizes");
  const int64_t nb = (n + kMeanRows - 1) / kMeanRows;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(colsum_partial_kernel, dim3(nb, (d + 63) / 64), dim3(256), 0, s, X, ldx, n,
                     d, partial);
  int rc = check_launch("colsum_partial");
  if (rc) return rc;
  hipLaunchKernelGGL(colsum_final_kernel, dim3((d + 63) / 64), dim3(256), 0, s, partial, nb, n,
                     d, mean);
  return check_launch("colsum_final");
}

int dsvgd_colcenter(const float* X, int64_t ldx, int64_t n, int64_t d, float* center,
                    void* stream) {
  DSVGD_REQUIRE(X && center, "null pointer");
  DSVGD_REQUIRE(n > 0 && d > 0 && ldx >= d, "sizes");
  DSVGD_REQUIRE(d <= 0x7fffffff, "d too large for the grid");
  hipLaunchKernelGGL(colcenter_kernel, dim3((unsigned)d), dim3(256), 0, (hipStream_t)stream, X, ldx,
                     n, center);
  return check_launch("colcenter");
}

int64_t dsvgd_pack_blocks(int64_t rows_pad) {
  const int64_t r = pack_rows_per_block(rows_pad);
  return (rows_pad + r - 1) / r;
}
int64_t dsvgd_pack_max_ldy(void) { return 256 * kPackQ; }

int dsvgd_pack_h2(const float* X, int64_t ldx, const float* S, int64_t lds, float score_scale,
                  const float* mean, int64_t n, int64_t d, int64_t rows_pad, float* Y, int64_t ldy,
                  float* norms, uint32_t* partial, uint32_t* gmax, float* rowscale,
                  void* stream) {
  DSVGD_REQUIRE(Y && (X ? (mean && norms) : (S != nullptr)), "null pointer");
  DSVGD_REQUIRE(!partial == !gmax, "partial and gmax go together");
  DSVGD_REQUIRE(!rowscale || ldy <= dsvgd_pack_max_ldy(), "row scales need ldy <= 2048");
  DSVGD_REQUIRE(n > 0 && d > 0 && (!X || ldx >= d) && rows_pad >= n, "sizes");
  const int64_t dp = dsvgd_dp(d);
  DSVGD_REQUIRE(ldy >= 2 * dp && ldy % 4 == 0, "ldy");
  DSVGD_REQUIRE(!partial || ldy <= dsvgd_pack_max_ldy(), "column maxima need ldy <= 2048");
  DSVGD_REQUIRE(((uintptr_t)Y & 15) == 0, "Y: 16-byte alignment");
  DSVGD_REQUIRE(S == nullptr || lds >= d, "lds");
  hipStream_t s = (hipStream_t)stream;
  if (ldy > dsvgd_pack_max_ldy()) {
    hipLaunchKernelGGL(pack_wide_kernel, dim3((rows_pad + 3) / 4), dim3(256), 0, s, X, ldx, S,
                       lds, score_scale, mean, n, d, rows_pad, dp, Y, ldy, norms);
    return check_launch("pack_wide");
  }
  const bool vx = X && ((uintptr_t)X & 15) == 0 && ldx % 4 == 0 && ((uintptr_t)mean & 15) == 0;
  const bool vs = S && ((uintptr_t)S & 15) == 0 && lds % 4 == 0;
  const dim3 grid((unsigned)dsvgd_pack_blocks(rows_pad));
  const size_t lds_bytes = partial ? 4 * sizeof(uint32_t) * (size_t)ldy : 0;
#define DSVGD_PACK_Q(VX, VS, NQ)                                                              \
  hipLaunchKernelGGL((pack_kernel<VX, VS, NQ>), grid, dim3(256), lds_bytes, s, X, ldx, S, lds, \
                     score_scale, mean, n, d, rows_pad, dp, Y, ldy, norms, partial, gmax,      \
                     rowscale)
#define DSVGD_PACK(VX, VS)                                                                    \
  if (ldy <= 256) DSVGD_PACK_Q(VX, VS, 1);                                                    \
  else if (ldy <= 512) DSVGD_PACK_Q(VX, VS, 2);                                               \
  else if (ldy <= 1024) DSVGD_PACK_Q(VX, VS, 4);                                              \
  else DSVGD_PACK_Q(VX, VS, 8);
  if (vx && vs) { DSVGD_PACK(true, true) }
  else if (vx) { DSVGD_PACK(true, false) }
  else if (vs) { DSVGD_PACK(false, true) }
  else { DSVGD_PACK(false, false) }
#undef DSVGD_PACK
#undef DSVGD_PACK_Q
  return check_launch("pack");
}

int dsvgd_pack(const float* X, int64_t ldx, const float* S, int64_t lds, float score_scale,
               const float* mean, int64_t n, int64_t d, int64_t rows_pad, float* Y, int64_t ldy,
               float* norms, void* stream) {
  return dsvgd_pack_h2(X, ldx, S, lds, score_scale, mean, n, d, rows_pad, Y, ldy, norms, nullptr,
                       nullptr, nullptr, stream);
}

int dsvgd_score_gaussian(const float* X, int64_t ldx, int64_t n, int64_t d, const float* mu,
                         const float* lam, float scale, float* S, int64_t lds, void* stream) {
  DSVGD_REQUIRE(X && mu && lam && S, "null pointer");
  DSVGD_REQUIRE(n > 0 && d > 0 && ldx >= d && lds >= d, "sizes");
  hipLaunchKernelGGL(score_gaussian_kernel, dim3((n * d + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, X, ldx, n, d, mu, lam, scale, S, lds);
  return check_launch("score_gaussian");
}

int dsvgd_score_gmm(const float* X, int64_t ldx, int64_t n, int64_t d, float scale, float* S,
                    int64_t lds, void* stream) {
  DSVGD_REQUIRE(X && S, "null pointer");
  DSVGD_REQUIRE(n > 0 && d > 0 && ldx >= d && lds >= d, "sizes");
  hipLaunchKernelGGL(score_gmm_kernel, dim3((n * d + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, X, ldx, n, d, scale, S, lds);
  return check_launch("score_gmm");
}

int dsvgd_set_bandwidth(dsvgd_select_state* st, float h, void* stream) {
  DSVGD_REQUIRE(st, "null state");
  DSVGD_REQUIRE(h > 0.f && std::isfinite(h), "bandwidth must be finite and > 0");
  hipLaunchKernelGGL(set_bandwidth_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, st, h);
  return check_launch("set_bandwidth");
}

int dsvgd_set_cu_reserve(int cus) { return dsvgd::set_cu_reserve(cus); }

}  // extern "C"
