// sqdist.hip -- pairwise squared distances on MFMA + the exact radix select
// that turns them into the median-heuristic bandwidth.
//
// Roofline (per 128x128 output tile, d = dp): 2*128*128*dp MFMA flop against
// 64 KiB of D written -- MFMA-bound for dp >= 64 (2 dp flop per byte written
// vs 157 TF / 8 TB/s ~ 20 flop/B); the radix passes are pure HBM streams of D.
#include <cmath>

#include "gemm_tiles.hpp"

namespace dsvgd {

using GramTile = NTTile<2, 2, 2, 2>;  // 128 x 128 block, 4 waves of 64 x 64

// Per-lane radix-digit-1 histogram with an 8-bin register window: the bins of
// one tile's distances cluster within a factor ~2-4, so each lane counts them
// in a packed 64-bit register (8 x 8-bit counters) and only out-of-window keys
// hit the LDS histogram (an LDS atomic per element with 64 lanes on a few bins
// serialises the whole epilogue).  Counts per lane <= 128 (64 values x weight 2).
struct WindowHist {
  uint64_t packed = 0;
  int base = 0;
  __device__ __forceinline__ void init(float first) {
    base = __builtin_amdgcn_readfirstlane((int)(__float_as_uint(first) >> 21)) - 3;
  }
  __device__ __forceinline__ void add(float v, uint32_t w, uint32_t* shist) {
    const int bin = (int)(__float_as_uint(v) >> 21);
    const unsigned o = (unsigned)(bin - base);
    if (o < 8u)
      packed += (uint64_t)w << (8u * o);
    else
      atomicAdd(&shist[bin], w);
  }
  __device__ __forceinline__ void flush(uint32_t* shist) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 0; o < 8; ++o) {
      int c = (int)((packed >> (8 * o)) & 0xFFull);
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
      const int bin = base + o;
      if (lane == 0 && c > 0 && bin >= 0 && bin < DSVGD_RADIX_BINS) atomicAdd(&shist[bin], (uint32_t)c);
    }
  }
};

__device__ __forceinline__ void flush_block_hist(const uint32_t* shist, dsvgd_select_state* st) {
  for (int b = threadIdx.x; b < DSVGD_RADIX_BINS; b += 256) {
    const uint32_t c = shist[b];
    if (c) atomicAdd((unsigned long long*)&st->hist[b], (unsigned long long)c);
  }
}

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

// D (panel layout, m_pad x n_pad) for rows [row0, row0+m) of Y against rows
// [0,n) on MFMA.  SYM (m == n, row0 == 0): only tiles bi <= bj are computed,
// off-diagonal ones are stored twice (tile + transpose) and counted twice.
template <bool SYM>
__global__ __launch_bounds__(256) void sqdist_kernel(const float* __restrict__ Y, int64_t ldy,
                                                     const float* __restrict__ norms, int64_t row0,
                                                     int64_t m, int64_t n, int64_t n_pad, int dp,
                                                     float* __restrict__ D,
                                                     dsvgd_select_state* __restrict__ st) {
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
  if (st)
    for (int b = threadIdx.x; b < DSVGD_RADIX_BINS; b += 256) shist[b] = 0u;

  GramTile tile;
  tile.run(Y + (row0 + i0) * ldy, ldy, Y + j0 * ldy, ldy, dp, smem);

  for (int t = threadIdx.x; t < GramTile::BM + GramTile::BN; t += 256)
    snorm[t] = t < GramTile::BM ? norms[row0 + i0 + t] : norms[j0 + t - GramTile::BM];
  __syncthreads();

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w >> 1, wn = w & 1;
  const uint32_t weight = mirror ? 2u : 1u;
  WindowHist wh;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      const int cl = wn * 64 + ni * 32 + (lane & 31);
      const int64_t gj = j0 + cl;
      const float nj = snorm[GramTile::BM + cl];
      float vals[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rl = wm * 64 + mi * 32 + c_row(r, lane);
        const int64_t gi = i0 + rl;
        float v;
        if (gi < m && gj < n)
          v = (row0 + gi == gj) ? 0.f : fmaxf(0.f, (snorm[rl] + nj) - 2.f * tile.acc[mi][ni][r]);
        else
          v = INFINITY;
        vals[r] = v;
        D[panel_off(gi, gj, n_pad)] = v;
      }
      if (st) {
        if (mi == 0 && ni == 0) wh.init(vals[0]);
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (vals[r] != INFINITY) wh.add(vals[r], weight, shist);
      }
      if (mirror) {  // D[j][i]: 4 consecutive i per register quad -> 16-byte stores
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int64_t ci = i0 + wm * 64 + mi * 32 + 8 * q + 4 * (lane >> 5);
          f32x4 v4 = {vals[4 * q], vals[4 * q + 1], vals[4 * q + 2], vals[4 * q + 3]};
          *reinterpret_cast<f32x4*>(D + panel_off(gj, ci, n_pad)) = v4;
        }
      }
    }
  if (st) {
    wh.flush(shist);
    __syncthreads();
    flush_block_hist(shist, st);
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
                                                            float* __restrict__ D,
                                                            dsvgd_select_state* __restrict__ st) {
  __shared__ __attribute__((aligned(16))) float sA[kDirectMaxD][128];
  __shared__ __attribute__((aligned(16))) float sB[kDirectMaxD][128];
  __shared__ uint32_t shist[DSVGD_RADIX_BINS];
  const int t = threadIdx.x;
  const int64_t i0 = (int64_t)blockIdx.y * 128, j0 = (int64_t)blockIdx.x * 128;
  if (st)
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
  if (st) {
    const bool ok = (i0 + ty * 8 < m) && (j0 + tx * 8 < n);
    wh.init(ok ? acc[0][0] : INFINITY);
  }
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    const int64_t gi = i0 + ty * 8 + a;
    float v[8];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const int64_t gj = j0 + tx * 8 + b;
      const bool ok = gi < m && gj < n;
      v[b] = ok ? acc[a][b] : INFINITY;
      if (st && ok) wh.add(v[b], 1u, shist);
    }
    float* dst = D + panel_off(gi, j0 + tx * 8, n_pad);
    *reinterpret_cast<f32x4*>(dst) = f32x4{v[0], v[1], v[2], v[3]};
    *reinterpret_cast<f32x4*>(dst + 4) = f32x4{v[4], v[5], v[6], v[7]};
  }
  if (st) {
    wh.flush(shist);
    __syncthreads();
    flush_block_hist(shist, st);
  }
}

// ---------------------------------------------------------- radix select --
// keys: the fp32 bit patterns of D >= 0 (monotone as uint32).  +inf pads and
// NaN are never counted.  digit 1 = bits 31..21, 2 = 20..10, 3 = 9..0.
__device__ __forceinline__ void digit_of(int pass, uint32_t& shift, uint32_t& mask,
                                         uint32_t& hishift) {
  if (pass == 1) {
    shift = 21; mask = 0x7FFu; hishift = 32;
  } else if (pass == 2) {
    shift = 10; mask = 0x7FFu; hishift = 21;
  } else {
    shift = 0; mask = 0x3FFu; hishift = 10;
  }
}

__global__ __launch_bounds__(256) void radix_hist_kernel(const float* __restrict__ D, int64_t count4,
                                                         int pass,
                                                         dsvgd_select_state* __restrict__ st) {
  __shared__ uint32_t shist[DSVGD_RADIX_BINS];
  for (int b = threadIdx.x; b < DSVGD_RADIX_BINS; b += 256) shist[b] = 0u;
  uint32_t shift, mask, hishift;
  digit_of(pass, shift, mask, hishift);
  const uint32_t prefix = st->prefix;
  const uint32_t want = hishift >= 32 ? 0u : (prefix >> hishift);
  __syncthreads();
  const f32x4* D4 = reinterpret_cast<const f32x4*>(D);
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < count4;
       q += (int64_t)gridDim.x * 256) {
    const f32x4 v = D4[q];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t key = __float_as_uint(v[e]);
      if (key >= 0x7F800000u) continue;  // +inf pad / NaN
      const uint32_t hi = hishift >= 32 ? 0u : (key >> hishift);
      if (hi == want) atomicAdd(&shist[(key >> shift) & mask], 1u);
    }
  }
  __syncthreads();
  flush_block_hist(shist, st);
}

// One block: find the bin that holds rank k, fix its digit, clear the bins.
__global__ __launch_bounds__(256) void radix_pick_kernel(dsvgd_select_state* __restrict__ st,
                                                         int pass) {
  __shared__ unsigned long long part[256];
  __shared__ unsigned long long excl[256];
  const int t = threadIdx.x;
  uint32_t shift, mask, hishift;
  digit_of(pass, shift, mask, hishift);
  const int nb = (int)mask + 1;            // 2048 or 1024 bins
  const int per = nb / 256;                // 8 or 4 bins per thread
  unsigned long long loc[8];
  unsigned long long s = 0;
  for (int u = 0; u < per; ++u) {
    loc[u] = st->hist[t * per + u];
    s += loc[u];
  }
  part[t] = s;
  __syncthreads();
  if (t == 0) {
    unsigned long long run = 0;
    for (int q = 0; q < 256; ++q) {
      excl[q] = run;
      run += part[q];
    }
  }
  __syncthreads();
  const unsigned long long k = st->k;
  const unsigned long long lo = excl[t];
  __syncthreads();
  if (k >= lo && k < lo + part[t]) {
    unsigned long long run = lo;
    for (int u = 0; u < per; ++u) {
      if (k < run + loc[u]) {
        const uint32_t digit = (uint32_t)(t * per + u);
        const uint32_t prefix = st->prefix | (digit << shift);
        st->prefix = prefix;
        st->k = k - run;
        st->passes_done = (uint32_t)pass;
        if (pass == 3) {
          const float med = __uint_as_float(prefix);
          const double nt = (double)st->n_total;
          float h = 1.f;
          if (med > 0.f && nt > 1.0) h = (float)((double)med / log(nt));
          st->median = med;
          st->h = h;
          st->inv_h = 1.f / h;
        }
        break;
      }
      run += loc[u];
    }
  }
  for (int u = 0; u < 8; ++u) st->hist[t * 8 + u] = 0ull;  // clear all 2048 bins
}

__global__ void select_init_kernel(dsvgd_select_state* st, int64_t n_total) {
  const int t = threadIdx.x;
  for (int b = t; b < DSVGD_RADIX_BINS; b += blockDim.x) st->hist[b] = 0ull;
  if (t == 0) {
    const unsigned long long nn = (unsigned long long)n_total * (unsigned long long)n_total;
    st->k = (nn - 1ull) / 2ull;
    st->n_total = (unsigned long long)n_total;
    st->prefix = 0u;
    st->passes_done = 0u;
    st->median = NAN;
    st->h = NAN;
    st->inv_h = NAN;
  }
}

}  // namespace dsvgd

using namespace dsvgd;

extern "C" {

int dsvgd_sqdist(const float* Y, int64_t ldy, const float* norms, int64_t row0, int64_t m,
                 int64_t n, int64_t d, float* D, int64_t ldd, dsvgd_select_state* st,
                 void* stream) {
  DSVGD_REQUIRE(Y && norms && D, "null pointer");
  DSVGD_REQUIRE(m > 0 && n > 0 && row0 >= 0 && d > 0, "sizes");
  const int64_t dp = roundup(d, 32);
  DSVGD_REQUIRE(ldy >= dp && ldy % 4 == 0, "ldy < roundup(d,32)");
  const int64_t m_pad = roundup(m, 128), n_pad = roundup(n, 128);
  DSVGD_REQUIRE(ldd == n_pad, "ldd must equal roundup(n,128) (panel layout)");
  DSVGD_REQUIRE(((uintptr_t)Y & 15) == 0 && ((uintptr_t)D & 15) == 0, "16-byte alignment");
  DSVGD_REQUIRE(m_pad / 128 <= 65535, "too many row tiles");
  hipStream_t s = (hipStream_t)stream;
  if (d <= kDirectMaxD) {
    hipLaunchKernelGGL(sqdist_direct_kernel, dim3(n_pad / 128, m_pad / 128), dim3(256), 0, s, Y,
                       ldy, row0, m, n, n_pad, (int)d, D, st);
    return check_launch("sqdist_direct");
  }
  if (m == n && row0 == 0) {
    const int64_t T = n_pad / 128;
    hipLaunchKernelGGL((sqdist_kernel<true>), dim3(T * (T + 1) / 2), dim3(256), 0, s, Y, ldy,
                       norms, row0, m, n, n_pad, (int)dp, D, st);
  } else {
    hipLaunchKernelGGL((sqdist_kernel<false>), dim3(n_pad / 128, m_pad / 128), dim3(256), 0, s, Y,
                       ldy, norms, row0, m, n, n_pad, (int)dp, D, st);
  }
  return check_launch("sqdist");
}

int dsvgd_select_init(dsvgd_select_state* st, int64_t n_total, void* stream) {
  DSVGD_REQUIRE(st && n_total > 0, "args");
  hipLaunchKernelGGL(select_init_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, st, n_total);
  return check_launch("select_init");
}

int dsvgd_radix_hist(const float* D, int64_t ldd, int64_t m, int64_t n, int pass,
                     dsvgd_select_state* st, void* stream) {
  DSVGD_REQUIRE(D && st, "null pointer");
  DSVGD_REQUIRE(pass >= 1 && pass <= 3, "pass must be 1..3");
  const int64_t m_pad = roundup(m, 128), n_pad = roundup(n, 128);
  DSVGD_REQUIRE(ldd == n_pad, "ldd must equal roundup(n,128) (panel layout)");
  const int64_t count4 = m_pad * n_pad / 4;
  int64_t blocks = (count4 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(radix_hist_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, D, count4,
                     pass, st);
  return check_launch("radix_hist");
}

int dsvgd_radix_pick(dsvgd_select_state* st, int pass, void* stream) {
  DSVGD_REQUIRE(st, "null state");
  DSVGD_REQUIRE(pass >= 1 && pass <= 3, "pass must be 1..3");
  hipLaunchKernelGGL(radix_pick_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, st, pass);
  return check_launch("radix_pick");
}

}  // extern "C"
