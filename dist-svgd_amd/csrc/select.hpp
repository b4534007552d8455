// select.hpp -- device-side accounting the distance kernels do for the exact
// median select (lower median, k = (n^2-1)//2 over the full
// n x n matrix).  Two modes, chosen by the caller per step:
//
//  kSelHist     the epilogue accumulates radix digit 1 (key bits 31..21) of
//               every valid entry; passes 2 and 3 then stream D again.
//  kSelBracket  a 2^18-pair sample has fixed lo <= median <= hi (6 sigma of
//               the sample rank); the epilogue counts entries < lo and
//               compacts the entries in [lo, hi] (~1 %) into a candidate
//               buffer, so the three radix passes read the candidates, not D.
//               Exactness is checked on device (below <= k < below + ncand);
//               a miss or an overflow falls back to the passes over D.
#pragma once
#include "common.hpp"

namespace dsvgd {

enum SelMode { kSelNone = 0, kSelHist = 1, kSelBracket = 2 };

// Per-lane digit-1 histogram with an 8-bin register window (a tile's
// distances cluster within a factor 2-4): packed 8 x 8-bit counters per lane,
// out-of-window keys go to the LDS histogram.  Counts per lane <= 128.
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
      if (lane == 0 && c > 0 && bin >= 0 && bin < DSVGD_RADIX_BINS)
        atomicAdd(&shist[bin], (uint32_t)c);
    }
  }
};

__device__ __forceinline__ void flush_block_hist(const uint32_t* shist, dsvgd_select_state* st) {
  for (int b = threadIdx.x; b < DSVGD_RADIX_BINS; b += blockDim.x) {
    const uint32_t c = shist[b];
    if (c) atomicAdd((unsigned long long*)&st->hist[b], (unsigned long long)c);
  }
}

// histogram of a lane's NV values (+inf = invalid, skipped), weight w
template <int NV>
__device__ __forceinline__ void hist_account(WindowHist& wh, const float (&v)[NV], uint32_t w,
                                             uint32_t* shist) {
#pragma unroll
  for (int i = 0; i < NV; ++i)
    if (v[i] != INFINITY) wh.add(v[i], w, shist);
}

__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t x, uint32_t& total) {
  const int lane = threadIdx.x & 63;
  uint32_t inc = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  total = __shfl(inc, 63, 64);
  return inc - x;
}

// bracket accounting of a lane's NV values (+inf = invalid), each of weight w
// (w = 2 for the mirrored tiles of the symmetric Gram): one atomic per wave.
template <int NV>
__device__ __forceinline__ void bracket_account(const float (&v)[NV], uint32_t w,
                                                dsvgd_select_state* __restrict__ st,
                                                float* __restrict__ cand) {
  const float lo = st->lo, hi = st->hi;
  uint32_t below = 0, inb = 0;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    below += (v[i] < lo) ? w : 0u;
    inb += (v[i] >= lo && v[i] <= hi) ? w : 0u;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) below += __shfl_xor(below, o, 64);
  uint32_t total;
  const uint32_t off = wave_excl_scan(inb, total);
  const int lane = threadIdx.x & 63;
  if (lane == 0 && below)
    atomicAdd((unsigned long long*)&st->below, (unsigned long long)below);
  if (total == 0) return;
  unsigned long long base = 0;
  if (lane == 0) base = atomicAdd((unsigned long long*)&st->ncand, (unsigned long long)total);
  base = __shfl(base, 0, 64);
  const unsigned long long cap = st->cand_cap;
  unsigned long long pos = base + off;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    if (v[i] >= lo && v[i] <= hi) {
      for (uint32_t r = 0; r < w; ++r, ++pos)
        if (pos < cap) cand[pos] = v[i];
    }
  }
}

}  // namespace dsvgd
