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

// ---- bracketed mode --------------------------------------------------------
// Phase 1 (while storing D): each lane counts its values < lo and in [lo, hi].
// Phase 2 (block-collective): one returning atomic per BLOCK on the list
// counter of the block's candidate list (256 lists: no counter sees more than
// a few hundred atomics per launch -- same-address float/int atomics from every
// CU serialise, MI355X_MICROARCH.md "Global float atomics", contention row).
// Phase 3: each lane re-derives its values (deterministic) and writes the
// in-bracket ones at its reserved positions.
struct BracketCounter {
  uint32_t below = 0, inb = 0;
  uint64_t mask = 0;  // bit i: value i of this lane is in [lo, hi]
  float lo = 0.f, hi = -1.f;
  __device__ __forceinline__ void load(const dsvgd_select_state* st) {
    lo = st->lo;
    hi = st->hi;
  }
  __device__ __forceinline__ void count(float v, uint32_t w, int idx) {
    const bool in = v >= lo && v <= hi;
    below += (v < lo) ? w : 0u;
    inb += in ? w : 0u;
    mask |= (uint64_t)in << idx;
  }
};

struct BracketWriter {
  float* dst = nullptr;
  unsigned long long pos = 0, cap = 0;
  float lo = 0.f, hi = -1.f;
  __device__ __forceinline__ void put(float v, uint32_t w) {
    for (uint32_t r = 0; r < w; ++r, ++pos)
      if (pos < cap) dst[pos] = v;
  }
};

constexpr int kCandLists = DSVGD_CAND_LISTS;

// sred: LDS scratch of >= 2*NW + 4 u32 (NW = waves per block).  Every thread
// of the block must call it.
template <int NW>
__device__ __forceinline__ BracketWriter bracket_reserve(const BracketCounter& bc,
                                                         dsvgd_select_state* __restrict__ st,
                                                         float* __restrict__ cand, int list,
                                                         uint32_t* sred) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t below = bc.below;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) below += __shfl_xor(below, o, 64);
  uint32_t wtotal;
  const uint32_t off = wave_excl_scan(bc.inb, wtotal);
  if (lane == 0) {
    sred[wave] = wtotal;
    sred[NW + wave] = below;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t run = 0, bsum = 0;
    for (int w = 0; w < NW; ++w) {
      const uint32_t t = sred[w];
      sred[w] = run;
      run += t;
      bsum += sred[NW + w];
    }
    unsigned long long base = 0;
    if (run) base = atomicAdd((unsigned long long*)&st->list_cnt[list], (unsigned long long)run);
    if (bsum) atomicAdd((unsigned long long*)&st->list_below[list], (unsigned long long)bsum);
    sred[2 * NW] = (uint32_t)(base & 0xffffffffull);
    sred[2 * NW + 1] = (uint32_t)(base >> 32);
  }
  __syncthreads();
  BracketWriter bw;
  const unsigned long long cap = st->cand_cap / kCandLists;
  bw.dst = cand + (unsigned long long)list * cap;
  bw.cap = cap;
  bw.pos = (((unsigned long long)sred[2 * NW + 1] << 32) | sred[2 * NW]) + sred[wave] + off;
  bw.lo = bc.lo;
  bw.hi = bc.hi;
  return bw;
}

}  // namespace dsvgd
