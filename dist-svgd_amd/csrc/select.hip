// select.hip -- exact k-th order statistic of the squared distances (the
// median-heuristic bandwidth; absent from the reference, pinned in SURVEY.md
// a18) as an LSD-free radix select over the fp32 key bits (monotone as uint32
// for D >= 0): digit 1 = bits 31..21, 2 = 20..10, 3 = 9..0.  Each pass is a
// histogram (LDS per block, u64 global bins, all-reducible across ranks)
// followed by a one-block pick; no host synchronisation anywhere.
//
// Sources of a pass: the D panel buffer (HBM stream, 4 B per entry per pass)
// or, in bracketed mode, the candidate buffer the distance epilogue compacted
// (~1 % of D).  The choice is made on device (st->fallback).
#include <algorithm>
#include <cmath>

#include "gemm_tiles.hpp"

#include "select.hpp"

namespace dsvgd {

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

__device__ __forceinline__ void hist_key(uint32_t key, uint32_t want, uint32_t shift,
                                         uint32_t mask, uint32_t hishift, uint32_t* shist,
                                         uint32_t w = 1u) {
  if (key >= 0x7F800000u) return;  // +inf pad / NaN
  const uint32_t hi = hishift >= 32 ? 0u : (key >> hishift);
  if (hi == want) atomicAdd(&shist[(key >> shift) & mask], w);
}

// hist_key for values that pile into few bins (the candidates of a bracket:
// all within [lo, hi], so digit 1 -- often digit 2 -- is the same for most of
// a wave): the lanes whose bin equals the first active lane's add with one
// atomic, the rest one each.
__device__ __forceinline__ void hist_key_agg(uint32_t key, uint32_t want, uint32_t shift,
                                             uint32_t mask, uint32_t hishift, uint32_t* shist,
                                             uint32_t w) {
  const uint32_t hi = hishift >= 32 ? 0u : (key >> hishift);
  const bool ok = key < 0x7F800000u && hi == want;
  const uint32_t bin = (key >> shift) & mask;
  const uint32_t b0 = __builtin_amdgcn_readfirstlane(bin);
  const bool agg = ok && bin == b0;
  const uint64_t m = __ballot(agg);
  if (agg) {
    if ((uint32_t)(threadIdx.x & 63) == (uint32_t)(__ffsll((long long)m) - 1))
      atomicAdd(&shist[b0], w * (uint32_t)__popcll(m));
  } else if (ok) {
    atomicAdd(&shist[bin], w);
  }
}

// workgroups walking the candidate slots (4096 -> 1024: S = 8 pass 0.058 ->
// 0.037 ms, config C -8.6 %; 512 slower at S = 1)
constexpr int kCandBlocks = 1024;

// count: entries of D (any order); cand: optional candidate buffer used
// instead of D when st->fallback == 0 (bracketed mode).
// sym_npad > 0: D is a symmetric n_pad x n_pad matrix stored as its
// upper-triangle 128 x 128 tiles only (panel layout; dsvgd_sqdist_x3 with
// layout 1): a panel of tile (I, J) counts 0x (J < I), 1x (J == I), 2x (J > I).
__global__ __launch_bounds__(256) void radix_hist_kernel(const float* __restrict__ D, int64_t count,
                                                         const float* __restrict__ cand, int pass,
                                                         dsvgd_select_state* __restrict__ st,
                                                         int64_t sym_npad,
                                                         const uint8_t* __restrict__ wmap = nullptr) {
  __shared__ uint32_t shist[DSVGD_RADIX_BINS];
  if (st->passes_done >= (uint32_t)pass) return;  // digit fixed by bracket_check
  for (int b = threadIdx.x; b < DSVGD_RADIX_BINS; b += 256) shist[b] = 0u;
  uint32_t shift, mask, hishift;
  digit_of(pass, shift, mask, hishift);
  const uint32_t prefix = st->prefix;
  const uint32_t want = hishift >= 32 ? 0u : (prefix >> hishift);
  const bool use_cand = cand != nullptr && st->fallback == 0u;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int64_t t0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (use_cand) {  // one wave per candidate slot (weight 2: a mirrored tile)
    // (measured: a block per slot with four loads in flight, or at most 256
    // workgroups, were both slower -- 0.14 / 0.69 ms vs 0.10 ms per pass)
    const int64_t ns = (int64_t)st->nslots, cap = (int64_t)st->slot_cap;
    const uint32_t* cnt = reinterpret_cast<const uint32_t*>(cand);
    const float* data = cand + 2 * ns;
    const int lane = threadIdx.x & 63;
    // at most kCandBlocks workgroups walk the slots (each flushes its bins
    // with global atomics onto the few bins the candidates share)
    const int64_t nb = min((int64_t)gridDim.x, (int64_t)kCandBlocks);
    const int64_t nw = nb * 4;
    // a slot holds a few hundred candidates: a wave takes two slots at a
    // time and loads the first 4 x 64 values of both together (padding lanes
    // read as +inf, which hist_key skips), so it is not one dependent
    // count -> data -> atomics round trip per 64 values
    constexpr uint32_t kInf = 0x7F800000u;
    int64_t sl = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    for (; blockIdx.x < nb && sl < ns; sl += 2 * nw) {
      const int64_t s2 = sl + nw;
      const uint32_t ca = cnt[sl], cb = s2 < ns ? cnt[s2] : 0u;
      const uint32_t wa = (ca & DSVGD_SLOT_WEIGHT2) ? 2u : 1u, wb = (cb & DSVGD_SLOT_WEIGHT2) ? 2u : 1u;
      const int64_t na = min((int64_t)(ca & ~DSVGD_SLOT_WEIGHT2), cap);
      const int64_t nb2 = min((int64_t)(cb & ~DSVGD_SLOT_WEIGHT2), cap);
      const float* sa = data + sl * cap;
      const float* sb = data + s2 * cap;
      uint32_t ka[4], kb[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t q = lane + 64 * u;
        ka[u] = q < na ? __float_as_uint(sa[q]) : kInf;
        kb[u] = q < nb2 ? __float_as_uint(sb[q]) : kInf;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) hist_key(ka[u], want, shift, mask, hishift, shist, wa);
#pragma unroll
      for (int u = 0; u < 4; ++u) hist_key(kb[u], want, shift, mask, hishift, shist, wb);
      for (int64_t q = lane + 256; q < na; q += 64)
        hist_key(__float_as_uint(sa[q]), want, shift, mask, hishift, shist, wa);
      for (int64_t q = lane + 256; q < nb2; q += 64)
        hist_key(__float_as_uint(sb[q]), want, shift, mask, hishift, shist, wb);
    }
  } else if (sym_npad > 0) {  // panel by panel (2048 floats = 2 float4 per thread)
    const int64_t pcols = sym_npad >> 4, npanels = count / kPanelElems;
    const f32x4* D4 = reinterpret_cast<const f32x4*>(D);
    for (int64_t pnl = blockIdx.x; pnl < npanels; pnl += gridDim.x) {
      const int64_t I = pnl / pcols, J = (pnl % pcols) >> 3;
      // wmap: the pair-split layout's tile weights; else the symmetric rule
      const uint32_t w = wmap ? (uint32_t)wmap[I * (pcols >> 3) + J] : (J < I ? 0u : J == I ? 1u : 2u);
      if (w == 0u) continue;  // block-uniform
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 v = D4[pnl * (kPanelElems / 4) + h * 256 + threadIdx.x];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          hist_key(__float_as_uint(v[e]), want, shift, mask, hishift, shist, w);
      }
    }
  } else {
    const int64_t c4 = count >> 2;
    const f32x4* D4 = reinterpret_cast<const f32x4*>(D);
    for (int64_t q = t0; q < c4; q += stride) {
      const f32x4 v = D4[q];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        hist_key(__float_as_uint(v[e]), want, shift, mask, hishift, shist);
    }
    for (int64_t q = 4 * c4 + t0; q < count; q += stride)
      hist_key(__float_as_uint(D[q]), want, shift, mask, hishift, shist);
  }
  __syncthreads();
  flush_block_hist(shist, st);
}

template <bool COHERENT>
__device__ __forceinline__ unsigned long long load_bin(const uint64_t* p) {
  if constexpr (COHERENT)  // bins other workgroups of this launch just added to
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    return *p;
}

// One block of 256: find the bin of `hist` that holds rank st->k, fix its
// digit in st (prefix, remaining rank; the median and h after pass 3).
template <bool COHERENT>
__device__ void pick_digit(const uint64_t* hist, dsvgd_select_state* st, int pass,
                           unsigned long long* part) {
  const int t = threadIdx.x;
  uint32_t shift, mask, hishift;
  digit_of(pass, shift, mask, hishift);
  const int nb = (int)mask + 1;  // 2048 or 1024 bins
  const int per = nb / 256;      // 8 or 4 bins per thread
  unsigned long long loc[8];
  unsigned long long s = 0;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    loc[u] = u < per ? load_bin<COHERENT>(&hist[t * per + u]) : 0ull;
    s += loc[u];
  }
  // block-wide exclusive scan of the per-thread sums: wave scans, then the
  // four wave totals (a serial 256-step loop on one lane was ~5 us per pick)
  const int lane = t & 63, wv = t >> 6;
  unsigned long long inc = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  if (lane == 63) part[wv] = inc;
  __syncthreads();
  unsigned long long lo = inc - s;  // exclusive prefix of this thread's bins
  for (int q = 0; q < wv; ++q) lo += part[q];
  const unsigned long long k = st->k;
  __syncthreads();                   // all reads of part / st->k before any pick writes
  if (k >= lo && k < lo + s) {
    unsigned long long run = lo;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (u < per && k < run + loc[u]) {
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
      run += u < per ? loc[u] : 0ull;
    }
  }
  __syncthreads();  // st and part / excl are reused by the caller
}

__device__ __forceinline__ void clear_bins(uint64_t* hist) {
#pragma unroll
  for (int u = 0; u < 8; ++u) hist[threadIdx.x * 8 + u] = 0ull;  // all 2048 bins (256 threads)
}

// One block: find the bin that holds rank k, fix its digit, clear the bins.
__global__ __launch_bounds__(256) void radix_pick_kernel(dsvgd_select_state* __restrict__ st,
                                                         int pass) {
  __shared__ unsigned long long part[4];
  if (st->passes_done >= (uint32_t)pass) return;  // digit fixed, bins untouched (zero)
  pick_digit<false>(st->hist, st, pass, part);
  clear_bins(st->hist);
}

__device__ void reset_state(dsvgd_select_state* st, unsigned long long k,
                            unsigned long long n_total) {
  st->k = k;
  st->n_total = n_total;
  st->prefix = 0u;
  st->passes_done = 0u;
  st->median = NAN;
  st->h = NAN;
  st->inv_h = NAN;
  st->fallback = 1u;
  st->below_total = 0ull;
  st->ncand_total = 0ull;
  st->overflow = 0ull;
}

__global__ void select_init_kernel(dsvgd_select_state* st, int64_t n_total, int64_t k_rank) {
  const int t = threadIdx.x;
  for (int b = t; b < DSVGD_RADIX_BINS; b += blockDim.x) st->hist[b] = 0ull;
  if (t == 0) {
    const unsigned long long nn = (unsigned long long)n_total * (unsigned long long)n_total;
    reset_state(st, k_rank >= 0 ? (unsigned long long)k_rank : (nn - 1ull) / 2ull,
                (unsigned long long)n_total);
  }
}

// bracket [lo, hi] = the medians the two sample selects found
__device__ __forceinline__ void bracket_reset(dsvgd_select_state* st, int64_t n_total, float lo,
                                              float hi, int64_t cap) {
  const int t = threadIdx.x;
  for (int b = t; b < DSVGD_RADIX_BINS; b += blockDim.x) st->hist[b] = 0ull;
  if (t == 0) {
    const unsigned long long nn = (unsigned long long)n_total * (unsigned long long)n_total;
    reset_state(st, (nn - 1ull) / 2ull, (unsigned long long)n_total);
    st->fallback = 0u;
    st->lo = lo;
    st->hi = hi;
    st->cand_cap = (unsigned long long)cap;
    st->nslots = 0ull;
    st->slot_cap = 0ull;
  }
}

__global__ void bracket_init_kernel(dsvgd_select_state* st, int64_t n_total,
                                    const dsvgd_select_state* lo_st,
                                    const dsvgd_select_state* hi_st, int64_t cap) {
  bracket_reset(st, n_total, lo_st->median, hi_st->median, cap);
}

// Sum the local candidate slots into (below_total, ncand_total, overflow),
// the int64[3] a distributed caller all-reduces before bracket_check
// (zeroed by bracket_init; integer atomics, so the sums are exact).
__global__ __launch_bounds__(256) void bracket_totals_kernel(dsvgd_select_state* st,
                                                             const float* __restrict__ cand) {
  __shared__ unsigned long long sb[256], sc[256], so[256];
  const int t = threadIdx.x;
  const int64_t ns = (int64_t)st->nslots;
  const uint64_t cap = st->slot_cap;
  const uint32_t* cnt = reinterpret_cast<const uint32_t*>(cand);
  const uint32_t* below = cnt + ns;
  unsigned long long b = 0, c = 0, o = 0;
  for (int64_t sl = (int64_t)blockIdx.x * 256 + t; sl < ns; sl += (int64_t)gridDim.x * 256) {
    const uint32_t x = cnt[sl];
    const uint64_t w = (x & DSVGD_SLOT_WEIGHT2) ? 2u : 1u;
    const uint64_t k = x & ~DSVGD_SLOT_WEIGHT2;
    b += w * below[sl];
    c += w * k;
    o += k > cap ? 1u : 0u;
  }
  sb[t] = b;
  sc[t] = c;
  so[t] = o;
  __syncthreads();
  for (int q = 128; q > 0; q >>= 1) {
    if (t < q) {
      sb[t] += sb[t + q];
      sc[t] += sc[t + q];
      so[t] += so[t + q];
    }
    __syncthreads();
  }
  if (t == 0) {
    if (sb[0]) atomicAdd((unsigned long long*)&st->below_total, sb[0]);
    if (sc[0]) atomicAdd((unsigned long long*)&st->ncand_total, sc[0]);
    if (so[0]) atomicAdd((unsigned long long*)&st->overflow, so[0]);
  }
}

// Does the bracket provably hold rank k (global totals)?  Yes -> select rank
// k - below among the candidates; no (or a list overflowed on any rank) ->
// select rank k over D itself.
__global__ void bracket_check_kernel(dsvgd_select_state* st) {
  const unsigned long long k = st->k, below = st->below_total, nc = st->ncand_total;
  if (st->overflow == 0ull && below <= k && k < below + nc) {
    st->k = k - below;
    st->fallback = 0u;
    // every candidate key lies in [bits(lo), bits(hi)]: when those share
    // digit 1 (the bracket spans ~1 % of the value, the usual case) the
    // digit-1 pass would put them all in that one bin -- fix it here and let
    // the pass-1 hist / pick launches return at once (one candidate read less)
    const uint32_t a = __float_as_uint(st->lo), b = __float_as_uint(st->hi);
    if ((a >> 21) == (b >> 21)) {
      st->prefix = a & 0xFFE00000u;
      st->passes_done = 1u;
    }
  } else {
    st->fallback = 1u;
  }
}

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

// out[p] = ||y_i - y_j||^2 (explicit differences) for s hash-chosen pairs
// (i, j) in [0,n)^2; one wave per pair, deterministic for a given seed.
// 16 lanes per sampled pair (4 pairs per wave), 16-byte row loads: a
// 256-wide row pair is one float4 pair per lane per 64 columns, so a wave
// keeps 4 pairs' gathers in flight instead of walking one pair 64 floats at
// a time.  Needs ldy % 4 == 0 and a 16-byte aligned Y (checked by the host);
// columns >= d inside the last float4 are masked out.
__global__ __launch_bounds__(256) void sample_sqdist_kernel(const float* __restrict__ Y,
                                                            int64_t ldy, int64_t n, int d,
                                                            int64_t s, uint64_t seed,
                                                            float* __restrict__ out,
                                                            int64_t p0 = 0) {
  // pairs [p0, s) (a rank's share of the sample: dsvgd_sample_sqdist_range)
  const int l16 = threadIdx.x & 15;
  for (int64_t p = p0 + (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4); p < s;
       p += (int64_t)gridDim.x * 16) {
    const uint64_t h = mix64(seed ^ (0x9e3779b97f4a7c15ull * (uint64_t)(p + 1)));
    const int64_t i = (int64_t)((h & 0xffffffffull) % (uint64_t)n);
    const int64_t j = (int64_t)((h >> 32) % (uint64_t)n);
    const float* yi = Y + i * ldy;
    const float* yj = Y + j * ldy;
    float acc = 0.f;
    for (int c = l16 * 4; c < d; c += 64) {
      const float4 a = *reinterpret_cast<const float4*>(yi + c);
      const float4 b = *reinterpret_cast<const float4*>(yj + c);
      const float d0 = a.x - b.x;
      const float d1 = c + 1 < d ? a.y - b.y : 0.f;
      const float d2 = c + 2 < d ? a.z - b.z : 0.f;
      const float d3 = c + 3 < d ? a.w - b.w : 0.f;
      acc = fmaf(d0, d0, acc);
      acc = fmaf(d1, d1, acc);
      acc = fmaf(d2, d2, acc);
      acc = fmaf(d3, d3, acc);
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (l16 == 0) out[p] = acc;
  }
}

// generic layout (any ldy / alignment): one wave per pair
__global__ __launch_bounds__(256) void sample_sqdist_any_kernel(const float* __restrict__ Y,
                                                                int64_t ldy, int64_t n, int d,
                                                                int64_t s, uint64_t seed,
                                                                float* __restrict__ out,
                                                                int64_t p0 = 0) {
  const int lane = threadIdx.x & 63;
  for (int64_t p = p0 + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); p < s;
       p += (int64_t)gridDim.x * 4) {
    const uint64_t h = mix64(seed ^ (0x9e3779b97f4a7c15ull * (uint64_t)(p + 1)));
    const int64_t i = (int64_t)((h & 0xffffffffull) % (uint64_t)n);
    const int64_t j = (int64_t)((h >> 32) % (uint64_t)n);
    const float* yi = Y + i * ldy;
    const float* yj = Y + j * ldy;
    float acc = 0.f;
    for (int c = lane; c < d; c += 64) {
      const float df = yi[c] - yj[c];
      acc = fmaf(df, df, acc);
    }
    acc = warp_sum(acc);
    if (lane == 0) out[p] = acc;
  }
}

// ---- the sample bracket in seven launches -----------------------------------
// (1 sample + 2 x (init + 3 x (hist + pick)) + bracket_init = 16
// launches before.)  The two sample selects (ranks k_lo, k_hi of the s
// sampled distances) share every sweep over the sample: digit 1 has one
// histogram for both ranks (prefix 0), digits 2 and 3 two histograms under
// each select's own prefix, filled in the same pass; one single-block launch
// picks both digits.  The digit-1 pick also re-arms both selects (k, prefix),
// the digit-3 pick arms the bracketed select of D (bracket_init's work).
// Few workgroups per sweep (kSampleHistBlocks): every workgroup flushes its
// bins with global atomics, and the sampled distances fall into a handful of
// digit-1 bins, so thousands of workgroups would queue on the same addresses.
constexpr int kSampleHistBlocks = 256;

template <int PASS>
__global__ __launch_bounds__(256) void sample_hist_kernel(const float* __restrict__ sample,
                                                          int64_t s,
                                                          dsvgd_select_state* __restrict__ lo,
                                                          dsvgd_select_state* __restrict__ hi) {
  constexpr int kHists = PASS == 1 ? 1 : 2;
  __shared__ uint32_t shist[kHists][DSVGD_RADIX_BINS];
  for (int b = threadIdx.x; b < kHists * DSVGD_RADIX_BINS; b += 256) (&shist[0][0])[b] = 0u;
  uint32_t shift, mask, hishift;
  digit_of(PASS, shift, mask, hishift);
  const uint32_t want_lo = PASS == 1 ? 0u : lo->prefix >> hishift;
  const uint32_t want_hi = PASS == 1 ? 0u : hi->prefix >> hishift;
  __syncthreads();
  const f32x4* S4 = reinterpret_cast<const f32x4*>(sample);
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < s / 4;
       q += (int64_t)gridDim.x * 256) {
    const f32x4 v = S4[q];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      hist_key_agg(__float_as_uint(v[e]), want_lo, shift, mask, hishift, shist[0], 1u);
      if constexpr (PASS > 1)
        hist_key_agg(__float_as_uint(v[e]), want_hi, shift, mask, hishift, shist[1], 1u);
    }
  }
  __syncthreads();
  flush_block_hist(shist[0], lo);
  if constexpr (PASS > 1) flush_block_hist(shist[1], hi);
}

template <int PASS>
__global__ __launch_bounds__(256) void sample_pick_kernel(dsvgd_select_state* __restrict__ lo,
                                                          dsvgd_select_state* __restrict__ hi,
                                                          int64_t s, int64_t k_lo, int64_t k_hi,
                                                          dsvgd_select_state* __restrict__ st,
                                                          int64_t n_total, int64_t cand_cap) {
  __shared__ unsigned long long part[4];
  if constexpr (PASS == 1) {
    if (threadIdx.x == 0) {
      reset_state(lo, (unsigned long long)k_lo, (unsigned long long)s);
      reset_state(hi, (unsigned long long)k_hi, (unsigned long long)s);
    }
    __syncthreads();
  }
  // digit 1: both ranks pick from the one shared histogram (lo's bins)
  pick_digit<false>(lo->hist, lo, PASS, part);
  pick_digit<false>(PASS == 1 ? lo->hist : hi->hist, hi, PASS, part);
  clear_bins(lo->hist);
  clear_bins(hi->hist);
  if constexpr (PASS == 3) bracket_reset(st, n_total, lo->median, hi->median, cand_cap);
}

}  // namespace dsvgd

using namespace dsvgd;

extern "C" {

int dsvgd_select_init(dsvgd_select_state* st, int64_t n_total, int64_t k_rank, void* stream) {
  DSVGD_REQUIRE(st && n_total > 0, "args");
  hipLaunchKernelGGL(select_init_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, st, n_total,
                     k_rank);
  return check_launch("select_init");
}

int dsvgd_radix_hist(const float* D, int64_t count, const float* cand, int pass,
                     dsvgd_select_state* st, int64_t sym_npad, void* stream) {
  DSVGD_REQUIRE(D && st, "null pointer");
  DSVGD_REQUIRE(pass >= 1 && pass <= 3, "pass must be 1..3");
  DSVGD_REQUIRE(count >= 0 && ((uintptr_t)D & 15) == 0, "count / alignment");
  DSVGD_REQUIRE(sym_npad == 0 || (sym_npad % 128 == 0 && count == sym_npad * sym_npad),
                "sym_npad: count must be sym_npad^2 (a square panel-layout matrix)");
  int64_t blocks = (count / 4 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (cand && blocks < 1024) blocks = 1024;  // candidate slots: one wave each, grid-stride
  hipLaunchKernelGGL(radix_hist_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, D, count,
                     cand, pass, st, sym_npad);
  return check_launch("radix_hist");
}

int dsvgd_radix_hist_wmap(const float* D, int64_t m_pad, int64_t n_pad, const float* cand,
                          int pass, dsvgd_select_state* st, const uint8_t* wmap, void* stream) {
  DSVGD_REQUIRE(D && st && wmap, "null pointer");
  DSVGD_REQUIRE(pass >= 1 && pass <= 3, "pass must be 1, 2 or 3");
  DSVGD_REQUIRE(m_pad > 0 && n_pad > 0 && m_pad % 128 == 0 && n_pad % 128 == 0,
                "m_pad, n_pad must be positive multiples of 128");
  const int64_t count = m_pad * n_pad;
  int64_t blocks = min((int64_t)4096, max((int64_t)1, count / kPanelElems));
  if (cand && blocks < 1024) blocks = 1024;  // candidate slots: one wave each, grid-stride
  hipLaunchKernelGGL(radix_hist_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                     D, count, cand, pass, st, n_pad, wmap);
  return check_launch("radix_hist_wmap");
}

int dsvgd_radix_pick(dsvgd_select_state* st, int pass, void* stream) {
  DSVGD_REQUIRE(st, "null state");
  DSVGD_REQUIRE(pass >= 1 && pass <= 3, "pass must be 1..3");
  hipLaunchKernelGGL(radix_pick_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, st, pass);
  return check_launch("radix_pick");
}

int dsvgd_sample_sqdist(const float* Y, int64_t ldy, int64_t n, int64_t d, int64_t s,
                        uint64_t seed, float* out, void* stream) {
  DSVGD_REQUIRE(Y && out, "null pointer");
  DSVGD_REQUIRE(n > 0 && d > 0 && s > 0 && ldy >= d, "sizes");
  if (ldy % 4 == 0 && ((uintptr_t)Y & 15) == 0) {
    const int64_t blocks = std::min<int64_t>((s + 15) / 16, 8192);
    hipLaunchKernelGGL(sample_sqdist_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, Y,
                       ldy, n, (int)d, s, seed, out);
    return check_launch("sample_sqdist");
  }
  const int64_t blocks = std::min<int64_t>((s + 3) / 4, 8192);
  hipLaunchKernelGGL(sample_sqdist_any_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, Y,
                     ldy, n, (int)d, s, seed, out);
  return check_launch("sample_sqdist_any");
}

int dsvgd_sample_sqdist_range(const float* Y, int64_t ldy, int64_t n, int64_t d, int64_t s,
                              uint64_t seed, int64_t p0, int64_t p1, float* out, void* stream) {
  DSVGD_REQUIRE(Y && out, "null pointer");
  DSVGD_REQUIRE(n > 0 && d > 0 && s > 0 && ldy >= d && 0 <= p0 && p0 < p1 && p1 <= s, "sizes");
  const int64_t np = p1 - p0;
  if (ldy % 4 == 0 && ((uintptr_t)Y & 15) == 0) {
    const int64_t blocks = std::min<int64_t>((np + 15) / 16, 8192);
    hipLaunchKernelGGL(sample_sqdist_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, Y,
                       ldy, n, (int)d, p1, seed, out, p0);
    return check_launch("sample_sqdist");
  }
  const int64_t blocks = std::min<int64_t>((np + 3) / 4, 8192);
  hipLaunchKernelGGL(sample_sqdist_any_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, Y,
                     ldy, n, (int)d, p1, seed, out, p0);
  return check_launch("sample_sqdist_any");
}

int dsvgd_sample_bracket_select(const float* sample, int64_t s, int64_t k_lo, int64_t k_hi,
                                dsvgd_select_state* lo_st, dsvgd_select_state* hi_st,
                                dsvgd_select_state* st, int64_t n_total, int64_t cand_cap,
                                void* stream) {
  DSVGD_REQUIRE(sample && lo_st && hi_st && st, "null pointer");
  DSVGD_REQUIRE(n_total > 0 && cand_cap > 0, "sizes");
  DSVGD_REQUIRE(s > 0 && s % 4 == 0 && ((uintptr_t)sample & 15) == 0,
                "s must be a positive multiple of 4, sample 16-byte aligned");
  DSVGD_REQUIRE(0 <= k_lo && k_lo <= k_hi && k_hi < s, "ranks: 0 <= k_lo <= k_hi < s");
  hipStream_t strm = (hipStream_t)stream;
  const dim3 hb((unsigned)std::min<int64_t>((s / 4 + 255) / 256, kSampleHistBlocks));
#define DSVGD_SAMPLE_PASS(P)                                                                     \
  hipLaunchKernelGGL(sample_hist_kernel<P>, hb, dim3(256), 0, strm, sample, s, lo_st, hi_st);   \
  hipLaunchKernelGGL(sample_pick_kernel<P>, dim3(1), dim3(256), 0, strm, lo_st, hi_st, s, k_lo, \
                     k_hi, st, n_total, cand_cap)
  DSVGD_SAMPLE_PASS(1);
  DSVGD_SAMPLE_PASS(2);
  DSVGD_SAMPLE_PASS(3);
#undef DSVGD_SAMPLE_PASS
  return check_launch("sample_bracket_select");
}

int dsvgd_sample_bracket(const float* Y, int64_t ldy, int64_t n, int64_t d, int64_t s,
                         uint64_t seed, int64_t k_lo, int64_t k_hi, float* sample,
                         dsvgd_select_state* lo_st, dsvgd_select_state* hi_st,
                         dsvgd_select_state* st, int64_t n_total, int64_t cand_cap,
                         void* stream) {
  DSVGD_REQUIRE(Y && sample && lo_st && hi_st && st, "null pointer");
  DSVGD_REQUIRE(n > 0 && d > 0 && ldy >= d && n_total > 0 && cand_cap > 0, "sizes");
  DSVGD_REQUIRE(s > 0 && s % 4 == 0 && ((uintptr_t)sample & 15) == 0,
                "s must be a positive multiple of 4, sample 16-byte aligned");
  DSVGD_REQUIRE(0 <= k_lo && k_lo <= k_hi && k_hi < s, "ranks: 0 <= k_lo <= k_hi < s");
  int rc = dsvgd_sample_sqdist(Y, ldy, n, d, s, seed, sample, stream);
  if (rc) return rc;
  hipStream_t strm = (hipStream_t)stream;
  const dim3 hb((unsigned)std::min<int64_t>((s / 4 + 255) / 256, kSampleHistBlocks));
#define DSVGD_SAMPLE_PASS(P)                                                                     \
  hipLaunchKernelGGL(sample_hist_kernel<P>, hb, dim3(256), 0, strm, sample, s, lo_st, hi_st);   \
  hipLaunchKernelGGL(sample_pick_kernel<P>, dim3(1), dim3(256), 0, strm, lo_st, hi_st, s, k_lo, \
                     k_hi, st, n_total, cand_cap)
  DSVGD_SAMPLE_PASS(1);
  DSVGD_SAMPLE_PASS(2);
  DSVGD_SAMPLE_PASS(3);
#undef DSVGD_SAMPLE_PASS
  return check_launch("sample_bracket");
}

int dsvgd_bracket_init(dsvgd_select_state* st, int64_t n_total, const dsvgd_select_state* lo_st,
                       const dsvgd_select_state* hi_st, int64_t cand_cap, void* stream) {
  DSVGD_REQUIRE(st && lo_st && hi_st && n_total > 0, "args");
  DSVGD_REQUIRE(cand_cap > 0, "cand_cap must be positive");
  hipLaunchKernelGGL(bracket_init_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, st, n_total,
                     lo_st, hi_st, cand_cap);
  return check_launch("bracket_init");
}

int dsvgd_bracket_totals(dsvgd_select_state* st, const float* cand, void* stream) {
  DSVGD_REQUIRE(st && cand, "null pointer");
  hipLaunchKernelGGL(bracket_totals_kernel, dim3(256), dim3(256), 0, (hipStream_t)stream, st,
                     cand);
  return check_launch("bracket_totals");
}

int dsvgd_bracket_check(dsvgd_select_state* st, void* stream) {
  DSVGD_REQUIRE(st, "null state");
  hipLaunchKernelGGL(bracket_check_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, st);
  return check_launch("bracket_check");
}

}  // extern "C"
