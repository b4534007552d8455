// select.hpp -- device-side accounting the distance kernels do for the exact
// median select (lower median, k = (n^2-1)//2 over the full
// n x n matrix).  Two modes, chosen by the caller per step:
//
//  kSelHist     the epilogue accumulates radix digit 1 (key bits 31..21) of
//               every valid entry; passes 2 and 3 then stream D again.
//  kSelBracket  a 2^18-pair sample has fixed lo <= median <= hi (6 sigma of
//               the sample rank); the epilogue counts entries < lo and
//               compacts the entries in [lo, hi] (~1 %) into per-wave
//               candidate slots, so the three radix passes read the
//               candidates, not D.
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
// Every wave of a distance launch owns one fixed-capacity candidate slot
// (layout: include/dsvgd.h, DSVGD_SLOT_WEIGHT2).  Per value: the lane counts
// it if < lo; values in [lo, hi] (~1 %) are compacted into the slot with a
// wave ballot + mbcnt (no atomics, no block barrier, no re-reads).  finish()
// writes the slot's counts; a slot that fills up is detected by
// bracket_totals (count > slot_cap) and the select falls back to D.
struct SlotLayout {
  uint32_t* cnt;
  uint32_t* below;
  float* data;
  int64_t nslots, cap;
  __device__ __forceinline__ SlotLayout(float* cand, int64_t nslots_, uint64_t cand_cap)
      : nslots(nslots_) {
    cnt = reinterpret_cast<uint32_t*>(cand);
    below = cnt + nslots_;
    data = cand + 2 * nslots_;
    const int64_t c = ((int64_t)cand_cap - 2 * nslots_) / nslots_;
    cap = c > 0 ? c : 0;
  }
  // block 0 publishes the geometry for the select passes / totals
  __device__ __forceinline__ void publish(dsvgd_select_state* st, int64_t block) const {
    if (block == 0 && threadIdx.x == 0) {
      st->nslots = (uint64_t)nslots;
      st->slot_cap = (uint64_t)cap;
    }
  }
};

struct SlotWriter {
  float* dst = nullptr;
  uint32_t cnt = 0;    // wave-uniform: entries in [lo, hi] so far (may exceed cap)
  uint32_t below = 0;  // wave-uniform: entries < lo so far
  uint32_t cap = 0;
  // keys: fp32 bit patterns of values >= 0 (and +inf pads): monotone, all
  // < 2^31.  One subtraction d = key - klo (mod 2^32) serves both tests:
  // key < klo <=> d >= 2^31 (both < 2^31), in bracket <=> d <= khi - klo;
  // each is one compare whose lane mask is counted on the scalar unit.
  uint32_t klo = 1u, kspan = 0u;
  __device__ __forceinline__ void begin(const dsvgd_select_state* st, const SlotLayout& L,
                                        int64_t slot) {
    const float lo = st->lo, hi = st->hi;
    // an unordered bracket (NaN sample) counts everything below and nothing
    // in range, so bracket_check falls back to the exact passes over D
    // (klo = 2^31 - 1 exceeds every key; d = 0 never happens for it)
    const bool ok = hi >= lo && lo >= 0.f;
    klo = ok ? __float_as_uint(lo) : 0x7FFFFFFFu;
    kspan = ok ? __float_as_uint(hi) - klo : 0u;
    dst = L.data + slot * L.cap;
    cap = (uint32_t)L.cap;
  }
  // every lane of the wave must call add() for the same value index
  __device__ __forceinline__ void add(float v) {
    const uint32_t d = __float_as_uint(v) - klo;
    below += (uint32_t)__popcll(__ballot(d >= 0x80000000u));
    const bool in = d <= kspan;
    const uint64_t bal = __ballot(in);
    if (bal) {
      if (in) {
        const uint32_t pos = cnt + __builtin_amdgcn_mbcnt_hi(
                                       (uint32_t)(bal >> 32),
                                       __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
        if (pos < cap) dst[pos] = v;
      }
      cnt += (uint32_t)__popcll(bal);
    }
  }
  static constexpr int kDepth = 1 << 30;  // flush() is a no-op
  __device__ __forceinline__ void flush() {}
  __device__ __forceinline__ void finish(const SlotLayout& L, int64_t slot, bool weight2) {
    const uint32_t b = below;
    if ((threadIdx.x & 63) == 0) {
      const uint32_t flag = weight2 ? DSVGD_SLOT_WEIGHT2 : 0u;
      L.cnt[slot] = (cnt < DSVGD_SLOT_WEIGHT2 ? cnt : DSVGD_SLOT_WEIGHT2 - 1u) | flag;
      L.below[slot] = b;
    }
  }
};

// LDS-staged form of SlotWriter (the 256-tile Gram's epilogue): no branch
// and no wave-wide ballot per value.  add() writes every value to the lane's
// private list in LDS (entry k of lane l at stage[64 k + l]: distinct banks
// whatever the lanes' positions) and advances the lane's position only for
// values in [lo, hi]; an out-of-range value is overwritten by the next one.
// flush() -- after at most DEPTH add()s -- moves the lists to the slot in
// lane order (one wave prefix sum of the positions).  Below-counts are per
// lane, summed at finish().  Per value: a subtract, a shift-add, a compare,
// an LDS store and a conditional add (the ballot form compiled to ~25
// instructions with exec-mask branches per value).  DEPTH 8 on a list area
// of its own; 32 on the retired ring stage of the 256-tile Gram (a wave's own
// chunks, NTX3Tile WC): a quarter of the flushes.
constexpr int kStageDepth = 8;
template <int DEPTH = kStageDepth>
struct SlotWriterLdsT {
  static constexpr int kDepth = DEPTH;
  float* dst = nullptr;
  float* stage = nullptr;  // this wave's 64 x DEPTH floats
  uint32_t cnt = 0;        // wave-uniform: entries in [lo, hi] flushed so far
  uint32_t cap = 0;
  uint32_t below = 0;      // per lane
  uint32_t pos = 0;        // per lane: staged entries
  uint32_t klo = 1u, kspan = 0u;
  __device__ __forceinline__ void begin(const dsvgd_select_state* st, const SlotLayout& L,
                                        int64_t slot, float* wave_stage) {
    const float lo = st->lo, hi = st->hi;
    const bool ok = hi >= lo && lo >= 0.f;  // as SlotWriter::begin
    klo = ok ? __float_as_uint(lo) : 0x7FFFFFFFu;
    kspan = ok ? __float_as_uint(hi) - klo : 0u;
    dst = L.data + slot * L.cap;
    cap = (uint32_t)L.cap;
    stage = wave_stage + (threadIdx.x & 63);
  }
  __device__ __forceinline__ void add(float v) {
    const uint32_t d = __float_as_uint(v) - klo;
    below += d >> 31;
    stage[pos * 64] = v;
    pos += d <= kspan ? 1u : 0u;
  }
  __device__ __forceinline__ void flush() {
    if (__ballot(pos != 0u) == 0ull) return;
    uint32_t total;
    const uint32_t pre = wave_excl_scan(pos, total);
    for (uint32_t k = 0;; ++k) {
      const bool act = k < pos;
      if (__ballot(act) == 0ull) break;
      if (act) {
        const uint32_t p = cnt + pre + k;
        if (p < cap) dst[p] = stage[k * 64];
      }
    }
    cnt += total;
    pos = 0u;
  }
  __device__ __forceinline__ void finish(const SlotLayout& L, int64_t slot, bool weight2) {
    flush();
    uint32_t b = below;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) b += __shfl_xor(b, o, 64);
    if ((threadIdx.x & 63) == 0) {
      const uint32_t flag = weight2 ? DSVGD_SLOT_WEIGHT2 : 0u;
      L.cnt[slot] = (cnt < DSVGD_SLOT_WEIGHT2 ? cnt : DSVGD_SLOT_WEIGHT2 - 1u) | flag;
      L.below[slot] = b;
    }
  }
};

using SlotWriterLds = SlotWriterLdsT<>;

// slots of a wave that has no values (padding blocks): empty counts
__device__ __forceinline__ void slot_clear(const SlotLayout& L, int64_t slot) {
  if ((threadIdx.x & 63) == 0) {
    L.cnt[slot] = 0u;
    L.below[slot] = 0u;
  }
}

}  // namespace dsvgd
