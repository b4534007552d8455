// w2.hip -- the W2 / JKO term of DistSampler.make_step
// (reference dsvgd/distsampler.py:103-129, applied at :190-198).
//
// The reference solves  min <P, C>  s.t.  P >= 0, P 1 = 1/m, P^T 1 = 1/n  with
// C_ij = ||x_i - y_j||^2 (x: the m owned particles, y: the n previous ones)
// by scipy linprog and returns  sum_j P_ij (x_i - y_j).  In every DistSampler
// mode n = R m (R = 1 for partitions, R = num_shards when particles are
// exchanged), and after scaling by n the supplies are R and the demands 1, so
// the LP's vertices are integral: the optimum is an assignment of n "slots"
// (slot s belongs to row s / R) to the n columns, each carrying mass 1/n.
//
// Solver: forward auction (Bertsekas) with epsilon scaling, Jacobi bidding,
// rows bidding as classes of R identical "similar persons":
//   * one wave per row with u > 0 free slots scans its cost row for the
//     u + 1 best values v_k of -C_ij - p_j (prices in fp64) over the columns
//     the row does not already hold, and its free slots bid
//     p_jk + (v_k - v_{u+1} + eps) on the u best.  Excluding the row's own
//     columns is what stops sibling slots (identical cost rows) from
//     outbidding each other by eps -- the price war that makes slot-level
//     bidding take 5-50x more rounds when R > 1;
//   * bids are resolved with one 64-bit atomicMax per bid, key =
//     (fp32 increment rounded down) << 32 | slot, so a round's outcome does
//     not depend on scheduling (ties go to the higher slot id);
//   * the last resolve block (agent-scope release/acquire ticket) runs the
//     control step: it ends a phase when every slot is assigned, divides eps
//     by kTheta and starts the next phase by bumping an epoch counter
//     (assignments of older epochs read as unassigned -- no reset pass over
//     n); prices carry over between phases.  A round = 2 launches.
// With eps_final = cmax * 2^-24 / n the final assignment is within cmax *
// 2^-24 (one fp32 ulp of the largest cost) of the optimum.  The host wrapper
// enqueues rounds in batches and polls the control block (pinned, double
// buffered: batch k+1 is queued before batch k's state is waited for).
#include <float.h>

#include <algorithm>
#include <vector>

#include "common.hpp"

namespace dsvgd {

struct W2Ctl {
  double eps, eps_final;
  float cmax;
  int32_t epoch;
  int32_t done;  // 0 running, 1 converged, 2 degenerate (all costs 0), 3 bad input
  int32_t fresh;  // this round starts a phase with the last one's plan: keep-checks first
  unsigned long long unassigned;
  long long rounds, phases;
  unsigned int ticket;  // resolve-kernel arrival counter (last arriver resets it)
  unsigned long long viol;  // warm start: the previous plan's CS violation (fp64 bits, >= 0)
  int32_t tail;     // this round is the one-workgroup tail's (unassigned <= kTailMax)
  int32_t keep_on;  // phases keep the last plan's eps-CS slots (dsvgd_w2_set_keep)
  double theta;     // eps divisor between phases (dsvgd_w2_set_theta; kTheta)
  unsigned long long tail_bids, tail_scans;  // the tails' work (dsvgd_w2_tail_stats)
  unsigned long long tail_t[3];  // their time in the cached bids, the scans, the resolves (10 ns)
  // the tail's scan mailbox (w2_tail_kernel: workgroup 0 posts, the helper
  // workgroups scan a column share each and count themselves done)
  unsigned long long mb_seq;  // (round << 20) | k
  unsigned int mb_done;
  unsigned int tail_off;  // no phase tails this solve: its helpers could not be
                          // co-resident (occupancy) or one stalled (the bid rounds finish)
  unsigned int tail_stalls;  // tails that gave up on their helpers (dsvgd_w2_tail_stats)
  unsigned int debug_nohelp;  // tests: the helpers exit at once (dsvgd_w2_set_tail_debug)
  long long mb_row;
  double mb_floor;
};

constexpr size_t kW2CtlBytes = 256;
static_assert(sizeof(W2Ctl) <= kW2CtlBytes, "control block outgrew its slot");
constexpr double kTheta = 8.0;
constexpr int kRoundBatch = 16;
constexpr int kTailMax = 64;  // the phase tail's unassigned slots (w2_tail_kernel)
constexpr int kBidBlocks = 1024;  // grid-stride bid kernel: 4096 waves
// R = 2 .. kCacheMaxR bids go through the per-row price cache (measured
// against full scans: same plans, 3-20x fewer cost-row reads)
constexpr bool kW2Cache = true;

// holder[j] = epoch tag << 21 | row holding column j (tag = epoch & 0x7ff,
// never 0: stale entries of earlier phases and the zeroed workspace read as
// "not held"); owner[j] = the holding slot.
constexpr int kRowBits = 21;
constexpr int64_t kMaxRows = (int64_t)1 << kRowBits;
constexpr int kMaxR = 32;
__device__ __forceinline__ uint32_t w2_tag(int ep) { return (uint32_t)(ep & 0x7ff) << kRowBits; }

// Price cache (R in [2, kCacheMaxR]): a row's full scan keeps its kCache
// best columns over ALL columns (col, cost) and the (kCache+1)-th value
// -C - p as `bound`.  Prices only rise (within and across phases), so every
// uncached column's current value is <= bound; a later bid that finds its
// u + 1 best non-held values among the cached columns (current prices) with
// the (u+1)-th >= bound is exactly the full scan's bid.  The row holds at most
// R - u columns, so its u + 1 best non-held are among its R + 1 best overall
// (R + 1 <= kCache).  Otherwise it rescans and refills.  valid[i] = 0 after
// the workspace memset of every solve (costs change between solves).
// 16 columns (32 measured the same: the tail's cost is not its rescans,
// profiles/r11n)
constexpr int kCache = 16;
constexpr int kCacheMaxR = 8;

// the phase tail's scan helpers (w2_tail_kernel): workgroups, list length
constexpr int kTailHelpers = 32;
constexpr int kTailListMax = 33;

struct W2Ws {
  W2Ctl* ctl;
  double* price;
  unsigned long long* bid;
  int32_t *owner, *assigned, *assigned_ep;
  uint32_t* holder;
  int32_t *ccol, *cvalid;
  float* ccost;
  double* cbound;
  double* tv;   // the tail helpers' lists: kTailHelpers x kTailListMax
  int32_t* tj;
  int32_t* cbcol;  // the column of each row's bound (its scan's 17th best)
  W2Ws(void* ws, int64_t n, int64_t m) {
    char* p = (char*)ws;
    ctl = (W2Ctl*)p;
    price = (double*)(p + kW2CtlBytes);
    bid = (unsigned long long*)(price + n);
    owner = (int32_t*)(bid + n);
    holder = (uint32_t*)(owner + n);
    assigned = (int32_t*)(holder + n);
    assigned_ep = assigned + n;
    cbound = (double*)(((uintptr_t)(assigned_ep + n) + 7) & ~(uintptr_t)7);
    ccol = (int32_t*)(cbound + m);
    ccost = (float*)(ccol + m * kCache);
    cvalid = (int32_t*)(ccost + m * kCache);
    tv = (double*)(((uintptr_t)(cvalid + m) + 7) & ~(uintptr_t)7);
    tj = (int32_t*)(tv + kTailHelpers * kTailListMax);
    cbcol = tj + kTailHelpers * kTailListMax;
  }
};

// C[i][j] = ||x_i - y_j||^2 from explicit fp32 differences (the reference's
// diffs / norm, distsampler.py:107-114).  128 x 128 tile per block, each
// thread 8 x 8 (rows 4rq..+3 and 64+4rq..+3, columns likewise); 32-dim chunks
// of both operands transposed into LDS ([k][row]) so a thread's rows / columns
// are two ds_read_b128 each: 64 outputs per four LDS reads keeps the packed
// f32 VALU (v_pk_add / v_pk_fma) the bound -- the 64 x 64 / 4 x 4 tiling it
// replaces issued one LDS read per eight outputs and ran at half that rate.
// Every C_ij is the same k-ordered fma chain as before (bitwise).
constexpr int kCostTile = 128;
__global__ __launch_bounds__(256) void w2_cost_kernel(const float* __restrict__ X, int64_t ldx,
                                                      int64_t m, const float* __restrict__ Y,
                                                      int64_t ldy, int64_t n, int64_t d,
                                                      float* __restrict__ C, int64_t ldc) {
  __shared__ __attribute__((aligned(16))) float xs[32][kCostTile + 4];
  __shared__ __attribute__((aligned(16))) float ys[32][kCostTile + 4];
  const int t = threadIdx.x, rq = t >> 4, cq = t & 15;
  const int64_t i0 = (int64_t)blockIdx.y * kCostTile, j0 = (int64_t)blockIdx.x * kCostTile;
  float acc[8][8] = {};
  // the next 32-dim chunk is loaded into registers while this one computes:
  // every load is unconditional (clamped address, zeroed after), so all 32
  // are in flight together instead of one load-wait-store at a time
  constexpr int kQ = kCostTile * 32 / 256;
  float xr[kQ], yr[kQ];
  auto load = [&](int64_t k0) {
#pragma unroll
    for (int q = 0; q < kQ; ++q) {
      const int e = t + 256 * q, r = e >> 5, k = e & 31;
      const int64_t i = i0 + r, j = j0 + r, kk = k0 + k;
      const int64_t kc = kk < d ? kk : d - 1;
      xr[q] = X[(i < m ? i : m - 1) * ldx + kc];
      yr[q] = Y[(j < n ? j : n - 1) * ldy + kc];
      if (!(i < m && kk < d)) xr[q] = 0.f;
      if (!(j < n && kk < d)) yr[q] = 0.f;
    }
  };
  load(0);
  for (int64_t k0 = 0; k0 < d; k0 += 32) {
#pragma unroll
    for (int q = 0; q < kQ; ++q) {
      const int e = t + 256 * q, r = e >> 5, k = e & 31;
      xs[k][r] = xr[q];
      ys[k][r] = yr[q];
    }
    __syncthreads();
    if (k0 + 32 < d) load(k0 + 32);
#pragma unroll 4
    for (int k = 0; k < 32; ++k) {
      const f32x4 xa = *reinterpret_cast<const f32x4*>(&xs[k][4 * rq]);
      const f32x4 xb = *reinterpret_cast<const f32x4*>(&xs[k][64 + 4 * rq]);
      const f32x4 ya = *reinterpret_cast<const f32x4*>(&ys[k][4 * cq]);
      const f32x4 yb = *reinterpret_cast<const f32x4*>(&ys[k][64 + 4 * cq]);
#pragma unroll
      for (int a = 0; a < 8; ++a) {
        const float xv = a < 4 ? xa[a] : xb[a - 4];
#pragma unroll
        for (int b = 0; b < 8; ++b) {
          const float df = xv - (b < 4 ? ya[b] : yb[b - 4]);
          acc[a][b] = fmaf(df, df, acc[a][b]);
        }
      }
    }
    __syncthreads();
  }
  const bool vec = (ldc & 3) == 0 && ((uintptr_t)C & 15) == 0;
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    const int64_t i = i0 + (a < 4 ? 4 * rq + a : 64 + 4 * rq + a - 4);
    if (i >= m) continue;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int64_t j = j0 + 64 * h + 4 * cq;
      float* dst = C + i * ldc + j;
      if (vec && j + 3 < n) {
        *reinterpret_cast<f32x4*>(dst) = f32x4{acc[a][4 * h], acc[a][4 * h + 1],
                                               acc[a][4 * h + 2], acc[a][4 * h + 3]};
      } else {
#pragma unroll
        for (int b = 0; b < 4; ++b)
          if (j + b < n) dst[b] = acc[a][4 * h + b];
      }
    }
  }
}

// cmax = max C (C >= 0: the fp32 bit patterns order like the values); any
// non-finite cost marks the control block invalid.
__global__ __launch_bounds__(256) void w2_cmax_kernel(const float* __restrict__ C, int64_t ldc,
                                                      int64_t m, int64_t n, W2Ctl* ctl) {
  uint32_t mx = 0;
  bool bad = false;
  // row segments of 2048 columns: one 64-bit division per segment, not per
  // element; eight independent loads in flight per thread
  const int64_t nseg = (n + 2047) / 2048, total = m * nseg;
  for (int64_t sg = blockIdx.x; sg < total; sg += gridDim.x) {
    const int64_t i = sg / nseg, jb = (sg - i * nseg) * 2048;
    const float* row = C + i * ldc;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t j = jb + 256 * u + threadIdx.x;
      if (j < n) {
        const float v = row[j];
        bad |= !(v >= 0.f && v <= FLT_MAX);
        mx = max(mx, __float_as_uint(v));
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
  if ((threadIdx.x & 63) == 0) atomicMax((unsigned int*)&ctl->cmax, mx);
  if (bad) atomicExch(&ctl->done, 3);
}

// cmax and the bad-input flag from the cost kernel's own (dsvgd_w2_cost_h2 cstat)
__global__ void w2_cstat_kernel(const uint32_t* __restrict__ cstat, W2Ctl* ctl) {
  if (threadIdx.x == 0) {
    ctl->cmax = __uint_as_float(cstat[0]);
    if (cstat[1]) ctl->done = 3;
  }
}

// Warm start, adaptive: how far the previous plan `prev` is from
// complementary slackness under the new costs and the kept prices,
//   viol = max_i [ max_j (-C_ij - p_j) - min_{slots s of i} (-C_i,prev[s] - p_prev[s]) ],
// one wave per row (fp64 values; the max goes out as the bit pattern of a
// non-negative double, which orders like the value).
__global__ __launch_bounds__(256) void w2_violation_kernel(const float* __restrict__ C, int64_t ldc,
                                                           int64_t m, int64_t n, int64_t R,
                                                           const int32_t* __restrict__ prev,
                                                           W2Ws w) {
  const int lane = threadIdx.x & 63;
  double vmax = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < m;
       i += (int64_t)gridDim.x * 4) {
    const float* row = C + i * ldc;
    double best = -DBL_MAX;
    int64_t j = lane;
    for (; j + 192 < n; j += 256) {   // four independent loads in flight per lane
      const float c0 = row[j], c1 = row[j + 64], c2 = row[j + 128], c3 = row[j + 192];
      const double p0 = w.price[j], p1 = w.price[j + 64], p2 = w.price[j + 128],
                   p3 = w.price[j + 192];
      best = fmax(fmax(fmax(best, -(double)c0 - p0), fmax(-(double)c1 - p1, -(double)c2 - p2)),
                  -(double)c3 - p3);
    }
    for (; j < n; j += 64) best = fmax(best, -(double)row[j] - w.price[j]);
    double worst = DBL_MAX;
    if (lane < R) {
      const int64_t a = prev[i * R + lane];
      worst = (a >= 0 && a < n) ? -(double)row[a] - w.price[a] : -DBL_MAX;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      best = fmax(best, __shfl_xor(best, o, 64));
      worst = fmin(worst, __shfl_xor(worst, o, 64));
    }
    vmax = fmax(vmax, best - worst);
  }
  if (lane == 0 && vmax > 0.0)
    atomicMax(&w.ctl->viol, (unsigned long long)__double_as_longlong(vmax));
}

// The same violation, eight rows per 256-thread block: each thread walks
// 16-byte column chunks, loading a chunk's four prices once for the eight
// rows (the one-wave-per-row form re-read all n prices per row: 34 GB of
// L2 traffic at 65536^2 against C's 17 GB).  max / min are exact, so viol
// has the same bits.  Needs n % 4 == 0, ldc % 4 == 0, C 16-byte aligned.
constexpr int kViolRows = 8;
__global__ __launch_bounds__(256) void w2_violation_rows_kernel(const float* __restrict__ C,
                                                                int64_t ldc, int64_t m, int64_t n,
                                                                int64_t R,
                                                                const int32_t* __restrict__ prev,
                                                                W2Ws w) {
  __shared__ double red[4][kViolRows];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t i0 = (int64_t)blockIdx.x * kViolRows;
  const int nr = (int)min<int64_t>(kViolRows, m - i0);
  double best[kViolRows];
#pragma unroll
  for (int r = 0; r < kViolRows; ++r) best[r] = -DBL_MAX;
  for (int64_t j = 4 * (int64_t)t; j < n; j += 1024) {
    const double2 pa = *reinterpret_cast<const double2*>(w.price + j);
    const double2 pb = *reinterpret_cast<const double2*>(w.price + j + 2);
#pragma unroll
    for (int r = 0; r < kViolRows; ++r) {
      if (r < nr) {
        const float4 c = *reinterpret_cast<const float4*>(C + (i0 + r) * ldc + j);
        best[r] = fmax(best[r], fmax(fmax(-(double)c.x - pa.x, -(double)c.y - pa.y),
                                     fmax(-(double)c.z - pb.x, -(double)c.w - pb.y)));
      }
    }
  }
#pragma unroll
  for (int r = 0; r < kViolRows; ++r) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) best[r] = fmax(best[r], __shfl_xor(best[r], o, 64));
    if (lane == 0) red[wv][r] = best[r];
  }
  __syncthreads();
  if (wv == 0) {
    double vmax = 0.0;
    for (int r = 0; r < nr; ++r) {
      const double b = fmax(fmax(red[0][r], red[1][r]), fmax(red[2][r], red[3][r]));
      const int64_t i = i0 + r;
      double worst = DBL_MAX;
      if (lane < R) {
        const int64_t a = prev[i * R + lane];
        worst = (a >= 0 && a < n) ? -(double)C[i * ldc + a] - w.price[a] : -DBL_MAX;
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) worst = fmin(worst, __shfl_xor(worst, o, 64));
      vmax = fmax(vmax, b - worst);
    }
    if (lane == 0 && vmax > 0.0)
      atomicMax(&w.ctl->viol, (unsigned long long)__double_as_longlong(vmax));
  }
}

// Warm start at R = 1 (no price cache, keep off): the first round's bids and
// the violation above from ONE pass over C.  Every slot is free in that round
// and nothing is held, so w2_bid_kernel<2> would scan each whole row for its
// best value, that value's column (the lowest on a tie) and the second best
// value (a tie counts twice) -- exactly what the violation pass reads too,
// minus the column and the second value.  This pass keeps all three per row
// (w2_bid_first_kernel bids from them once w2_start_kernel has set eps from
// the violation) and the violation, eight rows per block as in
// w2_violation_rows_kernel.  Same values, same tie rule, so the same bids and
// the same viol bits; the unfused order (violation pass, full-scan bid round)
// stays behind dsvgd_w2_set_fuse_first(0).  Needs n % 4 == 0, ldc % 4 == 0,
// C 16-byte aligned.  The row results go to the price cache's arrays, unused
// at R = 1: best -> cbound, second -> ccost (as doubles), column -> ccol.
__device__ __forceinline__ void top2_push(double x, int c, double& b1, int& j1, double& b2) {
  const bool gt = x > b1;  // columns arrive in increasing order: a tie keeps the lower
  b2 = fmax(b2, gt ? b1 : x);
  j1 = gt ? c : j1;
  b1 = gt ? x : b1;
}
__device__ __forceinline__ void top2_merge(double p1, int q1, double p2, double& b1, int& j1,
                                           double& b2) {
  const bool first = b1 > p1 || (b1 == p1 && j1 < q1);
  b2 = fmax(first ? p1 : b1, fmax(b2, p2));
  if (!first) {
    b1 = p1;
    j1 = q1;
  }
}
__global__ __launch_bounds__(256) void w2_scan_first_kernel(const float* __restrict__ C,
                                                            int64_t ldc, int64_t m, int64_t n,
                                                            const int32_t* __restrict__ prev,
                                                            W2Ws w) {
  __shared__ double r1[4][kViolRows], r2[4][kViolRows];
  __shared__ int rj[4][kViolRows];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t i0 = (int64_t)blockIdx.x * kViolRows;
  const int nr = (int)min<int64_t>(kViolRows, m - i0);
  double b1[kViolRows], b2[kViolRows];
  int j1[kViolRows];
#pragma unroll
  for (int r = 0; r < kViolRows; ++r) {
    b1[r] = b2[r] = -DBL_MAX;
    j1[r] = INT32_MAX;
  }
  for (int64_t j = 4 * (int64_t)t; j < n; j += 1024) {
    const double2 pa = *reinterpret_cast<const double2*>(w.price + j);
    const double2 pb = *reinterpret_cast<const double2*>(w.price + j + 2);
#pragma unroll
    for (int r = 0; r < kViolRows; ++r) {
      if (r < nr) {
        const float4 c = *reinterpret_cast<const float4*>(C + (i0 + r) * ldc + j);
        top2_push(-(double)c.x - pa.x, (int)j, b1[r], j1[r], b2[r]);
        top2_push(-(double)c.y - pa.y, (int)j + 1, b1[r], j1[r], b2[r]);
        top2_push(-(double)c.z - pb.x, (int)j + 2, b1[r], j1[r], b2[r]);
        top2_push(-(double)c.w - pb.y, (int)j + 3, b1[r], j1[r], b2[r]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < kViolRows; ++r) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double p1 = __shfl_xor(b1[r], o, 64), p2 = __shfl_xor(b2[r], o, 64);
      const int q1 = __shfl_xor(j1[r], o, 64);
      top2_merge(p1, q1, p2, b1[r], j1[r], b2[r]);
    }
    if (lane == 0) {
      r1[wv][r] = b1[r];
      r2[wv][r] = b2[r];
      rj[wv][r] = j1[r];
    }
  }
  __syncthreads();
  if (wv == 0) {
    double vmax = 0.0;
    if (lane < nr) {
      double a1 = r1[0][lane], a2 = r2[0][lane];
      int aj = rj[0][lane];
#pragma unroll
      for (int q = 1; q < 4; ++q) top2_merge(r1[q][lane], rj[q][lane], r2[q][lane], a1, aj, a2);
      const int64_t i = i0 + lane;
      w.cbound[i] = a1;
      reinterpret_cast<double*>(w.ccost)[i] = a2;
      w.ccol[i] = aj;
      const int64_t a = prev[i];
      const double worst = (a >= 0 && a < n) ? -(double)C[i * ldc + a] - w.price[a] : -DBL_MAX;
      vmax = fmax(vmax, a1 - worst);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) vmax = fmax(vmax, __shfl_xor(vmax, o, 64));
    if (lane == 0 && vmax > 0.0)
      atomicMax(&w.ctl->viol, (unsigned long long)__double_as_longlong(vmax));
  }
}

// warm_phases > 0: the prices are the previous solve's (a nearby problem:
// SVGD moves rows and columns by one step), so the auction starts only
// warm_phases epsilon-scaling phases above eps_final instead of at cmax/theta;
// warm_phases < 0: it starts at viol / kWarmDiv (the violation kernel's
// measure of how far the previous plan is off, so the first phase neither
// wastes rounds at a coarse epsilon nor fights a price war at a fine one:
// VERDICT r2 item 9).  Any initial prices give the same eps_final-optimality
// guarantee.
constexpr double kWarmDiv = 64.0;
__global__ void w2_start_kernel(W2Ctl* ctl, int64_t n, int warm_phases, int keep, double theta,
                                int tail_off, int debug_nohelp) {
  ctl->theta = theta;
  ctl->tail_off = tail_off ? 1u : 0u;
  ctl->tail_stalls = 0;
  ctl->debug_nohelp = debug_nohelp ? 1u : 0u;
  const double cmax = (double)ctl->cmax;
  ctl->eps_final = fmax(cmax * 0x1p-24 / (double)n, cmax * 1e-13);
  double e0 = cmax / theta;
  if (warm_phases > 0) {
    double ew = ctl->eps_final;
    for (int k = 0; k < warm_phases; ++k) ew *= theta;
    e0 = fmin(e0, ew);
  } else if (warm_phases < 0) {
    e0 = fmin(e0, __longlong_as_double((long long)ctl->viol) / kWarmDiv);
  }
  ctl->eps = fmax(e0, ctl->eps_final);
  ctl->epoch = 1;
  ctl->unassigned = (unsigned long long)n;
  ctl->rounds = 0;
  ctl->phases = 1;
  ctl->keep_on = keep & 1;
  ctl->fresh = keep >> 1;
  ctl->tail = !tail_off && n <= kTailMax;
  if (ctl->done == 0 && !(cmax > 0.0)) ctl->done = 2;
}

// Warm start: the previous plan as epoch 0's assignment, so that the first
// phase keeps every slot whose column still meets eps-CS (w2_keep).
__global__ __launch_bounds__(256) void w2_load_prev_kernel(int64_t n, const int32_t* __restrict__ prev,
                                                           W2Ws w) {
  const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (s >= n) return;
  const int32_t j = prev[s];
  w.assigned[s] = (j >= 0 && j < n) ? j : -1;
  w.assigned_ep[s] = 0;
}

// A lane's K best (value, column) pairs, sorted descending; ties keep the
// lower column (a lane sees its columns in increasing order).
template <int K>
struct TopK {
  double v[K];
  int j[K];
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      v[k] = -DBL_MAX;
      j[k] = INT32_MAX;
    }
  }
  __device__ __forceinline__ void push(double x, int c) {
    if (!(x > v[K - 1])) return;
#pragma unroll
    for (int k = K - 1; k > 0; --k) {
      const bool up = x > v[k - 1];
      const bool here = x > v[k];
      j[k] = up ? j[k - 1] : (here ? c : j[k]);
      v[k] = up ? v[k - 1] : (here ? x : v[k]);
    }
    if (x > v[0]) {
      v[0] = x;
      j[0] = c;
    }
  }
  __device__ __forceinline__ void pop() {
#pragma unroll
    for (int k = 0; k < K - 1; ++k) {
      v[k] = v[k + 1];
      j[k] = j[k + 1];
    }
    v[K - 1] = -DBL_MAX;
    j[K - 1] = INT32_MAX;
  }
};

// ---- block-cooperative scans (one workgroup per bidding row) -------------
// A full scan of a cost row reads n costs, n fp64 prices (and n holders):
// ~1 MB at n = 65536.  One wave walking it with a load -> top-K dependency per
// column was latency-bound (~150 us: the ~180 us rounds of the cold solve,
// profiles/r8j); here the workgroup's 256 threads take columns t, t + 256,
// ... with four columns' loads in flight each, then the four waves' top-K
// lists are merged.  Same values and the same tie rule (lower column first).
constexpr int kScanUnroll = 8;

// Wave w's K best of its lanes' lists (lane k < K: the k-th) into sv / sj
// [w K + k]; every lane's list is sorted descending, columns unique.
template <int K>
__device__ __forceinline__ void wave_topk_to_lds(TopK<K>& t, int lane, int wv, double* sv,
                                                 int* sj) {
  for (int k = 0; k < K; ++k) {
    double bv = t.v[0];
    int bj = t.j[0];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double ov = __shfl_xor(bv, o, 64);
      const int oj = __shfl_xor(bj, o, 64);
      if (ov > bv || (ov == bv && oj < bj)) {
        bv = ov;
        bj = oj;
      }
    }
    if (bj == INT32_MAX) {  // (uniform) the wave's lists are spent: pad, stop
      for (int r = k + lane; r < K; r += 64) {
        sv[wv * K + r] = -DBL_MAX;
        sj[wv * K + r] = INT32_MAX;
      }
      break;
    }
    if (lane == 0) {
      sv[wv * K + k] = bv;
      sj[wv * K + k] = bj;
    }
    if (t.j[0] == bj) t.pop();
  }
}

// The workgroup's K best (value, column) of -C_ij - p_j over the columns j
// the row does not hold (skip_held) or over all columns, sorted descending,
// into out_v / out_j [K] (LDS, visible to the whole block on return).
template <int K, int NW = 4, int U = kScanUnroll>
__device__ __forceinline__ void block_topk(const float* __restrict__ row, int64_t n, const W2Ws& w,
                           uint32_t mine, bool skip_held, double* sv, int* sj, double* out_v,
                           int* out_j, double floor = -DBL_MAX, int64_t col0 = 0) {
  constexpr int NT = NW * 64;   // the workgroup's threads
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  TopK<K> tk;
  tk.init();
  // batches of U columns per thread, double-buffered: the next batch's loads
  // are in flight while this one is pushed (2 U loads of each array per
  // thread outstanding; a lone workgroup -- the phase tail -- reading other
  // XCDs' writes was latency-bound at 4: ~130 us per scan, profiles/r11p)
  const int64_t step = (int64_t)U * NT;
  int64_t j = t;
  if (j + (U - 1) * NT < n) {
    float c0[U], c1[U];
    double p0[U], p1[U];
    uint32_t h0[U], h1[U];
    auto load = [&](float (&c)[U], double (&p)[U], uint32_t (&h)[U], int64_t jj) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        c[u] = row[jj + u * NT];
        p[u] = w.price[col0 + jj + u * NT];
        h[u] = skip_held ? w.holder[col0 + jj + u * NT] : 0u;
      }
    };
    auto push = [&](const float (&c)[U], const double (&p)[U], const uint32_t (&h)[U],
                    int64_t jj) {
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (!skip_held || h[u] != mine) {
          // floor: a value at or below the K-th best overall (the caller
          // knows K such values); below it nothing can enter the list, so
          // most lanes skip the insertion (a wave pays for one whenever any
          // of its lanes inserts)
          const double x = -(double)c[u] - p[u];
          if (x >= floor) tk.push(x, (int)(col0 + jj + u * NT));
        }
    };
    load(c0, p0, h0, j);
    for (;;) {
      const int64_t j1 = j + step;
      const bool more1 = j1 + (U - 1) * NT < n;
      if (more1) load(c1, p1, h1, j1);
      push(c0, p0, h0, j);
      j = j1;
      if (!more1) break;
      const int64_t j2 = j + step;
      const bool more2 = j2 + (U - 1) * NT < n;
      if (more2) load(c0, p0, h0, j2);
      push(c1, p1, h1, j);
      j = j2;
      if (!more2) break;
    }
  }
  for (; j < n; j += NT)
    if (!skip_held || w.holder[col0 + j] != mine) {
      const double x = -(double)row[j] - w.price[col0 + j];
      if (x >= floor) tk.push(x, (int)(col0 + j));
    }
  wave_topk_to_lds<K>(tk, lane, wv, sv, sj);
  __syncthreads();
  if (t == 0) {  // merge the NW sorted lists
    int pos[NW];
#pragma unroll
    for (int q = 0; q < NW; ++q) pos[q] = 0;
    for (int k = 0; k < K; ++k) {
      int bq = -1;
      double bv = -DBL_MAX;
      int bj = INT32_MAX;
#pragma unroll
      for (int q = 0; q < NW; ++q) {
        if (pos[q] >= K) continue;
        const double v = sv[q * K + pos[q]];
        const int jj = sj[q * K + pos[q]];
        if (bq < 0 || v > bv || (v == bv && jj < bj)) {
          bq = q;
          bv = v;
          bj = jj;
        }
      }
      out_v[k] = bv;
      out_j[k] = bj;
#pragma unroll
      for (int q = 0; q < NW; ++q) pos[q] += q == bq;   // (registers: no dynamic index)
    }
  }
  __syncthreads();
}

// The bid of row i's u free slots from the u + 1 best non-held columns
// (kv, kj in lane k < u + 1; lanes >= u + 1 hold -DBL_MAX / INT32_MAX) --
// the tail of a row's bid
__device__ __forceinline__ void bid_from_best(double kv, int kj, int u, int64_t i, int64_t R,
                                              unsigned long long free, int lane, double eps,
                                              const W2Ws& w) {
  const double vu1 = __shfl(kv, u, 64), vu = __shfl(kv, u - 1, 64);
  const double vref = (vu1 > -DBL_MAX) ? vu1 : vu;
  if (lane >= u || kj == INT32_MAX) return;
  unsigned long long rest = free;
  for (int k = 0; k < lane; ++k) rest &= rest - 1;
  const int64_t s = i * R + (__ffsll((long long)rest) - 1);
  const double inc = kv - vref + eps;
  float f = (float)inc;
  if ((double)f > inc) f = nextafterf(f, 0.f);  // round down: keeps eps-CS
  if (!(f > 0.f)) f = FLT_MIN;
  const unsigned long long key =
      ((unsigned long long)__float_as_uint(f) << 32) | (unsigned long long)(uint32_t)s;
  atomicMax(&w.bid[kj], key);
}

// The u + 1 best (value, column) of the wave's lane candidates (cv, cj),
// in order, into lane k's (kv, kj) (ties -> lower column)
__device__ __forceinline__ void wave_best(double cv, int cj, int u, int lane, double& kv, int& kj) {
  kv = -DBL_MAX;
  kj = INT32_MAX;
  for (int k = 0; k <= u; ++k) {
    double bv = cv;
    int bj = cj;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double ov = __shfl_xor(bv, o, 64);
      const int oj = __shfl_xor(bj, o, 64);
      if (ov > bv || (ov == bv && oj < bj)) {
        bv = ov;
        bj = oj;
      }
    }
    if (lane == k) {
      kv = bv;
      kj = bj;
    }
    if (cj == bj) cv = -DBL_MAX;  // taken (columns are unique across lanes)
  }
}

// wave_best with u = 1 over the price cache's lanes 0 .. kCache-1 (16):
// one four-step butterfly carrying (best, its column, second best) instead
// of two six-step passes -- the tail's bids are a dependent chain, and the
// shuffles were most of a cached bid.  Ties: the lower column first.
__device__ __forceinline__ void top2_16(double cv, int cj, double& b1, int& j1, double& b2) {
  static_assert(kCache == 16, "top2_16 reduces over 16 lanes");
  double a1 = cv, a2 = -DBL_MAX;
  int i1 = cj;
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) {
    const double p1 = __shfl_xor(a1, o, 64), p2 = __shfl_xor(a2, o, 64);
    const int q1 = __shfl_xor(i1, o, 64);
    const bool first = a1 > p1 || (a1 == p1 && i1 < q1);
    a2 = fmax(first ? p1 : a1, fmax(a2, p2));
    if (!first) {
      a1 = p1;
      i1 = q1;
    }
  }
  b1 = __shfl(a1, 0, 64);
  b2 = __shfl(a2, 0, 64);
  j1 = __shfl(i1, 0, 64);
}

// ---- keeping the last phase's plan -----------------------------------------
// A new eps phase (and a warm start, whose "last phase" is the previous
// solve's plan) starts with every slot unassigned in the new epoch.  The
// slots whose column still meets eps-complementary slackness for the new eps
//   -C_ij - p_j >= max_k (-C_ik - p_k) - eps       (max over ALL columns)
// keep it instead (Bertsekas' auction keeps such pairs across phases): the
// invariant the auction maintains holds for them, so the phase still ends
// eps-optimal, and only the slots that violate it bid again.  Called by the
// wave that owns row i in the first round of a phase (ctl->fresh), with the
// row's best value over all columns; returns the kept slots' mask.
__device__ __forceinline__ unsigned long long w2_keep(const float* __restrict__ row, int64_t i,
                                                      int64_t R, int lane, int ep, uint32_t mine,
                                                      double best, double eps, const W2Ws& w) {
  bool k = false;
  if (lane < R) {
    const int64_t s = i * R + lane;
    const int j = w.assigned[s];
    if (w.assigned_ep[s] == ep - 1 && j >= 0) {
      const double v = -(double)row[j] - w.price[j];
      if (v >= best - eps) {
        k = true;
        w.assigned_ep[s] = ep;
        w.holder[j] = mine;
        w.owner[j] = (int)s;
      }
    }
  }
  const unsigned long long km = __ballot(k);
  if (lane == 0 && km)
    atomicAdd(&w.ctl->unassigned, (unsigned long long)(-(long long)__popcll(km)));
  __threadfence_block();  // the new holders before this wave's held-column tests
  return km;
}

// Whether lane's slot of row i holds a column of the previous epoch (wave-uniform result)
__device__ __forceinline__ bool w2_has_prev(int64_t i, int64_t R, int lane, int ep, const W2Ws& w) {
  bool hp = false;
  if (lane < R) {
    const int64_t s = i * R + lane;
    hp = w.assigned_ep[s] == ep - 1 && w.assigned[s] >= 0;
  }
  return __ballot(hp) != 0ull;
}

// ---- the phase tail, Gauss-Seidel (one workgroup) -----------------------
// A phase ends with long runs of rounds in which a handful of slots bid
// (profiles/r8j: 17k of the 19k rounds of a warm m = 8192, n = 65536 solve
// had <= 16 unassigned slots), each round two launches.  Once the unassigned
// count is <= kTailMax, the one-workgroup tail launch (queued every round,
// a no-op otherwise; the bid launch is then the no-op) runs the rest of the
// phase itself: the unassigned slots (found by a scan, sorted: deterministic)
// bid one at a time -- the u = 1 bid of the parallel rounds, from the row's
// price cache or a workgroup scan -- and each bid is resolved on the spot (a
// displaced slot goes back on the stack).  The same eps-complementary-
// slackness invariant as the Jacobi rounds, so the phase ends eps-optimal;
// the resolve launch behind it then runs the control step.  At most
// kTailBids bids per launch (the next round's launch continues).
//
// A tail bid is a chain of dependent reads (the row's cache, its columns'
// prices and holders, the won column's holder and owner): ~5 L2 round trips
// when they go to global memory.  The tail is the only writer while it runs,
// so it keeps direct-mapped LDS tables of the columns and rows it touches,
// written through to global memory on every update (the scans and the next
// launch read global memory, which is therefore always current): a price war
// over a few columns then runs out of LDS.
constexpr int kTailBids = 16384;
// eight waves: the scans are one workgroup's reads of other XCDs' writes,
// latency-bound -- twice the waves, twice the loads in flight
constexpr int kTailWaves = 8;
constexpr int kTailThreads = kTailWaves * 64;
// the cached tail's scans' batch (x2 in flight, double-buffered; 16
// measured the same, r11s)
constexpr int kTailUnroll = 8;
constexpr int kTabCols = 4096;  // column entries: price, holder, owner, tag
constexpr int kTabRows = 512;   // row entries: the price cache of a row
constexpr size_t kTailLds =
    (size_t)kTabCols * (8 + 4 + 4 + 4) + (size_t)kTabRows * (8 + 4 + 4 + kCache * 8);

struct TailTab {
  double* cp;
  int32_t *ct, *co;
  uint32_t* ch;
  double* rb;
  int32_t *rt, *rv, *rc;
  float* rx;
  __device__ explicit TailTab(char* base) {
    cp = (double*)base;
    rb = cp + kTabCols;
    ct = (int32_t*)(rb + kTabRows);
    co = ct + kTabCols;
    ch = (uint32_t*)(co + kTabCols);
    rt = (int32_t*)(ch + kTabCols);
    rv = rt + kTabRows;
    rc = rv + kTabRows;
    rx = (float*)(rc + kTabRows * kCache);
  }
};

// Workgroup 0's wave 0 runs the bids: a bid answered by the row's price
// cache (most of them in a price war) touches no barrier at all -- it pops
// the slot, bids, resolves and pushes the displaced slot.  A rescan goes to
// the kTailHelpers other workgroups of the launch: wave 0 posts the row and
// its floor in the control block's mailbox (sequence number tagged with the
// round, agent-scope release), each helper scans its column share with
// block_topk and publishes its sorted list, wave 0 merges the lists.  Every
// poll is bounded (kSpinMax): the helpers share the CUs with whatever else
// runs on the device (another stream's kernels, RCCL's), so one that is not
// dispatched in time ends the launch instead of hanging it -- the tail then
// turns itself off for the rest of the solve (tail_off) and the ordinary bid
// rounds finish the phase: a slower solve, never a failed one.
template <int K, bool CACHED>
__global__ __launch_bounds__(kTailThreads) void w2_tail_kernel(const float* __restrict__ C, int64_t ldc,
                                                      int64_t n, int64_t R, W2Ws w) {
  extern __shared__ __attribute__((aligned(16))) char w2_tail_lds[];
  constexpr int KS = CACHED ? kCache + 1 : K;  // the scans' list length
  __shared__ double sv[kTailWaves * KS], outv[KS];
  __shared__ int sj[kTailWaves * KS], outj[KS];
  __shared__ int stack[kTailMax], sorted[kTailMax];
  __shared__ int cnt;
  __shared__ long long req;     // helper workgroups: the row to scan, or -1: the tail is over
  __shared__ double req_floor;  // its scan's floor (block_topk)
  const W2Ctl* ctl = w.ctl;
  if (ctl->done || !ctl->tail) return;  // uniform over the grid
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int ep = ctl->epoch;
  const double eps = ctl->eps;
  const uint32_t tag = w2_tag(ep);
  // mailbox sequence numbers carry this round (stale posts of earlier tail
  // launches never match): (round << 20) | k, k = 1, 2, ... ; kQuit ends it
  constexpr unsigned long long kQuit = 0xFFFFFull;
  const unsigned long long rtag = (unsigned long long)ctl->rounds << 20;
  W2Ctl* mb = w.ctl;
  // every spin is bounded: a helper that never sees a post (or workgroup 0
  // that never sees its helpers) gives up; workgroup 0 then sets tail_off
  constexpr long long kSpinMax = 1ll << 20;   // ~1-2 s of polls
  if (blockIdx.x > 0) {  // a scan helper: columns [c0, c1)
    if (ctl->debug_nohelp) return;  // (tests: a helper that never answers)
    const int64_t share = ((n + kTailHelpers - 1) / kTailHelpers + 63) & ~(int64_t)63;
    const int64_t hc0 = min(n, (int64_t)(blockIdx.x - 1) * share), hc1 = min(n, hc0 + share);
    unsigned long long expect = 1;
    for (;;) {
      if (t == 0) {
        long long spins = 0;
        unsigned long long sq;
        for (;;) {
          sq = __hip_atomic_load(&mb->mb_seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
          if ((sq & ~kQuit) == rtag && ((sq & kQuit) == expect || (sq & kQuit) == kQuit)) break;
          if (++spins > kSpinMax) {
            sq = rtag | kQuit;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        req = ((sq & kQuit) == kQuit) ? -1 : mb->mb_row;
        req_floor = mb->mb_floor;
      }
      __syncthreads();
      const long long rq = req;
      if (rq < 0) return;
      if (hc1 > hc0)
        block_topk<KS, kTailWaves, CACHED ? kTailUnroll : kScanUnroll>(
            C + rq * ldc + hc0, hc1 - hc0, w, tag | (uint32_t)rq, !CACHED, sv, sj, outv, outj,
            req_floor, hc0);
      const int h = blockIdx.x - 1;
      if (t < KS) {
        w.tv[h * kTailListMax + t] = hc1 > hc0 ? outv[t] : -DBL_MAX;
        w.tj[h * kTailListMax + t] = hc1 > hc0 ? outj[t] : INT32_MAX;
      }
      __syncthreads();
      if (t == 0) {
        __threadfence();  // the list before the count (agent scope)
        __hip_atomic_fetch_add(&mb->mb_done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      }
      ++expect;
    }
  }
  TailTab T(w2_tail_lds);
  for (int e = t; e < kTabCols; e += kTailThreads) T.ct[e] = -1;
  for (int e = t; e < kTabRows; e += kTailThreads) T.rt[e] = -1;
  if (t == 0) {
    cnt = 0;
    __hip_atomic_store(&mb->mb_done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  for (int64_t s0 = t; s0 < n; s0 += kTailThreads)
    if (!(w.assigned_ep[s0] == ep && w.assigned[s0] >= 0)) {
      const int pos = atomicAdd(&cnt, 1);
      if (pos < kTailMax) stack[pos] = (int)s0;
    }
  __syncthreads();
  const int c0 = min(cnt, kTailMax);
  if (t < c0) {  // sort (descending: the lowest slot bids first, from the top)
    const int v = stack[t];
    int r = 0;
    for (int q = 0; q < c0; ++q) r += stack[q] > v;
    sorted[r] = v;
  }
  __syncthreads();
  if (t < c0) stack[t] = sorted[t];
  __syncthreads();
  if (wv != 0) return;  // wave 0 bids; the scans are the helper workgroups'
  // wave 0: the bids
  unsigned nseq = 0;
  bool stalled = false;
  auto scan = [&](int64_t i, uint32_t mine, double floor) {  // post row i, merge the helpers' lists
    __threadfence();  // this wave's price / holder writes before the helpers read (agent)
    ++nseq;
    if (lane == 0) {
      mb->mb_row = i;
      mb->mb_floor = floor;
      __hip_atomic_store(&mb->mb_seq, rtag | (unsigned long long)nseq, __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_AGENT);
      long long spins = 0;
      while (__hip_atomic_load(&mb->mb_done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) <
             nseq * (unsigned)kTailHelpers) {
        if (++spins > kSpinMax) {   // (a tight poll: the helpers answer in microseconds)
          stalled = true;
          break;
        }
      }
    }
    stalled = __shfl(stalled, 0, 64);
    __threadfence();
    // the helpers' sorted lists, one per lane, merged by the wave
    TopK<KS> tk;
    tk.init();
    if (lane < kTailHelpers && !stalled)
      for (int k = KS - 1; k >= 0; --k)
        tk.push(w.tv[lane * kTailListMax + k], w.tj[lane * kTailListMax + k]);
    wave_topk_to_lds<KS>(tk, lane, 0, sv, sj);
    if (lane < KS) {
      outv[lane] = sv[lane];
      outj[lane] = sj[lane];
    }
  };
  int sp = c0;
  int nbids = 0;
  unsigned long long tl = 0, tsc = 0, trs = 0;   // wall clock (100 MHz): lookups, scans, resolves
  for (int b = 0; b < kTailBids && sp > 0 && !stalled; ++b) {
    ++nbids;
    const unsigned long long t0 = wall_clock64();
    unsigned long long tsc0 = 0;
    const int s = stack[sp - 1];
    const int64_t i = s / R;
    const uint32_t mine = tag | (uint32_t)i;
    const float* row = C + i * ldc;
    double b1 = -DBL_MAX, b2 = -DBL_MAX;
    int bj = INT32_MAX;
    bool hit = false;
    double pj = 0.0;   // the bid column's price / holder / owner, when read already
    uint32_t hj = 0;
    int oj = -1;
    bool have_j = false;
    double floor = -DBL_MAX;   // the rescan's (block_topk)
    if (CACHED) {  // the row's cache (table, else global + install), its bid
      const int re = (int)(i & (kTabRows - 1));
      int valid, c = INT32_MAX;
      float cc = 0.f;
      double bound;
      if (T.rt[re] == (int)i) {
        valid = T.rv[re];
        bound = T.rb[re];
        if (lane < kCache) {
          c = T.rc[re * kCache + lane];
          cc = T.rx[re * kCache + lane];
        }
      } else {
        valid = w.cvalid[i];
        bound = w.cbound[i];
        if (lane < kCache) {
          c = w.ccol[i * kCache + lane];
          cc = w.ccost[i * kCache + lane];
          T.rc[re * kCache + lane] = c;
          T.rx[re * kCache + lane] = cc;
        }
        if (lane == 0) {
          T.rt[re] = (int)i;
          T.rv[re] = valid;
          T.rb[re] = bound;
        }
      }
      if (valid) {
        double cv = -DBL_MAX;
        int cj = INT32_MAX;
        double p = 0.0;
        uint32_t hd = 0;
        int own = -1;
        if (lane < kCache && c != INT32_MAX) {
          // price, holder and owner together: the resolve below needs no
          // read of its own when the bid is the cache's (one round trip less)
          const int e = c & (kTabCols - 1);
          if (T.ct[e] == c) {
            p = T.cp[e];
            hd = T.ch[e];
            own = T.co[e];
          } else {
            p = w.price[c];
            hd = w.holder[c];
            own = w.owner[c];
          }
          if (hd != mine) {  // held columns never bid
            cj = c;
            cv = -(double)cc - p;
          }
        }
        top2_16(cv, cj, b1, bj, b2);
        hit = b2 >= bound;
        if (!hit) {
          // the rescan's floor: the 16 cached columns and the last scan's
          // 17th (the bound's column) are 17 known values now, so the 17th
          // best overall is at least their minimum
          double fv = lane < kCache ? (c != INT32_MAX ? -(double)cc - p : -DBL_MAX) : DBL_MAX;
#pragma unroll
          for (int o = 8; o > 0; o >>= 1) fv = fmin(fv, __shfl_xor(fv, o, 64));
          const int jb = w.cbcol[i];
          const double vb = (jb >= 0 && jb < n) ? -(double)row[jb] - w.price[jb] : -DBL_MAX;
          floor = fmin(__shfl(fv, 0, 64), vb);
        }
        if (hit && bj != INT32_MAX) {
          const unsigned long long at = __ballot(c == bj && lane < kCache);
          const int L = __ffsll((long long)at) - 1;
          pj = __shfl(p, L, 64);
          hj = (uint32_t)__shfl((int)hd, L, 64);
          oj = __shfl(own, L, 64);
          have_j = true;
        }
      }
      if (!hit) {  // full scan over all columns, refill the cache (global + table)
        tsc0 = wall_clock64();
        scan(i, mine, floor);
        if (stalled) break;   // no lists: leave the row's cache and the slot as they are
        const double ev = lane < kCache + 1 ? outv[lane] : -DBL_MAX;
        const int ej = lane < kCache + 1 ? outj[lane] : INT32_MAX;
        if (lane < kCache) {
          const float c2 = ej != INT32_MAX ? row[ej] : 0.f;
          w.ccol[i * kCache + lane] = ej;
          w.ccost[i * kCache + lane] = c2;
          T.rc[re * kCache + lane] = ej;
          T.rx[re * kCache + lane] = c2;
        }
        if (lane == kCache) {
          w.cbound[i] = ev;
          w.cbcol[i] = ej;
          T.rb[re] = ev;
        }
        if (lane == 0) {
          w.cvalid[i] = 1;
          T.rv[re] = 1;
          T.rt[re] = (int)i;
        }
        double cv = -DBL_MAX;
        int cj = INT32_MAX;
        if (lane < kCache && ej != INT32_MAX && w.holder[ej] != mine) {
          cj = ej;
          cv = ev;
        }
        top2_16(cv, cj, b1, bj, b2);
      }
    } else {
      scan(i, mine, -DBL_MAX);
      if (stalled) break;
      b1 = outv[0];
      b2 = outv[1];
      bj = outj[0];
    }
    const unsigned long long t1 = wall_clock64();
    if (tsc0) {
      tl += tsc0 - t0;
      tsc += t1 - tsc0;
    } else {
      tl += t1 - t0;
    }
    // resolve on the spot (lane 0), the stack kept by the whole wave
    int old = -1;
    if (bj != INT32_MAX && lane == 0) {
      const double vref = (b2 > -DBL_MAX) ? b2 : b1;
      const double inc = b1 - vref + eps;
      float f = (float)inc;
      if ((double)f > inc) f = nextafterf(f, 0.f);  // round down: keeps eps-CS
      if (!(f > 0.f)) f = FLT_MIN;
      const int e = bj & (kTabCols - 1);
      double p;
      uint32_t h;
      int own;
      if (have_j) {
        p = pj;
        h = hj;
        own = oj;
      } else if (T.ct[e] == bj) {
        p = T.cp[e];
        h = T.ch[e];
        own = T.co[e];
      } else {
        p = w.price[bj];
        h = w.holder[bj];
        own = w.owner[bj];
      }
      p += (double)f;
      old = ((h & ~(uint32_t)(kMaxRows - 1)) == tag) ? own : -1;
      if (old >= 0)
        w.assigned[old] = -1;  // displaced: bids next
      else
        atomicAdd(&w.ctl->unassigned, (unsigned long long)(-1ll));
      T.ct[e] = bj;
      T.cp[e] = p;
      T.ch[e] = mine;
      T.co[e] = s;
      w.price[bj] = p;
      w.owner[bj] = s;
      w.holder[bj] = mine;
      w.assigned[s] = bj;
      w.assigned_ep[s] = ep;
    }
    old = __shfl(old, 0, 64);
    if (bj != INT32_MAX) {
      --sp;
      if (old >= 0) {
        if (lane == 0) stack[sp] = old;
        ++sp;
      }
    } else {
      --sp;  // no column to bid on (cannot happen with n slots = n columns)
    }
    // (no fence per bid: this wave's own later reads of these words are in
    // order after its writes; the helpers get one in scan())
    trs += wall_clock64() - t1;
  }
  // the launch's work, then release the helpers
  if (lane == 0) {
    atomicAdd(&w.ctl->tail_bids, (unsigned long long)nbids);
    atomicAdd(&w.ctl->tail_scans, (unsigned long long)nseq);
    atomicAdd(&w.ctl->tail_t[0], tl);
    atomicAdd(&w.ctl->tail_t[1], tsc);
    atomicAdd(&w.ctl->tail_t[2], trs);
    if (stalled) {   // no more tails this solve: the bid rounds finish the phase
      atomicExch(&mb->tail_off, 1u);
      atomicAdd(&mb->tail_stalls, 1u);
    }
    __hip_atomic_store(&mb->mb_seq, rtag | kQuit, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Rows in groups of four per workgroup-iteration (wave q: row base + q):
// each wave finds its row's free slots and, with the price cache, tries the
// cached bid; the rows left (no cache hit) are scanned one after the other by
// the whole workgroup (block_topk), which refills the cache and bids.  In the
// first round of a phase (fresh) the row's previous columns are kept where
// eps-CS allows (w2_keep) before its bid: with the cache's best value when
// the cache proves it the maximum over all columns, else after the scan.
__global__ __launch_bounds__(256) void w2_bid_cached_kernel(const float* __restrict__ C,
                                                            int64_t ldc, int64_t m, int64_t n,
                                                            int64_t R, W2Ws w) {
  constexpr int K = kCache + 1;
  __shared__ double sv[4 * K], outv[K];
  __shared__ int sj[4 * K], outj[K];
  __shared__ unsigned long long need[4];
  __shared__ int needkeep[4];
  const W2Ctl* ctl = w.ctl;
  if (ctl->done || ctl->tail) return;  // (uniform) the tail launch's round
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int ep = ctl->epoch;
  const double eps = ctl->eps;
  const bool fresh = ctl->fresh != 0;
  const uint32_t tag = w2_tag(ep);
  for (int64_t base = (int64_t)blockIdx.x * 4; base < m; base += (int64_t)gridDim.x * 4) {
    const int64_t i = base + wv;
    unsigned long long free = 0;
    if (i < m) {
      bool fr = false;
      if (lane < R) {
        const int64_t s = i * R + lane;
        fr = !(w.assigned_ep[s] == ep && w.assigned[s] >= 0);
      }
      free = __ballot(fr);
    }
    bool keep = free && fresh && w2_has_prev(i, R, lane, ep, w);
    bool scan = false;
    if (free && w.cvalid[i]) {  // wave-uniform: the cached bid
      const uint32_t mine = tag | (uint32_t)i;
      int c = INT32_MAX;
      double cval = -DBL_MAX;
      if (lane < kCache) {
        c = w.ccol[i * kCache + lane];
        if (c != INT32_MAX) cval = -(double)w.ccost[i * kCache + lane] - w.price[c];
      }
      const double bound = w.cbound[i];
      if (keep) {  // the row's best over all columns, if the cache proves it
        double b1 = cval;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) b1 = fmax(b1, __shfl_xor(b1, o, 64));
        if (b1 >= bound) {
          free &= ~w2_keep(C + i * ldc, i, R, lane, ep, mine, b1, eps, w);
          keep = false;
        } else {
          scan = true;
        }
      }
      if (!scan && free) {
        const int u = __popcll(free);
        double cv = -DBL_MAX;
        int cj = INT32_MAX;
        if (c != INT32_MAX && w.holder[c] != mine) {  // held columns never bid
          cj = c;
          cv = cval;
        }
        double kv;
        int kj;
        wave_best(cv, cj, u, lane, kv, kj);
        if (__shfl(kv, u, 64) >= bound)
          bid_from_best(kv, kj, u, i, R, free, lane, eps, w);
        else
          scan = true;
      }
    } else if (free) {
      scan = true;
    }
    if (lane == 0) {
      need[wv] = scan ? free : 0ull;
      needkeep[wv] = scan && keep;
    }
    __syncthreads();
    for (int q = 0; q < 4; ++q) {
      const unsigned long long fq = need[q];  // block-uniform
      if (fq == 0ull) continue;
      const int64_t iq = base + q;
      const uint32_t mine = tag | (uint32_t)iq;
      const float* row = C + iq * ldc;
      block_topk<K>(row, n, w, mine, false, sv, sj, outv, outj);
      if (wv == 0) {
        const double ev = lane < K ? outv[lane] : -DBL_MAX;
        const int ej = lane < K ? outj[lane] : INT32_MAX;
        if (lane < kCache) {
          w.ccol[iq * kCache + lane] = ej;
          w.ccost[iq * kCache + lane] = ej != INT32_MAX ? row[ej] : 0.f;
        }
        if (lane == kCache) {
          w.cbound[iq] = ev;
          w.cbcol[iq] = ej;
        }
        if (lane == 0) w.cvalid[iq] = 1;
        unsigned long long f2 = fq;
        if (needkeep[q]) f2 &= ~w2_keep(row, iq, R, lane, ep, mine, __shfl(ev, 0, 64), eps, w);
        if (f2) {
          // bid from the fresh list (current values), held columns excluded
          double cv = -DBL_MAX;
          int cj = INT32_MAX;
          if (lane < kCache && ej != INT32_MAX && w.holder[ej] != mine) {
            cj = ej;
            cv = ev;
          }
          const int u = __popcll(f2);
          double kv;
          int kj;
          wave_best(cv, cj, u, lane, kv, kj);
          bid_from_best(kv, kj, u, iq, R, f2, lane, eps, w);
        }
      }
      __syncthreads();  // sv / outv reused by the next row
    }
  }
}

// Without the cache (R = 1, R > kCacheMaxR): every bidding row is a full
// scan over the columns it does not hold, by the whole workgroup (in a fresh
// round nothing is held yet: the scan's best is over all columns, the keep
// test's reference, and the kept columns are then dropped from the list).
template <int K>
__global__ __launch_bounds__(256) void w2_bid_kernel(const float* __restrict__ C, int64_t ldc,
                                                     int64_t m, int64_t n, int64_t R, W2Ws w) {
  __shared__ double sv[4 * K], outv[K];
  __shared__ int sj[4 * K], outj[K];
  __shared__ unsigned long long need[4];
  __shared__ int needkeep[4];
  const W2Ctl* ctl = w.ctl;
  if (ctl->done || ctl->tail) return;  // (uniform) the tail launch's round
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int ep = ctl->epoch;
  const double eps = ctl->eps;
  const bool fresh = ctl->fresh != 0;
  const uint32_t tag = w2_tag(ep);
  for (int64_t base = (int64_t)blockIdx.x * 4; base < m; base += (int64_t)gridDim.x * 4) {
    const int64_t i = base + wv;
    unsigned long long free = 0;
    if (i < m) {
      bool fr = false;
      if (lane < R) {
        const int64_t s = i * R + lane;
        fr = !(w.assigned_ep[s] == ep && w.assigned[s] >= 0);
      }
      free = __ballot(fr);
    }
    const bool keep = free && fresh && w2_has_prev(i, R, lane, ep, w);
    if (lane == 0) {
      need[wv] = free;
      needkeep[wv] = keep;
    }
    __syncthreads();
    for (int q = 0; q < 4; ++q) {
      const unsigned long long fq = need[q];  // block-uniform
      if (fq == 0ull) continue;
      const int64_t iq = base + q;
      const uint32_t mine = tag | (uint32_t)iq;
      const float* row = C + iq * ldc;
      block_topk<K>(row, n, w, mine, true, sv, sj, outv, outj);
      if (wv == 0) {
        unsigned long long f2 = fq;
        double kv = -DBL_MAX;
        int kj = INT32_MAX;
        if (needkeep[q]) {
          f2 &= ~w2_keep(row, iq, R, lane, ep, mine, outv[0], eps, w);
          if (f2) {
            double cv = -DBL_MAX;
            int cj = INT32_MAX;
            if (lane < K && outj[lane] != INT32_MAX && w.holder[outj[lane]] != mine) {
              cj = outj[lane];
              cv = outv[lane];
            }
            wave_best(cv, cj, __popcll(f2), lane, kv, kj);
          }
        } else {
          const int u = __popcll(fq);
          kv = lane <= u && lane < K ? outv[lane] : -DBL_MAX;
          kj = lane <= u && lane < K ? outj[lane] : INT32_MAX;
        }
        if (f2) bid_from_best(kv, kj, __popcll(f2), iq, R, f2, lane, eps, w);
      }
      __syncthreads();
    }
  }
}

// The first round of a fused R = 1 warm start (w2_scan_first_kernel): row i's
// one slot bids for its best column with the row's best and second values,
// as bid_from_best with u = 1 -- one thread per row, no scan.
__global__ __launch_bounds__(256) void w2_bid_first_kernel(int64_t m, W2Ws w) {
  const W2Ctl* ctl = w.ctl;
  if (ctl->done || ctl->tail) return;  // (uniform) as w2_bid_kernel
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= m) return;
  const int kj = w.ccol[i];
  if (kj == INT32_MAX) return;
  const double kv = w.cbound[i], vu1 = reinterpret_cast<const double*>(w.ccost)[i];
  const double vref = (vu1 > -DBL_MAX) ? vu1 : kv;
  const double inc = kv - vref + ctl->eps;
  float f = (float)inc;
  if ((double)f > inc) f = nextafterf(f, 0.f);  // round down: keeps eps-CS
  if (!(f > 0.f)) f = FLT_MIN;
  const unsigned long long key =
      ((unsigned long long)__float_as_uint(f) << 32) | (unsigned long long)(uint32_t)i;
  atomicMax(&w.bid[kj], key);
}

__device__ void w2_control(W2Ctl* ctl, int64_t n) {
  ctl->rounds += 1;
  ctl->fresh = 0;
  const unsigned long long un =
      __hip_atomic_load(&ctl->unassigned, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (un != 0) {
    ctl->tail = !ctl->tail_off && un <= (unsigned long long)kTailMax;
    return;
  }
  if (ctl->eps <= ctl->eps_final) {
    ctl->done = 1;
    return;
  }
  ctl->eps = fmax(ctl->eps / ctl->theta, ctl->eps_final);
  ctl->epoch += 1;
  ctl->phases += 1;
  ctl->unassigned = (unsigned long long)n;
  ctl->fresh = ctl->keep_on;  // the next round keeps what still meets eps-CS
  ctl->tail = !ctl->tail_off && n <= kTailMax;
}

// One thread per column: award the column to its highest bidder; the last
// block to arrive runs the control step (release/acquire ticket,
// cdna_hip_programming.md Guideline 16).  `done` is uniform over the grid:
// only the last arriver writes it, after every block has read it.
__global__ __launch_bounds__(256) void w2_resolve_kernel(int64_t n, int64_t R, W2Ws w) {
  W2Ctl* ctl = w.ctl;
  if (ctl->done) return;
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  unsigned long long gained = 0;
  if (j < n) {
    const unsigned long long b = w.bid[j];
    if (b) {
      w.bid[j] = 0;
      const int s = (int)(uint32_t)b;
      const float inc = __uint_as_float((uint32_t)(b >> 32));
      const int ep = ctl->epoch;
      const uint32_t tag = w2_tag(ep);
      w.price[j] += (double)inc;
      const uint32_t h = w.holder[j];
      const int old = ((h & ~(uint32_t)(kMaxRows - 1)) == tag) ? w.owner[j] : -1;
      if (old >= 0)
        w.assigned[old] = -1;  // displaced: bids again next round
      else
        gained = 1;
      w.owner[j] = s;
      w.holder[j] = tag | (uint32_t)(s / R);
      w.assigned[s] = (int)j;
      w.assigned_ep[s] = ep;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) gained += __shfl_xor(gained, o, 64);
  if ((threadIdx.x & 63) == 0 && gained)
    atomicAdd(&ctl->unassigned, (unsigned long long)(-(long long)gained));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t =
        __hip_atomic_fetch_add(&ctl->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == gridDim.x - 1) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      ctl->ticket = 0;
      w2_control(ctl, n);
    }
  }
}

__global__ __launch_bounds__(256) void w2_emit_kernel(int64_t n, W2Ws w, int32_t* assign) {
  const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (s >= n) return;
  assign[s] = (w.ctl->done == 2) ? (int32_t)s : w.assigned[s];
}

// G[i][c] = h/n * sum_{r<R} (x_i - y_{assign[iR+r]})[c]   (distsampler.py:128
// times the JKO step h of :198)
__global__ __launch_bounds__(256) void w2_grad_kernel(const float* __restrict__ X, int64_t ldx,
                                                      int64_t m, const float* __restrict__ Y,
                                                      int64_t ldy, int64_t n, int64_t d,
                                                      const int32_t* __restrict__ assign,
                                                      float h, float* __restrict__ G,
                                                      int64_t ldg) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= m * d) return;
  const int64_t i = t / d, c = t % d, R = n / m;
  const float x = X[i * ldx + c];
  float acc = 0.f;
  for (int64_t r = 0; r < R; ++r) acc += x - Y[(int64_t)assign[i * R + r] * ldy + c];
  G[i * ldg + c] = h * (acc / (float)n);
}

}  // namespace dsvgd

using namespace dsvgd;

// phases keep the last plan's eps-CS slots (default off: every phase and
// warm start re-assigns all slots; on measured slower warm, profiles/r11g)
static bool& w2_keep_flag() {
  static bool k = false;
  return k;
}

// the last dsvgd_w2_assign's tail work on this host thread: (bids, scans,
// three times, stalls)
static long long* w2_tail_stats() {
  static thread_local long long st[6] = {0, 0, 0, 0, 0, 0};
  return st;
}

// tests: the tails' helpers exit at once (a stall on every tail launch)
static bool& w2_nohelp_flag() {
  static bool k = false;
  return k;
}

// R = 1 warm starts: the violation and the first round's scans in one pass
// (w2_scan_first_kernel; default on, dsvgd_w2_set_fuse_first)
static bool& w2_fuse_first_flag() {
  static bool k = true;
  return k;
}

// eps divisor between phases (default kTheta; A/B: dsvgd_w2_set_theta)
static double& w2_theta() {
  static double th = kTheta;
  return th;
}

// the last dsvgd_w2_assign's progress on this host thread: (rounds, phase,
// unassigned slots) at every control readback (kRoundBatch rounds apart)
static std::vector<long long>& w2_trace() {
  static thread_local std::vector<long long> t;
  return t;
}

extern "C" {

int64_t dsvgd_w2_trace(int64_t* out, int64_t cap) {
  const std::vector<long long>& t = w2_trace();
  const int64_t k = (int64_t)t.size() / 3;
  for (int64_t e = 0; out && e < std::min(k, cap) * 3; ++e) out[e] = t[e];
  return k;
}

int dsvgd_w2_set_keep(int keep) {
  const int old = w2_keep_flag() ? 1 : 0;
  w2_keep_flag() = keep != 0;
  return old;
}

int64_t dsvgd_w2_tail_stats(int64_t* out) {
  if (out) {
    for (int k = 0; k < 6; ++k) out[k] = w2_tail_stats()[k];
  }
  return 6;
}

int dsvgd_w2_set_fuse_first(int on) {
  const int old = w2_fuse_first_flag() ? 1 : 0;
  w2_fuse_first_flag() = on != 0;
  return old;
}

int dsvgd_w2_set_tail_debug(int nohelp) {
  const int old = w2_nohelp_flag() ? 1 : 0;
  w2_nohelp_flag() = nohelp != 0;
  return old;
}

double dsvgd_w2_set_theta(double theta) {
  const double old = w2_theta();
  if (theta >= 2.0 && theta <= 1024.0) w2_theta() = theta;
  return old;
}

size_t dsvgd_w2_workspace_bytes(int64_t m, int64_t n) {
  return kW2CtlBytes + (size_t)n * (sizeof(double) + sizeof(unsigned long long) + 4 * sizeof(int32_t)) +
         8 + (size_t)m * (sizeof(double) + kCache * (sizeof(int32_t) + sizeof(float)) + sizeof(int32_t)) +
         8 + (size_t)kTailHelpers * kTailListMax * (sizeof(double) + sizeof(int32_t)) +
         (size_t)m * sizeof(int32_t);
}

int dsvgd_w2_cost(const float* X, int64_t ldx, int64_t m, const float* Y, int64_t ldy, int64_t n,
                  int64_t d, float* C, int64_t ldc, void* stream) {
  DSVGD_REQUIRE(X && Y && C, "null pointer");
  DSVGD_REQUIRE(m > 0 && n > 0 && d > 0 && ldx >= d && ldy >= d && ldc >= n, "sizes");
  DSVGD_REQUIRE((n + kCostTile - 1) / kCostTile <= INT32_MAX &&
                    (m + kCostTile - 1) / kCostTile <= 65535,
                "grid too large");
  hipLaunchKernelGGL(w2_cost_kernel,
                     dim3((n + kCostTile - 1) / kCostTile, (m + kCostTile - 1) / kCostTile),
                     dim3(256), 0,
                     (hipStream_t)stream, X, ldx, m, Y, ldy, n, d, C, ldc);
  return check_launch("w2_cost");
}

static int w2_assign(const float* C, int64_t ldc, int64_t m, int64_t n, void* ws,
                     int64_t max_rounds, int warm_phases, const int32_t* prev, int32_t* assign,
                     int64_t* rounds_out, void* stream, const uint32_t* cstat);

int dsvgd_w2_assign(const float* C, int64_t ldc, int64_t m, int64_t n, void* ws,
                    int64_t max_rounds, int warm_phases, int32_t* assign, int64_t* rounds_out,
                    void* stream) {
  DSVGD_REQUIRE(warm_phases >= 0, "warm_phases");
  return w2_assign(C, ldc, m, n, ws, max_rounds, warm_phases, nullptr, assign, rounds_out, stream,
                   nullptr);
}

int dsvgd_w2_assign_warm(const float* C, int64_t ldc, int64_t m, int64_t n, void* ws,
                         int64_t max_rounds, const int32_t* prev_assign, int32_t* assign,
                         int64_t* rounds_out, void* stream) {
  DSVGD_REQUIRE(prev_assign, "null prev_assign");
  return w2_assign(C, ldc, m, n, ws, max_rounds, -1, prev_assign, assign, rounds_out, stream,
                   nullptr);
}

int dsvgd_w2_assign_stat(const float* C, int64_t ldc, int64_t m, int64_t n, void* ws,
                         int64_t max_rounds, int warm_phases, const int32_t* prev_assign,
                         int32_t* assign, int64_t* rounds_out, const uint32_t* cstat,
                         void* stream) {
  DSVGD_REQUIRE(cstat, "null cstat");
  DSVGD_REQUIRE(prev_assign || warm_phases >= 0, "warm_phases");
  return w2_assign(C, ldc, m, n, ws, max_rounds, prev_assign ? -1 : warm_phases, prev_assign,
                   assign, rounds_out, stream, cstat);
}

static int w2_assign(const float* C, int64_t ldc, int64_t m, int64_t n, void* ws,
                     int64_t max_rounds, int warm_phases, const int32_t* prev, int32_t* assign,
                     int64_t* rounds_out, void* stream, const uint32_t* cstat) {
  DSVGD_REQUIRE(C && ws && assign, "null pointer");
  DSVGD_REQUIRE(m > 0 && n > 0 && ldc >= n, "sizes");
  DSVGD_REQUIRE(n % m == 0, "n must be a multiple of m (n = R m slots)");
  DSVGD_REQUIRE(n <= INT32_MAX - 1, "n too large for 32-bit slot ids");
  DSVGD_REQUIRE(m < kMaxRows, "m too large (2^21 rows)");
  DSVGD_REQUIRE(n / m <= kMaxR, "n / m must be <= 32 (slots per row)");
  DSVGD_REQUIRE(max_rounds > 0, "max_rounds");
  hipStream_t s = (hipStream_t)stream;
  W2Ws w(ws, n, m);
  const int64_t R = n / m;
  // warm start keeps the price array (the previous call's duals on this
  // workspace); everything else restarts
  const size_t prices = (size_t)n * sizeof(double);
  const size_t total_b = dsvgd_w2_workspace_bytes(m, n);
  if ((warm_phases == 0 && hipMemsetAsync(ws, 0, total_b, s) != hipSuccess) ||
      (warm_phases != 0 &&
       (hipMemsetAsync(ws, 0, kW2CtlBytes, s) != hipSuccess ||
        hipMemsetAsync((char*)ws + kW2CtlBytes + prices, 0, total_b - kW2CtlBytes - prices, s) !=
            hipSuccess)))
    return check_launch("w2 workspace memset");
  if (cstat) {  // taken while the cost was written (dsvgd_w2_cost_h2)
    hipLaunchKernelGGL(w2_cstat_kernel, dim3(1), dim3(64), 0, s, cstat, w.ctl);
  } else {
    const int cblocks = (int)std::min<int64_t>(4096, m * ((n + 2047) / 2048));
    hipLaunchKernelGGL(w2_cmax_kernel, dim3(cblocks), dim3(256), 0, s, C, ldc, m, n, w.ctl);
  }
  const bool keep = w2_keep_flag();
  const bool rows4 = n % 4 == 0 && ldc % 4 == 0 && ((uintptr_t)C & 15) == 0;
  // R = 1 warm start: the violation and the first round's scans in one pass
  bool fused_first = prev && rows4 && R == 1 && !keep && w2_fuse_first_flag();
  if (fused_first)
    hipLaunchKernelGGL(w2_scan_first_kernel, dim3((unsigned)((m + kViolRows - 1) / kViolRows)),
                       dim3(256), 0, s, C, ldc, m, n, prev, w);
  else if (prev && rows4)
    hipLaunchKernelGGL(w2_violation_rows_kernel, dim3((unsigned)((m + kViolRows - 1) / kViolRows)),
                       dim3(256), 0, s, C, ldc, m, n, n / m, prev, w);
  else if (prev)
    hipLaunchKernelGGL(w2_violation_kernel, dim3((unsigned)std::min<int64_t>(1024, (m + 3) / 4)),
                       dim3(256), 0, s, C, ldc, m, n, n / m, prev, w);
  if (prev && keep)
    hipLaunchKernelGGL(w2_load_prev_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n,
                       prev, w);
  const dim3 gb((unsigned)std::min<int64_t>(kBidBlocks, (m + 3) / 4));
  // the phase tail: one workgroup, its LDS tables as dynamic LDS
  const bool cached = kW2Cache && R >= 2 && R <= kCacheMaxR;
  const void* tail_fn = cached ? reinterpret_cast<const void*>(&w2_tail_kernel<2, true>)
                      : R <= 1 ? reinterpret_cast<const void*>(&w2_tail_kernel<2, false>)
                      : R <= 2 ? reinterpret_cast<const void*>(&w2_tail_kernel<3, false>)
                      : R <= 4 ? reinterpret_cast<const void*>(&w2_tail_kernel<5, false>)
                      : R <= 8 ? reinterpret_cast<const void*>(&w2_tail_kernel<9, false>)
                      : R <= 16 ? reinterpret_cast<const void*>(&w2_tail_kernel<17, false>)
                                : reinterpret_cast<const void*>(&w2_tail_kernel<33, false>);
  if (hipFuncSetAttribute(tail_fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kTailLds) !=
      hipSuccess)
    return fail_arg("w2 tail: cannot reserve its LDS tables");
  // the tail's helpers poll a mailbox beside workgroup 0: if the device
  // cannot hold all 1 + kTailHelpers workgroups at once even when idle, the
  // solve runs without tails (bid rounds only)
  int occ = 0, cus = 0, dev = 0;
  const bool resident =
      hipGetDevice(&dev) == hipSuccess &&
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, tail_fn, kTailThreads, kTailLds) ==
          hipSuccess &&
      (int64_t)occ * cus >= 1 + kTailHelpers;
  // keep bit 0: phases keep eps-CS slots; bit 1: the first round keeps prev's
  hipLaunchKernelGGL(w2_start_kernel, dim3(1), dim3(1), 0, s, w.ctl, n, warm_phases,
                     (keep ? 1 : 0) | ((prev && keep) ? 2 : 0), w2_theta(), resident ? 0 : 1,
                     w2_nohelp_flag() ? 1 : 0);
  int rc = check_launch("w2_start");
  if (rc) return rc;
  auto bid = [&]() {
    if (fused_first) {  // round 1 from the scan pass's row results (R = 1: not cached)
      hipLaunchKernelGGL(w2_bid_first_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s,
                         m, w);
      hipLaunchKernelGGL((w2_tail_kernel<2, false>), dim3(1 + kTailHelpers), dim3(kTailThreads),
                         kTailLds, s, C, ldc, n, R, w);
      fused_first = false;
      return;
    }
    if (cached) {
      hipLaunchKernelGGL(w2_bid_cached_kernel, gb, dim3(256), 0, s, C, ldc, m, n, R, w);
      hipLaunchKernelGGL((w2_tail_kernel<2, true>), dim3(1 + kTailHelpers), dim3(kTailThreads),
                         kTailLds, s, C, ldc, n, R,
                         w);
      return;
    }
#define DSVGD_W2_BID(KK)                                                                       \
  do {                                                                                         \
    hipLaunchKernelGGL(w2_bid_kernel<KK>, gb, dim3(256), 0, s, C, ldc, m, n, R, w);            \
    hipLaunchKernelGGL((w2_tail_kernel<KK, false>), dim3(1 + kTailHelpers), dim3(kTailThreads),    \
                       kTailLds, s, C, ldc, n,                                                  \
                       R, w);                                                                  \
  } while (0)
    if (R <= 1)
      DSVGD_W2_BID(2);
    else if (R <= 2)
      DSVGD_W2_BID(3);
    else if (R <= 4)
      DSVGD_W2_BID(5);
    else if (R <= 8)
      DSVGD_W2_BID(9);
    else if (R <= 16)
      DSVGD_W2_BID(17);
    else
      DSVGD_W2_BID(33);
#undef DSVGD_W2_BID
  };
  const dim3 gr((unsigned)((n + 255) / 256));
  // pinned, double-buffered control readback (one pair per host thread)
  static thread_local W2Ctl* hbuf = nullptr;
  if (!hbuf && hipHostMalloc((void**)&hbuf, 2 * sizeof(W2Ctl), hipHostMallocDefault) != hipSuccess) {
    hbuf = nullptr;
    return check_launch("w2 pinned control buffer");
  }
  hipEvent_t ev[2];
  if (hipEventCreateWithFlags(&ev[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ev[1], hipEventDisableTiming) != hipSuccess)
    return check_launch("w2 events");
  W2Ctl h{};
  rc = 0;
  w2_trace().clear();
  for (int64_t batch = 0;; ++batch) {
    for (int b = 0; b < kRoundBatch; ++b) {
      bid();
      hipLaunchKernelGGL(w2_resolve_kernel, gr, dim3(256), 0, s, n, R, w);
    }
    W2Ctl* slot = hbuf + (batch & 1);
    if ((rc = check_launch("w2 auction round")) ||
        hipMemcpyAsync(slot, w.ctl, sizeof(W2Ctl), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipEventRecord(ev[batch & 1], s) != hipSuccess) {
      rc = rc ? rc : check_launch("w2 control readback");
      break;
    }
    if (batch == 0) continue;  // keep one batch queued ahead of the poll
    if (hipEventSynchronize(ev[(batch - 1) & 1]) != hipSuccess) {
      rc = check_launch("w2 control readback");
      break;
    }
    h = hbuf[(batch - 1) & 1];
    w2_trace().insert(w2_trace().end(), {h.rounds, h.phases, (long long)h.unassigned});
    w2_tail_stats()[0] = (long long)h.tail_bids;
    w2_tail_stats()[1] = (long long)h.tail_scans;
    for (int k = 0; k < 3; ++k) w2_tail_stats()[2 + k] = (long long)(h.tail_t[k] / 100);  // us
    w2_tail_stats()[5] = (long long)h.tail_stalls;
    if (h.done) break;
    if ((batch - 1) * kRoundBatch >= max_rounds) {
      set_error("dsvgd_w2_assign: no convergence after %lld rounds (%lld phases, %llu unassigned)",
                (long long)h.rounds, (long long)h.phases, (unsigned long long)h.unassigned);
      rc = -3;
      break;
    }
  }
  // the batch queued after the poll is a no-op once done is set; make the
  // pinned slots quiescent before the next call reuses them
  if (hipStreamSynchronize(s) != hipSuccess && !rc) rc = check_launch("w2 drain");
  (void)hipEventDestroy(ev[0]);
  (void)hipEventDestroy(ev[1]);
  if (rc) return rc;
  if (h.done == 3) {
    set_error("dsvgd_w2_assign: non-finite or negative cost");
    return -2;
  }
  if (rounds_out) *rounds_out = h.rounds;
  hipLaunchKernelGGL(w2_emit_kernel, gr, dim3(256), 0, s, n, w, assign);
  return check_launch("w2_emit");
}

int dsvgd_w2_grad(const float* X, int64_t ldx, int64_t m, const float* Y, int64_t ldy, int64_t n,
                  int64_t d, const int32_t* assign, float h, float* G, int64_t ldg, void* stream) {
  DSVGD_REQUIRE(X && Y && assign && G, "null pointer");
  DSVGD_REQUIRE(m > 0 && n > 0 && d > 0 && ldx >= d && ldy >= d && ldg >= d, "sizes");
  DSVGD_REQUIRE(n % m == 0, "n must be a multiple of m");
  hipLaunchKernelGGL(w2_grad_kernel, dim3((unsigned)((m * d + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, X, ldx, m, Y, ldy, n, d, assign, h, G, ldg);
  return check_launch("w2_grad");
}

}  // extern "C"
