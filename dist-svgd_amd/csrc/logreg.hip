// logreg.hip -- batched score of the Bayesian logistic-regression posterior
// of experiments/logreg.py:45-58 for ALL n particles at once, replacing the
// per-particle autograd _dlogp (dsvgd/sampler.py:28-33, distsampler.py:77-82):
//
//   x = [log a, w],  log p = log Gamma(1,1)(a) + log N(w; 0, I/a) - sum_q log(1+exp(-t_q xd_q.w))
//   d/dx0 = -a + p/2 - (a/2)|w|^2          d/dw = -a w + sum_q t_q xd_q sigma(-t_q xd_q.w)
//
// as Z = W Xd^T (NT MFMA engine, sigmoid epilogue -> G in panel layout) and
// G Xd (NN MFMA engine); 4 n N p flop, MFMA-bound.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <string>
#include <type_traits>

#include "gemm_tiles.hpp"
#include "gemm_x3.hpp"

namespace dsvgd {

int nn_gemm(bool exp_, const float* A, int64_t K, const float* B, int64_t ldb, int64_t cols,
            int splits, const dsvgd_select_state* st, float* C, int64_t ldc, float* rowsum,
            int64_t m, int64_t row0, hipStream_t s, const float* gate);
int nn_x3_gemm(bool exp_, const float* A, int64_t K, const __bf16* Yx, int64_t ldy, int splits,
               const dsvgd_select_state* st, float* C, int64_t ldc, float* rowsum, int64_t m,
               int64_t row0, hipStream_t s, int sym, int m16, const float* gate);
int nn_h2_gemm(bool exp_, const float* A, int64_t K, const _Float16* Yh, int64_t ldy, int splits,
               const dsvgd_select_state* st, float* C, int64_t ldc, float* rowsum, int64_t m,
               int64_t row0, hipStream_t s, int sym, const float* colinv, const float* gate);
int h2_colscale(const float* A, int64_t lda, int64_t rows, int64_t cols, int64_t dp, float* ws, float* out,
                hipStream_t s);
int h2_ysplit(const float* Y, int64_t ldy, int64_t rows, const float* colscale, void* Yh,
              hipStream_t s);
int h2_rowsplit(const float* A, int64_t lda, int64_t rows, int64_t cols, int64_t rows_pad,
                int64_t kpad, const float* tscale, void* img, hipStream_t s);
int h2_rowsplit_rows(const float* A, int64_t lda, int64_t rows, int64_t cols, int64_t rows_pad,
                     int64_t kpad, const float* rscale, void* img, hipStream_t s);
int h2_rowscale(const float* A, int64_t lda, int64_t rows, int64_t cols, int64_t rows_pad,
                float* rscale, float* rinv, hipStream_t s);
int h2_rowimage(const float* A, int64_t lda, int64_t rows, int64_t cols, int64_t rows_pad,
                int64_t kpad, float* rscale, float* rinv, void* img, hipStream_t s);
size_t h2_colscale_ws_floats(int64_t rows, int64_t cols);

static int64_t nn_cols(int64_t w) {
  if (w <= 128) return 128;
  if (w <= 256) return 256;
  return roundup(w, 512);
}

struct LogregWs {
  int64_t N, n_pad, N_pad, pp, ldb;
  size_t off_w, off_xd, off_t, off_g, off_gw, off_wx, off_xdx, off_xdy, off_rsw, off_riw, off_sxd,
      off_sws, off_xdp, total;
};

// G . Xd (K = N data rows, 256-row blocks): split K so that a launch has
// about two blocks per CU (n = 65536 gives only 256 row blocks), each slice
// at least 1024 rows deep; logreg_finish adds the slices in order.
constexpr int kGxdMaxSplits = 1;  // 2, 4 measured slower at S = 8
static int gxd_splits(int64_t n_pad, int64_t N_pad) {
  int sp = 1;
  while (sp < kGxdMaxSplits && (n_pad / 256) * sp < 512 && N_pad / (2 * sp) >= 1024) sp *= 2;
  return sp;
}

// the FmtH2 score as one fused kernel (1, default: 2.93-3.05 vs 3.37 ms at
// n = 65536, N = 16384; 0.48 vs 0.50 at N = 2048, profiles/r13v) or Z +
// G . Xd (0); dsvgd_logreg_set_fused
static int g_logreg_fused = 1;

// The fused score over data slices: a block is 128 particles, so a few
// particles (a rank's own block in DistSampler's gathered-data all_scores:
// m = 8192 at S = 8, 64 blocks) leave most CUs idle.  Split the data chunks
// into Z slices (blocks (x, z)) until the launch covers the CUs, each slice
// at least 16 chunks (512 data rows); logreg_finish adds the slices in order.
// Z = 1 (the same launch and bits as before) whenever n fills the CUs alone.
// The slices are equal: N_pad is a multiple of 256 = 8 chunks and Z | 8.
constexpr int kFusedMaxSplits = 8;
static int fused_splits(int64_t n_pad, int64_t N_pad) {
  int z = 1;
  while (z < kFusedMaxSplits && (n_pad / 128) * z < 256 && (N_pad / 32) / (2 * z) >= 16) z *= 2;
  return z;
}

static LogregWs logreg_ws(int64_t n, int64_t N, int64_t p) {
  LogregWs w;
  w.N = N;
  w.n_pad = roundup(n, 256);  // whole 256 x 256 Z tiles
  w.N_pad = roundup(N, 256);
  w.pp = roundup(p < 1 ? 1 : p, 32);
  w.ldb = nn_cols(w.pp);
  size_t o = 0;
  auto take = [&](size_t floats) {
    size_t at = o;
    o += roundup((int64_t)(floats * sizeof(float)), 256);
    return at;
  };
  w.off_w = take((size_t)w.n_pad * w.ldb);
  w.off_xd = take((size_t)w.N_pad * w.ldb);
  w.off_t = take((size_t)w.N_pad);
  w.off_g = take((size_t)w.n_pad * w.N_pad);
  // split-K slices of G . Xd (two-GEMM path) or of the fused score
  w.off_gw = take((size_t)std::max(kGxdMaxSplits, fused_splits(w.n_pad, w.N_pad)) * w.n_pad *
                  w.ldb);
  // split images (bf16 x 3 = 6 B per element, counted in floats)
  w.off_wx = take((size_t)w.n_pad * w.pp * 3 / 2);
  w.off_xdx = take((size_t)w.N_pad * w.pp * 3 / 2);
  w.off_xdy = take((size_t)w.N_pad * w.ldb * 3 / 2);
  // FmtH2 scales: per-row of W = X[:, 1:] (scale, inverse), of Xd
  // (dsvgd_h2_colscale layout), + scratch
  w.off_rsw = take((size_t)w.n_pad);
  w.off_riw = take((size_t)w.n_pad);
  w.off_sxd = take((size_t)(2 * w.ldb + 3));
  w.off_sws = take(h2_colscale_ws_floats(w.N_pad, w.ldb));
  // the fused score's column image of Xd, K order permuted (FmtH2, 4 B per entry)
  w.off_xdp = take((size_t)w.N_pad * w.ldb);
  w.total = o;
  return w;
}

// dst[r][c] = src[r][c0 + c] for r < rows, c < cols; zero elsewhere (rows_pad x ldd)
__global__ __launch_bounds__(256) void pad_copy_kernel(const float* __restrict__ src, int64_t lds,
                                                       int64_t c0, int64_t rows, int64_t cols,
                                                       int64_t rows_pad, float* __restrict__ dst,
                                                       int64_t ldd) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= rows_pad * ldd) return;
  const int64_t r = t / ldd, c = t % ldd;
  dst[t] = (r < rows && c < cols) ? src[r * lds + c0 + c] : 0.f;
}

// Xd[q][:] *= t[q] (then set_ones_kernel makes t = 1: rows past N had t = 0,
// so they stay zero rows); the Z epilogue's t_q sigma(-t_q z) is then
// sigma(-z') on the folded data.
__global__ __launch_bounds__(256) void fold_labels_kernel(float* __restrict__ Xd,
                                                          const float* __restrict__ t,
                                                          int64_t rows, int64_t ld) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e < rows * ld) Xd[e] *= t[e / ld];
}

__global__ __launch_bounds__(256) void set_ones_kernel(float* __restrict__ v, int64_t n) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e < n) v[e] = 1.f;
}

__device__ __forceinline__ float sigmoidf_stable(float u) {
  if (u >= 0.f) return 1.f / (1.f + expf(-u));
  const float e = expf(u);
  return e / (1.f + e);
}

// G[j][q] = t_q sigma(-t_q (w_j . xd_q)) = t_q / (1 + exp(t_q z)); after
// logreg_prepare's fold (xd' = t xd, t = 1) this is sigma(-z') in (0, 1), and
// padded q hold sigma(0) against a zero data row; panel layout.  The epilogue is VALU work beside
// the other resident blocks' f32 MFMAs (they share the SIMD's issue), so it
// is kept short: exp2 + rcp (~1 ulp each) and store addresses that are one
// per-lane base plus compile-time offsets (as the distance epilogue).
// Tile: 128 x 128, 4 waves of 64 x 64 (measured: a 256 x 128 tile with
// 128 accumulators per wave at 2 waves/SIMD is 6 % slower).
using ZTile = NTTile<2, 2, 2, 2>;

template <class T, class = void>
struct IsM16 : std::false_type {};
template <class T>
struct IsM16<T, std::void_t<decltype(T::M16_)>> : std::integral_constant<bool, T::M16_> {};

// zs: 1 / (Xd's FmtH2 tensor scale), 1 otherwise; rinv (FmtH2): 1 / (W row
// i's scale) per row i -- z_iq = rinv_i zs acc_iq, both exact powers of two
template <class T>
__device__ __forceinline__ void z_epilogue(T& tile, int64_t i0, int64_t q0,
                                           const float* __restrict__ tp, int64_t N_pad,
                                           float* __restrict__ G, float zs = 1.f,
                                           const float* __restrict__ rinv = nullptr) {
  if constexpr (IsM16<T>::value) {  // 16x16 tiles: column lane & 15, rows 4 (lane >> 4) + reg
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w / T::WN_, wn = w % T::WN_;
#pragma unroll
    for (int nt = 0; nt < 2 * T::TN_; ++nt) {
      const int64_t q = q0 + wn * 32 * T::TN_ + nt * 16 + (lane & 15);
      const float tq = tp[q];
      const float sc = tq * kLog2e;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const int64_t i = i0 + wm * 64 + mt * 16 + 4 * (lane >> 4);  // 4 rows in one panel
        float* const g0 = G + ((i >> 7) * (N_pad >> 4) + (q >> 4)) * kPanelElems + (q & 15) +
                          (i & 127) * 16;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = __builtin_amdgcn_exp2f(sc * tile.acc16[mt][nt][r]);
          __builtin_nontemporal_store(tq * __builtin_amdgcn_rcpf(1.f + e), g0 + r * 16);
        }
      }
    }
    return;
  }
  constexpr int WR = 32 * T::TM_, WC = 32 * T::TN_;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w / T::WN_, wn = w % T::WN_;
  const int h4 = 4 * (lane >> 5);
  // the 16 rows of each mi this lane holds: i + (r & 3) + 8 (r >> 2)
  f32x4 ri[T::TM_][4];
#pragma unroll
  for (int mi = 0; mi < T::TM_; ++mi)
#pragma unroll
    for (int g = 0; g < 4; ++g)
      ri[mi][g] = rinv ? *reinterpret_cast<const f32x4*>(rinv + i0 + wm * WR + mi * 32 + h4 + 8 * g)
                       : f32x4{1.f, 1.f, 1.f, 1.f};
#pragma unroll
  for (int ni = 0; ni < T::TN_; ++ni) {
    const int64_t q = q0 + wn * WC + ni * 32 + (lane & 31);
    const float tq = tp[q];
    const float sc = tq * kLog2e * zs;
#pragma unroll
    for (int mi = 0; mi < T::TM_; ++mi) {
      const int64_t i = i0 + wm * WR + mi * 32 + h4;  // 32-row group: one 128-row panel
      float* const g0 = G + ((i >> 7) * (N_pad >> 4) + (q >> 4)) * kPanelElems + (q & 15) +
                        (i & 127) * 16;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float a = rinv ? ri[mi][r >> 2][r & 3] * tile.acc[mi][ni][r] : tile.acc[mi][ni][r];
        const float e = __builtin_amdgcn_exp2f(sc * a);
        __builtin_nontemporal_store(tq * __builtin_amdgcn_rcpf(1.f + e),
                                    g0 + (r & 3) * 16 + (r >> 2) * 128);  // nt: G streams out
      }
    }
  }
}

// Persistent form: a grid of one block per CU walks each XCD's L2-grouped
// range of 256 x 256 tiles (sqdist_x3w_kernel's schedule) through a 2-stage
// DMA ring that runs across tile boundaries: the next tile's first K-step
// lands while this one's epilogue (exp2, rcp, G stores) runs.
// F = FmtX3: 16x16x32 (unswizzled W / Xd images); FmtH2: 32x32x16 on the
// swizzled fp16 images of s_i w_i (a power-of-two scale per particle row:
// no particle's weights fall below another's fp16 window) and t_x Xd
// (xinv = 1/t_x, rinv[i] = 1/s_i).
// FmtH2 Z tiles: two 16-deep image K-steps per ring stage (32-deep stages,
// half the barriers, as the distance Gram; scores -2.6 % vs one,
// profiles/r5a_z_ks2_rank_ab.log)
template <class F>
constexpr int z_ks() { return F::P == 2 ? 2 : 1; }

template <class F = FmtX3>
__global__ __launch_bounds__(512, 1) void logreg_z_x3p_kernel(
    const typename F::E* __restrict__ Wx, int64_t n_img, const typename F::E* __restrict__ Xdx,
    int64_t N_img, int nk, const float* __restrict__ tp, int64_t N_pad, float* __restrict__ G,
    int Tm2, int Tn2, int64_t total, const float* __restrict__ xinv,
    const float* __restrict__ rinv) {
  using ZX3PTile = NTX3Tile<2, 4, 4, 2, 2, F::P == 3, F, z_ks<F>()>;  // nk: ring stages per tile
  const float zs = F::P == 3 ? 1.f : *xinv;
  __shared__ __attribute__((aligned(16))) char smem[ZX3PTile::kSmemBytes];
  const int w = threadIdx.x >> 6, wr = w / ZX3PTile::WN_, wc = w % ZX3PTile::WN_;
  const int64_t x = blockIdx.x % kXcds, u = blockIdx.x / kXcds, U = gridDim.x / kXcds;
  const int64_t q = total / kXcds, rr = total % kXcds;
  const int64_t lo = x * q + min(x, rr);
  const int64_t hi = (int64_t)__builtin_amdgcn_readfirstlane((int)(lo + q + (x < rr ? 1 : 0)));
  auto next_valid = [&](int64_t L, int& BI, int& BJ) -> int64_t {
    for (; L < hi; L += U)
      if (tile_at(L, Tm2, Tn2, false, BI, BJ)) {
        BI = __builtin_amdgcn_readfirstlane(BI);
        BJ = __builtin_amdgcn_readfirstlane(BJ);
        return L;
      }
    return L;
  };
  ZX3PTile tile;
  auto issue = [&](char* stg, int BI, int BJ, int ks) {
    const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(Wx + (int64_t)BI * 256 * 16), (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(Xdx + (int64_t)BJ * 256 * 16), (short)0, 0x7fffffff, 0x00020000);
    tile.dma(stg, rA, n_img, rB, N_img, ks);
  };
  int BI = 0, BJ = 0;
  int64_t L = next_valid((int64_t)__builtin_amdgcn_readfirstlane((int)(lo + u)), BI, BJ);
  tile.zero();
  if (L < hi) issue(smem, BI, BJ, 0);
  ZX3PTile::template ring_barrier<0>();
  int ks = 0, stage = 0, BIn = BI, BJn = BJ;
  int64_t Ln = L;
  while (L < hi) {
    int ksn = ks + 1;
    if (ksn == nk) {
      Ln = next_valid(L + U, BIn, BJn);
      ksn = 0;
    }
    if (Ln < hi) issue(smem + (stage ^ 1) * ZX3PTile::kStage, BIn, BJn, ksn);
    tile.compute(smem + stage * ZX3PTile::kStage, wr, wc);
    ZX3PTile::template ring_barrier<0>();
    if (ks + 1 == nk) {
      z_epilogue(tile, (int64_t)BI * 256, (int64_t)BJ * 256, tp, N_pad, G, zs,
                 F::P == 3 ? nullptr : rinv);
      tile.zero();
      L = Ln;
      BI = BIn;
      BJ = BJn;
    }
    ks = ksn;
    stage ^= 1;
  }
}

// ---- the fused score (round 5): Z, sigma and G . Xd in one kernel ---------
// Per block 128 particles (4 waves x 32); per wave the 32 particles' W image
// fragments stay in registers (the B operand of Z^T = Xd W^T, 16 K-steps x
// 2 parts at p <= 255) and their 32 x 256 G . Xd accumulators in AGPRs.  The
// data go by in chunks of 32 rows, DMA'd to LDS one chunk ahead: the chunk's
// row image (Z^T's A operand, shared by the 4 waves) and its 2 K-steps of
// Xd's column image.  Z^T's C layout puts particle r in lane r & 31 and the
// data rows 4h + 8g + e (g < 4, e < 4) in its registers: those 16 values,
// sigma'd and split, ARE the A fragments of G . Xd for two 16-deep K-steps
// when the column image stores each K-step's rows in the order
// kFusedPerm (position 8h + j <-> row 4h + 8 (j >> 2) + (j & 3)) -- no G
// in memory, no transpose.  G . Xd of chunk c - 1 runs beside Z of chunk c.
__host__ __device__ constexpr int fused_perm(int p) { return 4 * (p >> 3) + 8 * ((p & 7) >> 2) + (p & 3); }

// Yp[kstep][part][column][16 k]: ysplit_h2_kernel's image with position k of
// each 16-row K-step holding row fused_perm(k)
__global__ __launch_bounds__(256) void ysplit_h2_perm_kernel(const float* __restrict__ Y,
                                                             int64_t ldy, int64_t ksteps,
                                                             const float* __restrict__ colscale,
                                                             _Float16* __restrict__ Yh) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= ksteps * ldy) return;
  const int64_t kb = t / ldy, c = t % ldy;
  const float sc = colscale[c];
  f16x8 sp[2][2];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    _Float16 v[2];
    split_fmt<FmtH2>(sc * Y[(kb * 16 + fused_perm(k)) * ldy + c], v);
    sp[0][k >> 3][k & 7] = v[0];
    sp[1][k >> 3][k & 7] = v[1];
  }
  const int sw = (int)((c >> 3) & 1);
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    _Float16* dst = Yh + ((kb * 2 + p) * ldy + c) * 16;
    *reinterpret_cast<f16x8*>(dst + 8 * sw) = sp[p][0];
    *reinterpret_cast<f16x8*>(dst + 8 * (sw ^ 1)) = sp[p][1];
  }
}

constexpr int kFusedRows = 128;   // particles per block
constexpr int kFusedChunk = 32;   // data rows per chunk
constexpr int kFusedKD = 16;      // K-steps over the weights (p <= 255)
constexpr int kFusedCols = 256;   // G . Xd columns (ldb)
constexpr int kFusedXdx = kFusedKD * 2 * kFusedChunk * 32;   // a chunk's row image (32 KiB)
constexpr int kFusedXdp = 2 * 2 * kFusedCols * 32;           // its 2 K-steps of column image

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void logreg_fused_kernel(
    const _Float16* __restrict__ Wx, int64_t n_img, const _Float16* __restrict__ Xdx,
    int64_t N_img, const _Float16* __restrict__ Xdp, int nchunks,
    const float* __restrict__ xinv, const float* __restrict__ rinv,
    const float* __restrict__ colinv, float* __restrict__ GW, int64_t ldg, int64_t n,
    int cpb) {
  using V8 = FmtH2::V8;
  __shared__ __attribute__((aligned(16))) char smem[2 * kFusedXdx + 2 * kFusedXdp];
  char* const abuf = smem;                       // row image ring (chunk c in abuf[c & 1])
  char* const xbuf = smem + 2 * kFusedXdx;       // column image ring (chunk c in xbuf[c & 1])
  const int t = threadIdx.x, lane = t & 63, r = lane & 31, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int64_t p0 = (int64_t)blockIdx.x * kFusedRows + w * 32;
  const __amdgpu_buffer_rsrc_t rW =
      __builtin_amdgcn_make_buffer_rsrc((void*)Wx, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rX =
      __builtin_amdgcn_make_buffer_rsrc((void*)Xdx, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rP =
      __builtin_amdgcn_make_buffer_rsrc((void*)Xdp, (short)0, 0x7fffffff, 0x00020000);
  // the wave's W fragments: K-step k, part p -> lane (r, h): particle p0 + r
  V8 wf[kFusedKD][2];
#pragma unroll
  for (int k = 0; k < kFusedKD; ++k)
#pragma unroll
    for (int p = 0; p < 2; ++p)
      wf[k][p] = __builtin_bit_cast(
          V8, __builtin_amdgcn_raw_buffer_load_b128(
                  rW, (int)(((int64_t)(k * 2 + p) * n_img) * 32 + x3_off((int)(p0 + r), h)), 0, 0));
  const float zsc = kLog2e * (*xinv) * rinv[p0 + r];   // z = acc / (t_x s_i)
  // LDS-DMA of chunk c's row image (into abuf[c & 1]) and column image (xbuf[c & 1]):
  // 16-byte units u * 256 + t, wave-uniform LDS bases
  auto dma_rows = [&](int c) {
    char* dst = abuf + (c & 1) * kFusedXdx;
    const int soff = c * kFusedChunk * 32;
#pragma unroll
    for (int u = 0; u < kFusedXdx / 4096; ++u) {
      const int e = u * 256 + t, kp = e >> 6, within = e & 63;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rX, (__attribute__((address_space(3))) void*)(dst + (u * 256 + w * 64) * 16), 16,
          (int)((int64_t)kp * N_img * 32 + within * 16), soff, 0, 0);
    }
  };
  auto dma_cols = [&](int c) {
    char* dst = xbuf + (c & 1) * kFusedXdp;
    const int soff = c * kFusedXdp;
#pragma unroll
    for (int u = 0; u < kFusedXdp / 4096; ++u) {
      const int e = u * 256 + t;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rP, (__attribute__((address_space(3))) void*)(dst + (u * 256 + w * 64) * 16), 16,
          e * 16, soff, 0, 0);
    }
  };
  auto barrier_dma = []() {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  };
  f32x16 acc[kFusedCols / 32];
#pragma unroll
  for (int ni = 0; ni < kFusedCols / 32; ++ni)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[ni][q] = 0.f;
  V8 g[2][2];   // G of the previous chunk: K-step kk (data rows 16 kk ..), part
  // G . Xd of the chunk whose G is in g, column image in xb
  auto gxd = [&](const char* xb) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int ni = 0; ni < kFusedCols / 32; ++ni) {
        const V8 bh = *reinterpret_cast<const V8*>(xb + (kk * 2 + 0) * kFusedCols * 32 + x3_off(ni * 32 + r, h));
        const V8 bl = *reinterpret_cast<const V8*>(xb + (kk * 2 + 1) * kFusedCols * 32 + x3_off(ni * 32 + r, h));
        acc[ni] = mfma_fmt<FmtH2>(g[kk][1], bh, acc[ni]);   // small terms first
        acc[ni] = mfma_fmt<FmtH2>(g[kk][0], bl, acc[ni]);
        acc[ni] = mfma_fmt<FmtH2>(g[kk][0], bh, acc[ni]);
      }
  };
  // chunk c: the next chunk's rows and this chunk's columns DMA'd, Z^T of
  // chunk c (two chains), G . Xd of chunk c - 1 beside it, then sigma(-z)
  // into the A fragments of chunk c's two K-steps (2^15 G, split).  The
  // first and last chunks are peeled so that the steady body is one basic
  // block (the scheduler interleaves the two GEMMs only inside one)
  auto chunk = [&](int c, auto NEXT_, auto PREV_) {
    constexpr bool PREV = decltype(PREV_)::value;
    if constexpr (decltype(NEXT_)::value) dma_rows(c + 1);
    dma_cols(c);
    const char* ab = abuf + (c & 1) * kFusedXdx;
    const char* xp = xbuf + ((c - 1) & 1) * kFusedXdp;
    // step s: Z^T's K-step s (A: the chunk's row image) and, beside it, G .
    // Xd's (K-step s >> 3, column block s & 7) of chunk c - 1; the LDS
    // fragments of step s + 1 are read while step s's MFMAs run
    V8 fa[2][2], fb[2][2];
    auto rd = [&](int st, int bi) {
      fa[bi][0] = *reinterpret_cast<const V8*>(ab + (st * 2 + 0) * kFusedChunk * 32 + x3_off(r, h));
      fa[bi][1] = *reinterpret_cast<const V8*>(ab + (st * 2 + 1) * kFusedChunk * 32 + x3_off(r, h));
      if constexpr (PREV) {
        const int kk = st >> 3, ni = st & 7;
        fb[bi][0] = *reinterpret_cast<const V8*>(xp + (kk * 2 + 0) * kFusedCols * 32 + x3_off(ni * 32 + r, h));
        fb[bi][1] = *reinterpret_cast<const V8*>(xp + (kk * 2 + 1) * kFusedCols * 32 + x3_off(ni * 32 + r, h));
      }
    };
    f32x16 z0 = {}, z1 = {};
    rd(0, 0);
#pragma unroll
    for (int st = 0; st < kFusedKD; ++st) {
      if (st + 1 < kFusedKD) rd(st + 1, (st + 1) & 1);
      const V8 ah = fa[st & 1][0], al = fa[st & 1][1];
      f32x16& z = (st & 1) ? z1 : z0;
      z = mfma_fmt<FmtH2>(al, wf[st][0], z);
      z = mfma_fmt<FmtH2>(ah, wf[st][1], z);
      z = mfma_fmt<FmtH2>(ah, wf[st][0], z);
      if constexpr (PREV) {
        const int kk = st >> 3, ni = st & 7;
        const V8 bh = fb[st & 1][0], bl = fb[st & 1][1];
        acc[ni] = mfma_fmt<FmtH2>(g[kk][1], bh, acc[ni]);   // small terms first
        acc[ni] = mfma_fmt<FmtH2>(g[kk][0], bl, acc[ni]);
        acc[ni] = mfma_fmt<FmtH2>(g[kk][0], bh, acc[ni]);
      }
    }
    // order: the first step's reads, then per step the next step's reads
    // ahead of this step's MFMAs (each read has a step of MFMAs to land)
    __builtin_amdgcn_sched_group_barrier(0x100, PREV ? 4 : 2, 0);
#pragma unroll
    for (int st = 0; st < kFusedKD; ++st) {
      if (st + 1 < kFusedKD) __builtin_amdgcn_sched_group_barrier(0x100, PREV ? 4 : 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, PREV ? 6 : 3, 0);
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const float zz = (z0[q] + z1[q]) * zsc;
      const float gv = __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(zz)) * FmtH2::kAScale;
      const _Float16 hi = (_Float16)gv;
      g[q >> 3][0][q & 7] = hi;
      g[q >> 3][1][q & 7] = (_Float16)(gv - (float)hi);
    }
    barrier_dma();
  };
  constexpr std::true_type yes{};
  constexpr std::false_type no{};
  // data slice blockIdx.y: chunks [c0, c0 + cpb) (>= 2, checked by the host)
  const int c0 = (int)blockIdx.y * cpb, c1 = min(nchunks, c0 + cpb);
  GW += (int64_t)blockIdx.y * n * ldg;
  dma_rows(c0);
  barrier_dma();
  chunk(c0, yes, no);
  for (int c = c0 + 1; c + 1 < c1; ++c) chunk(c, yes, yes);
  chunk(c1 - 1, no, yes);
  gxd(xbuf + ((c1 - 1) & 1) * kFusedXdp);
  // GW[i][c] = acc 2^-15 / s_c
#pragma unroll
  for (int ni = 0; ni < kFusedCols / 32; ++ni) {
    const int col = ni * 32 + r;
    const float cs = colinv[col] * (1.f / FmtH2::kAScale);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int64_t i = p0 + c_row(q, lane);
      if (i < n) GW[i * ldg + col] = acc[ni][q] * cs;
    }
  }
}

// One (particle tile, data tile) per block.
__global__ __launch_bounds__(256) void logreg_z_kernel(const float* __restrict__ W,
                                                       const float* __restrict__ Xd, int64_t ldb,
                                                       int pp, const float* __restrict__ tp,
                                                       int64_t N, int64_t N_pad,
                                                       float* __restrict__ G) {
  __shared__ __attribute__((aligned(16))) float smem[ZTile::kSmemFloats];
  const int64_t i0 = (int64_t)blockIdx.y * ZTile::BM, q0 = (int64_t)blockIdx.x * ZTile::BN;
  ZTile tile;
  tile.run(W + i0 * ldb, ldb, Xd + q0 * ldb, ldb, pp, smem);
  z_epilogue(tile, i0, q0, tp, N_pad, G);
}

// one wave per particle row
__global__ __launch_bounds__(256) void logreg_finish_kernel(const float* __restrict__ X,
                                                            int64_t ldx, int64_t n, int64_t p,
                                                            const float* __restrict__ GW,
                                                            int64_t ldg, float scale,
                                                            float* __restrict__ S, int64_t lds,
                                                            int splits = 1, float pw = 1.f) {
  const int lane = threadIdx.x & 63;
  const int64_t j = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j >= n) return;
  const float* x = X + j * ldx;
  if (p <= 256) {
    // every load of the row issued before the norm's reduction (a lane's
    // columns lane + 64 u in registers); the same sums in the same order
    float xv[4], gv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t c = lane + 64 * u;
      xv[u] = c < p ? x[1 + c] : 0.f;
      gv[u] = c < p ? GW[j * ldg + c] : 0.f;
    }
    const float a = expf(x[0]);
    for (int z = 1; z < splits; ++z)  // slice order
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (lane + 64 * u < p) gv[u] += GW[(int64_t)z * n * ldg + j * ldg + lane + 64 * u];
    float w2 = 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (lane + 64 * u < p) w2 = fmaf(xv[u], xv[u], w2);
    w2 = warp_sum(w2);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (lane + 64 * u < p) S[j * lds + 1 + lane + 64 * u] = scale * (gv[u] - (pw * a) * xv[u]);
    if (lane == 0) S[j * lds] = scale * (pw * (-a + 0.5f * (float)p - 0.5f * a * w2));
    return;
  }
  const float a = expf(x[0]);
  float w2 = 0.f;
  for (int64_t c = lane; c < p; c += 64) w2 = fmaf(x[1 + c], x[1 + c], w2);
  w2 = warp_sum(w2);
  for (int64_t c = lane; c < p; c += 64) {
    float g = GW[j * ldg + c];
    for (int z = 1; z < splits; ++z) g += GW[(int64_t)z * n * ldg + j * ldg + c];  // slice order
    S[j * lds + 1 + c] = scale * (g - (pw * a) * x[1 + c]);  // pw = 1: the same fma as before
  }
  if (lane == 0) S[j * lds] = scale * (pw * (-a + 0.5f * (float)p - 0.5f * a * w2));
}


// ---- posterior-predictive test accuracy (experiments/logreg_plots.py:42-50) --
using PTile = ZTile;
// prob[q] = (1/n) sum_j sigma(xt_q . w_j) over the particles' weights w_j =
// x_j[1:] (no bias, alpha unused, as the reference's _test_acc); the caller
// thresholds prob > 0.5 against t_q > 0.  Z tiles on the NT engine; each
// block reduces its 128 particle rows per test column into part[block row]
// and predict_finish sums those partials in row-block order (deterministic).
__global__ __launch_bounds__(256) void logreg_predict_kernel(const float* __restrict__ W,
                                                             const float* __restrict__ Xt,
                                                             int64_t ldb, int pp, int64_t n,
                                                             int64_t Nt_pad,
                                                             float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float smem[PTile::kSmemFloats];
  __shared__ float scol[2][128];
  const int64_t i0 = (int64_t)blockIdx.y * PTile::BM, q0 = (int64_t)blockIdx.x * PTile::BN;
  PTile tile;
  tile.run(W + i0 * ldb, ldb, Xt + q0 * ldb, ldb, pp, smem);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w >> 1, wn = w & 1;
#pragma unroll
  for (int ni = 0; ni < 2; ++ni) {
    float s = 0.f;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t i = i0 + wm * 64 + mi * 32 + c_row(r, lane);
        if (i < n) s += sigmoidf_stable(tile.acc[mi][ni][r]);
      }
    s += __shfl_xor(s, 32, 64);  // lanes l, l^32: the same column, the other 4-row half
    if (lane < 32) scol[wm][wn * 64 + ni * 32 + lane] = s;
  }
  __syncthreads();
  for (int t = threadIdx.x; t < 128; t += 256)
    part[(int64_t)blockIdx.y * Nt_pad + q0 + t] = scol[0][t] + scol[1][t];
}

__global__ __launch_bounds__(256) void predict_finish_kernel(const float* __restrict__ part,
                                                             int64_t nblk, int64_t Nt,
                                                             int64_t Nt_pad, float inv_n,
                                                             float* __restrict__ prob) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= Nt) return;
  float s = 0.f;
  for (int64_t b = 0; b < nblk; ++b) s += part[b * Nt_pad + q];
  prob[q] = s * inv_n;
}

struct PredictWs {
  int64_t n_pad, Nt_pad, pp;
  size_t off_w, off_xt, off_part, total;
};

static PredictWs predict_ws(int64_t n, int64_t Nt, int64_t p) {
  PredictWs w;
  w.n_pad = roundup(n, 128);
  w.Nt_pad = roundup(Nt, 128);
  w.pp = roundup(p < 1 ? 1 : p, 32);
  size_t o = 0;
  auto take = [&](size_t floats) {
    size_t at = o;
    o += roundup((int64_t)(floats * sizeof(float)), 256);
    return at;
  };
  w.off_w = take((size_t)w.n_pad * w.pp);
  w.off_xt = take((size_t)w.Nt_pad * w.pp);
  w.off_part = take((size_t)(w.n_pad / 128) * w.Nt_pad);
  w.total = o;
  return w;
}


// Few particles (the reference's Gauss-Seidel order refreshes ONE particle's
// score after each update): one block per particle, no workspace, one
// launch.  p <= 32 (the reference's benchmark datasets): a thread per data
// row computes g_q = t_q sigma(-t_q xd_q.w) and accumulates g_q xd_q into p
// register partials, reduced over the block in a fixed order.  Larger p: g in
// LDS (a wave per data row), then the columns.  s_0 = -a + p/2 - a/2 |w|^2.
constexpr int kSmallMaxN = 8192;   // g in LDS (32 KiB) on the large-p form
constexpr int64_t kSmallMaxRows = 32;
constexpr int kSmallRegP = 32;

__global__ __launch_bounds__(256) void logreg_small_kernel(const float* __restrict__ X, int64_t ldx,
                                                           int64_t p, const float* __restrict__ Xd,
                                                           int64_t ldxd,
                                                           const float* __restrict__ t,
                                                           int64_t N, float scale,
                                                           float* __restrict__ S, int64_t lds) {
  __shared__ float g[kSmallMaxN];
  __shared__ float red[4][kSmallRegP + 1];
  const int64_t j = blockIdx.x;
  const float* x = X + j * ldx;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const float a = expf(x[0]);
  float w2 = 0.f;
  for (int64_t c = threadIdx.x; c < p; c += 256) w2 = fmaf(x[1 + c], x[1 + c], w2);
  if (p <= kSmallRegP) {
    float part[kSmallRegP];
#pragma unroll
    for (int c = 0; c < kSmallRegP; ++c) part[c] = 0.f;
    for (int64_t q = threadIdx.x; q < N; q += 256) {
      const float* xq = Xd + q * ldxd;
      float z = 0.f;
#pragma unroll
      for (int c = 0; c < kSmallRegP; ++c)
        if (c < p) z = fmaf(xq[c], x[1 + c], z);
      const float tq = t[q];
      const float gq = tq / (1.f + expf(tq * z));   // t sigma(-t z)
#pragma unroll
      for (int c = 0; c < kSmallRegP; ++c)
        if (c < p) part[c] = fmaf(gq, xq[c], part[c]);
    }
#pragma unroll
    for (int c = 0; c < kSmallRegP; ++c) {
      if (c >= p) break;
      const float v = warp_sum(part[c]);
      if (lane == 0) red[wv][c] = v;
    }
    w2 = warp_sum(w2);
    if (lane == 0) red[wv][kSmallRegP] = w2;
    __syncthreads();
    for (int64_t c = threadIdx.x; c < p; c += 256)
      S[j * lds + 1 + c] =
          scale * (((red[0][c] + red[1][c]) + (red[2][c] + red[3][c])) - a * x[1 + c]);
  } else {
    for (int64_t q = wv; q < N; q += 4) {
      const float* xq = Xd + q * ldxd;
      float z = 0.f;
      for (int64_t c = lane; c < p; c += 64) z = fmaf(xq[c], x[1 + c], z);
      z = warp_sum(z);
      if (lane == 0) {
        const float tq = t[q];
        g[q] = tq / (1.f + expf(tq * z));
      }
    }
    w2 = warp_sum(w2);
    if (lane == 0) red[wv][kSmallRegP] = w2;
    __syncthreads();
    for (int64_t c = threadIdx.x; c < p; c += 256) {
      float acc = 0.f;
      for (int64_t q = 0; q < N; ++q) acc = fmaf(g[q], Xd[q * ldxd + c], acc);
      S[j * lds + 1 + c] = scale * (acc - a * x[1 + c]);
    }
  }
  if (threadIdx.x == 0) {
    const float ww = (red[0][kSmallRegP] + red[1][kSmallRegP]) +
                     (red[2][kSmallRegP] + red[3][kSmallRegP]);
    S[j * lds] = scale * (-a + 0.5f * (float)p - 0.5f * a * ww);
  }
}

}  // namespace dsvgd

using namespace dsvgd;

extern "C" {

int dsvgd_logreg_set_fused(int on) {
  const int prev = g_logreg_fused;
  g_logreg_fused = on ? 1 : 0;
  return prev;
}

size_t dsvgd_logreg_workspace_bytes(int64_t n, int64_t N, int64_t p) {
  return logreg_ws(n, N, p).total;
}

// engine: 0 = FmtH2 split engine (default), 1 = FmtX3, 2 = f32 MFMA (reference)
// The data-only half of the workspace (padded Xd / t, Xd's scales and images)
// depends on (Xd, t) alone: logreg_prepare fills it once per data set and
// logreg_step reuses it every step (the particles change, the data do not).
struct LogregPlan {
  LogregWs w;
  bool x3, h2;
  char* base;
};

static LogregPlan logreg_plan(int64_t n, int64_t N, int64_t p, void* workspace, int engine) {
  LogregPlan P;
  P.w = logreg_ws(n, N, p);
  const LogregWs& w = P.w;
  const bool fits =
      w.n_pad * w.pp * 6 < ((int64_t)1 << 31) && w.N_pad * w.ldb * 6 < ((int64_t)1 << 31);
  P.x3 = engine == 1 && fits;
  P.h2 = engine == 0 && fits;
  P.base = (char*)workspace;
  return P;
}

static bool logreg_small(int64_t n, int64_t N, int64_t p) {
  return n <= kSmallMaxRows && (p <= kSmallRegP || N <= kSmallMaxN);
}

static int logreg_prepare(const float* Xd, int64_t ldxd, const float* t, int64_t N, int64_t p,
                          const LogregPlan& P, hipStream_t s) {
  const LogregWs& w = P.w;
  float* Xdp = (float*)(P.base + w.off_xd);
  float* tp = (float*)(P.base + w.off_t);
  const int64_t tot = w.N_pad * w.ldb;
  hipLaunchKernelGGL(pad_copy_kernel, dim3((tot + 255) / 256), dim3(256), 0, s, Xd, ldxd, 0, N, p,
                     w.N_pad, Xdp, w.ldb);
  int rc = check_launch("pad_copy(Xd)");
  if (rc) return rc;
  hipLaunchKernelGGL(pad_copy_kernel, dim3((w.N_pad + 255) / 256), dim3(256), 0, s, t, 1, 0, N, 1,
                     w.N_pad, tp, 1);
  if ((rc = check_launch("pad_copy(t)"))) return rc;
  // t folded into the data: t_q sigma(-t_q z_q) xd_q = sigma(-z'_q) xd'_q with
  // xd' = t xd, z' = w . xd' -- so G = sigma(-z') lies in (0, 1) whatever the
  // labels (the FmtH2 A image of G holds 2^15 G: |t| > 2 would overflow fp16)
  hipLaunchKernelGGL(fold_labels_kernel, dim3((tot + 255) / 256), dim3(256), 0, s, Xdp, tp, w.N_pad,
                     w.ldb);
  if ((rc = check_launch("fold_labels"))) return rc;
  hipLaunchKernelGGL(set_ones_kernel, dim3((w.N_pad + 255) / 256), dim3(256), 0, s, tp, w.N_pad);
  if ((rc = check_launch("set_ones(t)"))) return rc;
  if (P.h2) {
    float* sxd = (float*)(P.base + w.off_sxd);
    float* sws = (float*)(P.base + w.off_sws);
    if ((rc = h2_colscale(Xdp, w.ldb, w.N_pad, w.ldb, 0, sws, sxd, s))) return rc;
    // the tensor scale for Z's Xd image, per-column ones for G . Xd's B image
    if ((rc = h2_rowsplit(Xdp, w.ldb, w.N_pad, w.pp, w.N_pad, w.pp, sxd + 2 * w.ldb,
                          P.base + w.off_xdx, s)))
      return rc;
    if ((rc = h2_ysplit(Xdp, w.ldb, w.N_pad, sxd, (_Float16*)(P.base + w.off_xdy), s))) return rc;
    // the fused score's column image: the same split, K order permuted
    const int64_t th = (w.N_pad / 16) * w.ldb;
    hipLaunchKernelGGL(ysplit_h2_perm_kernel, dim3((unsigned)((th + 255) / 256)), dim3(256), 0, s, Xdp,
                       w.ldb, w.N_pad / 16, sxd, (_Float16*)(P.base + w.off_xdp));
    return check_launch("ysplit_h2_perm");
  }
  if (P.x3) {
    // the persistent 16x16x32 Z form reads unswizzled images
    if ((rc = dsvgd_rowsplit(Xdp, w.ldb, w.N_pad, w.pp, w.N_pad, w.pp, P.base + w.off_xdx, 0, s)))
      return rc;
    const int m16 = w.ldb % 256 == 0;  // the 16x16x32 form (unswizzled image) when it applies
    return dsvgd_ysplit(Xdp, w.ldb, w.N_pad, P.base + w.off_xdy, m16 ? 0 : 1, nullptr, s);
  }
  return DSVGD_OK;
}

// pw: the prior's weight (1 = the reference's logp; DistSampler's gathered-data
// all_scores passes S, the prior the reference's all-reduce sums S times)
static int logreg_step(const float* X, int64_t ldx, int64_t n, int64_t p, float scale, float* S,
                       int64_t lds, const LogregPlan& P, hipStream_t s, float pw = 1.f) {
  const LogregWs& w = P.w;
  char* base = P.base;
  float* Xdp = (float*)(base + w.off_xd);
  float* tp = (float*)(base + w.off_t);
  float* G = (float*)(base + w.off_g);
  float* GW = (float*)(base + w.off_gw);
  int rc = 0, splits = 1;
  if (P.h2) {
    void* Wx = base + w.off_wx;
    _Float16* Xdy = (_Float16*)(base + w.off_xdy);
    float* rsw = (float*)(base + w.off_rsw);
    float* riw = (float*)(base + w.off_riw);
    float* sxd = (float*)(base + w.off_sxd);
    // W = X[:, 1:] in place, one power-of-two scale per particle row: scale
    // and image in one pass (rowimage_h2_kernel)
    if ((rc = h2_rowimage(X + 1, ldx, n, p, w.n_pad, w.pp, rsw, riw, Wx, s))) return rc;
    if (g_logreg_fused && w.pp == kFusedKD * 16 && w.ldb == kFusedCols &&
        w.N_pad % kFusedChunk == 0 && w.N_pad >= 2 * kFusedChunk && w.n_pad % kFusedRows == 0) {
      const int z = fused_splits(w.n_pad, w.N_pad);
      const int nchunks = (int)(w.N_pad / kFusedChunk);
      // every slice takes nchunks / z >= 2 whole chunks (none dropped)
      DSVGD_REQUIRE(nchunks % z == 0 && nchunks / z >= 2, "fused score: unequal data slices");
      hipLaunchKernelGGL(logreg_fused_kernel, dim3((unsigned)(w.n_pad / kFusedRows), (unsigned)z),
                         dim3(256), 0, s, (const _Float16*)Wx, w.n_pad,
                         (const _Float16*)(base + w.off_xdx), w.N_pad,
                         (const _Float16*)(base + w.off_xdp), nchunks,
                         (const float*)(sxd + 2 * w.ldb + 1), (const float*)riw,
                         (const float*)(sxd + w.ldb), GW, w.ldb, n, nchunks / z);
      if ((rc = check_launch("logreg_fused"))) return rc;
      hipLaunchKernelGGL(logreg_finish_kernel, dim3((n + 3) / 4), dim3(256), 0, s, X, ldx, n, p, GW,
                         w.ldb, scale, S, lds, z, pw);
      return check_launch("logreg_finish");
    }
    int blocks = 0;
    if ((rc = persistent_blocks(reinterpret_cast<const void*>(&logreg_z_x3p_kernel<FmtH2>),
                                &blocks, 512)))
      return rc;
    const int Tm2 = (int)(w.n_pad / 256), Tn2 = (int)(w.N_pad / 256);
    hipLaunchKernelGGL(logreg_z_x3p_kernel<FmtH2>, dim3((unsigned)blocks), dim3(512), 0, s,
                       (const _Float16*)Wx, w.n_pad, (const _Float16*)(base + w.off_xdx), w.N_pad,
                       (int)(w.pp / kX3Step / z_ks<FmtH2>()), tp, w.N_pad, G, Tm2, Tn2,
                       tile_grid(Tm2, Tn2, false), (const float*)(sxd + 2 * w.ldb + 1),
                       (const float*)riw);
    if ((rc = check_launch("logreg_z_h2"))) return rc;
    splits = gxd_splits(w.n_pad, w.N_pad);
    if ((rc = nn_h2_gemm(false, G, w.N_pad, Xdy, w.ldb, splits, nullptr, GW, w.ldb, nullptr, n, 0, s,
                         0, sxd + w.ldb, nullptr)))
      return rc;
  } else if (P.x3) {
    void* Wx = base + w.off_wx;
    if ((rc = dsvgd_rowsplit(X + 1, ldx, n, p, w.n_pad, w.pp, Wx, 0, s))) return rc;
    int blocks = 0;
    if ((rc = persistent_blocks(reinterpret_cast<const void*>(&logreg_z_x3p_kernel<FmtX3>),
                                &blocks, 512)))
      return rc;
    const int Tm2 = (int)(w.n_pad / 256), Tn2 = (int)(w.N_pad / 256);
    hipLaunchKernelGGL(logreg_z_x3p_kernel<FmtX3>, dim3((unsigned)blocks), dim3(512), 0, s,
                       (const __bf16*)Wx, w.n_pad, (const __bf16*)(base + w.off_xdx), w.N_pad,
                       (int)(w.pp / kX3Step), tp, w.N_pad, G, Tm2, Tn2,
                       tile_grid(Tm2, Tn2, false), nullptr, nullptr);
    if ((rc = check_launch("logreg_z_x3"))) return rc;
    const int m16 = w.ldb % 256 == 0;
    if ((rc = nn_x3_gemm(false, G, w.N_pad, (const __bf16*)(base + w.off_xdy), w.ldb, 1, nullptr,
                         GW, w.ldb, nullptr, n, 0, s, 0, m16, nullptr)))
      return rc;
  } else {
    float* Wp = (float*)(base + w.off_w);
    hipLaunchKernelGGL(pad_copy_kernel, dim3((w.n_pad * w.ldb + 255) / 256), dim3(256), 0, s, X,
                       ldx, 1, n, p, w.n_pad, Wp, w.ldb);
    if ((rc = check_launch("pad_copy(W)"))) return rc;
    hipLaunchKernelGGL(logreg_z_kernel, dim3(w.N_pad / ZTile::BN, w.n_pad / ZTile::BM), dim3(256),
                       0, s, Wp, Xdp, w.ldb, (int)w.pp, tp, w.N, w.N_pad, G);
    if ((rc = check_launch("logreg_z"))) return rc;
    if ((rc = nn_gemm(false, G, w.N_pad, Xdp, w.ldb, w.ldb, 1, nullptr, GW, w.ldb, nullptr, n, 0,
                      s, nullptr)))
      return rc;
  }
  hipLaunchKernelGGL(logreg_finish_kernel, dim3((n + 3) / 4), dim3(256), 0, s, X, ldx, n, p, GW,
                     w.ldb, scale, S, lds, splits, pw);
  return check_launch("logreg_finish");
}

static int score_logreg(const float* X, int64_t ldx, int64_t n, int64_t d, const float* Xd,
                        int64_t ldxd, const float* t, int64_t N, float scale, float* S, int64_t lds,
                        void* workspace, void* stream, int engine) {
  DSVGD_REQUIRE(X && Xd && t && S && workspace, "null pointer");
  DSVGD_REQUIRE(n > 0 && d >= 2 && N > 0 && ldx >= d && lds >= d && ldxd >= d - 1, "sizes");
  DSVGD_REQUIRE(((uintptr_t)workspace & 255) == 0, "workspace must be 256-byte aligned");
  const int64_t p = d - 1;
  if (logreg_small(n, N, p)) {  // latency path
    hipLaunchKernelGGL(logreg_small_kernel, dim3((unsigned)n), dim3(256), 0, (hipStream_t)stream,
                       X, ldx, p, Xd, ldxd, t, N, scale, S, lds);
    return check_launch("logreg_small");
  }
  DSVGD_REQUIRE(roundup(n, 128) / 128 <= 65535, "too many row tiles");
  const LogregPlan P = logreg_plan(n, N, p, workspace, engine);
  int rc = logreg_prepare(Xd, ldxd, t, N, p, P, (hipStream_t)stream);
  if (rc) return rc;
  return logreg_step(X, ldx, n, p, scale, S, lds, P, (hipStream_t)stream);
}

int dsvgd_score_logreg(const float* X, int64_t ldx, int64_t n, int64_t d, const float* Xd,
                       int64_t ldxd, const float* t, int64_t N, float scale, float* S, int64_t lds,
                       void* workspace, void* stream) {
  return score_logreg(X, ldx, n, d, Xd, ldxd, t, N, scale, S, lds, workspace, stream, 0);
}

int dsvgd_score_logreg_engine(const float* X, int64_t ldx, int64_t n, int64_t d, const float* Xd,
                              int64_t ldxd, const float* t, int64_t N, float scale, float* S,
                              int64_t lds, void* workspace, int engine, void* stream) {
  DSVGD_REQUIRE(engine >= 0 && engine <= 2, "engine must be 0 (h2), 1 (x3) or 2 (f32)");
  return score_logreg(X, ldx, n, d, Xd, ldxd, t, N, scale, S, lds, workspace, stream, engine);
}

int dsvgd_logreg_prepare(const float* Xd, int64_t ldxd, const float* t, int64_t N, int64_t n,
                         int64_t d, void* workspace, int engine, void* stream) {
  DSVGD_REQUIRE(Xd && t && workspace, "null pointer");
  DSVGD_REQUIRE(n > 0 && d >= 2 && N > 0 && ldxd >= d - 1, "sizes");
  DSVGD_REQUIRE(((uintptr_t)workspace & 255) == 0, "workspace must be 256-byte aligned");
  DSVGD_REQUIRE(engine >= 0 && engine <= 2, "engine must be 0 (h2), 1 (x3) or 2 (f32)");
  DSVGD_REQUIRE(!logreg_small(n, N, d - 1),
                "n <= 32 takes the one-block path: call dsvgd_score_logreg_engine");
  DSVGD_REQUIRE(roundup(n, 128) / 128 <= 65535, "too many row tiles");
  return logreg_prepare(Xd, ldxd, t, N, d - 1, logreg_plan(n, N, d - 1, workspace, engine),
                        (hipStream_t)stream);
}

int dsvgd_score_logreg_prepared(const float* X, int64_t ldx, int64_t n, int64_t d, int64_t N,
                                float scale, float* S, int64_t lds, void* workspace, int engine,
                                void* stream) {
  DSVGD_REQUIRE(X && S && workspace, "null pointer");
  DSVGD_REQUIRE(n > 0 && d >= 2 && N > 0 && ldx >= d && lds >= d, "sizes");
  DSVGD_REQUIRE(((uintptr_t)workspace & 255) == 0, "workspace must be 256-byte aligned");
  DSVGD_REQUIRE(engine >= 0 && engine <= 2, "engine must be 0 (h2), 1 (x3) or 2 (f32)");
  DSVGD_REQUIRE(!logreg_small(n, N, d - 1),
                "n <= 32 takes the one-block path: call dsvgd_score_logreg_engine");
  return logreg_step(X, ldx, n, d - 1, scale, S, lds,
                     logreg_plan(n, N, d - 1, workspace, engine), (hipStream_t)stream);
}

int dsvgd_score_logreg_prior(const float* X, int64_t ldx, int64_t n, int64_t d, int64_t N,
                             float scale, float prior_weight, float* S, int64_t lds,
                             void* workspace, int engine, void* stream) {
  DSVGD_REQUIRE(X && S && workspace, "null pointer");
  DSVGD_REQUIRE(n > 0 && d >= 2 && N > 0 && ldx >= d && lds >= d, "sizes");
  DSVGD_REQUIRE(((uintptr_t)workspace & 255) == 0, "workspace must be 256-byte aligned");
  DSVGD_REQUIRE(engine >= 0 && engine <= 2, "engine must be 0 (h2), 1 (x3) or 2 (f32)");
  DSVGD_REQUIRE(!logreg_small(n, N, d - 1),
                "n <= 32 takes the one-block path: call dsvgd_score_logreg_engine");
  return logreg_step(X, ldx, n, d - 1, scale, S, lds,
                     logreg_plan(n, N, d - 1, workspace, engine), (hipStream_t)stream,
                     prior_weight);
}

size_t dsvgd_logreg_predict_workspace_bytes(int64_t n, int64_t Nt, int64_t p) {
  return predict_ws(n, Nt, p).total;
}

int dsvgd_logreg_predict(const float* X, int64_t ldx, int64_t n, int64_t d, const float* Xt,
                         int64_t ldxt, int64_t Nt, float* prob, void* workspace, void* stream) {
  DSVGD_REQUIRE(X && Xt && prob && workspace, "null pointer");
  DSVGD_REQUIRE(n > 0 && d >= 2 && Nt > 0 && ldx >= d && ldxt >= d - 1, "sizes");
  DSVGD_REQUIRE(((uintptr_t)workspace & 255) == 0, "workspace must be 256-byte aligned");
  const int64_t p = d - 1;
  const PredictWs w = predict_ws(n, Nt, p);
  DSVGD_REQUIRE(w.n_pad / 128 <= 65535, "too many particle tiles");
  char* base = (char*)workspace;
  float* Wp = (float*)(base + w.off_w);
  float* Xtp = (float*)(base + w.off_xt);
  float* part = (float*)(base + w.off_part);
  hipStream_t s = (hipStream_t)stream;
  int64_t tot = w.n_pad * w.pp;
  hipLaunchKernelGGL(pad_copy_kernel, dim3((tot + 255) / 256), dim3(256), 0, s, X, ldx, 1, n, p,
                     w.n_pad, Wp, w.pp);
  int rc = check_launch("pad_copy(W)");
  if (rc) return rc;
  tot = w.Nt_pad * w.pp;
  hipLaunchKernelGGL(pad_copy_kernel, dim3((tot + 255) / 256), dim3(256), 0, s, Xt, ldxt, 0, Nt, p,
                     w.Nt_pad, Xtp, w.pp);
  if ((rc = check_launch("pad_copy(Xt)"))) return rc;
  hipLaunchKernelGGL(logreg_predict_kernel, dim3(w.Nt_pad / 128, w.n_pad / 128), dim3(256), 0, s,
                     Wp, Xtp, w.pp, (int)w.pp, n, w.Nt_pad, part);
  if ((rc = check_launch("logreg_predict"))) return rc;
  hipLaunchKernelGGL(predict_finish_kernel, dim3((Nt + 255) / 256), dim3(256), 0, s, part,
                     w.n_pad / 128, Nt, w.Nt_pad, 1.f / (float)n, prob);
  return check_launch("predict_finish");
}

}  // extern "C"
