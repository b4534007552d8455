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
            int64_t m, int64_t row0, hipStream_t s);
int nn_x3_gemm(bool exp_, const float* A, int64_t K, const __bf16* Yx, int64_t ldy, int splits,
               const dsvgd_select_state* st, float* C, int64_t ldc, float* rowsum, int64_t m,
               int64_t row0, hipStream_t s, int sym, int m16, const float* gate);
int nn_h2_gemm(bool exp_, const float* A, int64_t K, const _Float16* Yh, int64_t ldy, int splits,
               const dsvgd_select_state* st, float* C, int64_t ldc, float* rowsum, int64_t m,
               int64_t row0, hipStream_t s, int sym, const float* colinv, const float* gate);
int h2_colscale(const float* A, int64_t lda, int64_t rows, int64_t cols, float* ws, float* out,
                hipStream_t s);
int h2_ysplit(const float* Y, int64_t ldy, int64_t rows, const float* colscale, void* Yh,
              hipStream_t s);
int h2_rowsplit(const float* A, int64_t lda, int64_t rows, int64_t cols, int64_t rows_pad,
                int64_t kpad, const float* tscale, void* img, hipStream_t s);
int h2_rowsplit_rows(const float* A, int64_t lda, int64_t rows, int64_t cols, int64_t rows_pad,
                     int64_t kpad, const float* rscale, void* img, hipStream_t s);
int h2_rowscale(const float* A, int64_t lda, int64_t rows, int64_t cols, int64_t rows_pad,
                float* rscale, float* rinv, hipStream_t s);
size_t h2_colscale_ws_floats(int64_t rows, int64_t cols);

static int64_t nn_cols(int64_t w) {
  if (w <= 128) return 128;
  if (w <= 256) return 256;
  return roundup(w, 512);
}

// the fused score tile (logreg_fused_kernel, below)
constexpr int kFzQ = 32;                     // data rows per chunk
constexpr int kFzHalf = 32 * 1024;           // A_Z or A_G of one chunk
constexpr int kFzChunkBytes = 2 * kFzHalf;   // chunk image: [A_Z | A_G]
// it serves p = 255 (pp = ldb = 256): the bench's and config D's shape
static bool fused_ok(int64_t pp, int64_t ldb) { return pp == 256 && ldb == 256; }

struct LogregWs {
  int64_t N, n_pad, N_pad, pp, ldb;
  size_t off_w, off_xd, off_t, off_g, off_gw, off_wx, off_xdx, off_xdy, off_rsw, off_riw, off_sxd,
      off_sws, off_xdt, off_fimg, off_sfz, total;
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
  w.off_gw = take((size_t)kGxdMaxSplits * w.n_pad * w.ldb);  // split-K slices of G . Xd
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
  // the fused tile (logreg_fused_kernel): t (.) Xd, its chunk images, scales
  w.off_xdt = take((size_t)w.N_pad * w.ldb);
  w.off_fimg = take((size_t)(w.N_pad / kFzQ) * kFzChunkBytes / 4);
  w.off_sfz = take((size_t)(2 * w.ldb + 3));
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

__device__ __forceinline__ float sigmoidf_stable(float u) {
  if (u >= 0.f) return 1.f / (1.f + expf(-u));
  const float e = expf(u);
  return e / (1.f + e);
}

// G[j][q] = t_q sigma(-t_q (w_j . xd_q)) = t_q / (1 + exp(t_q z)), zero for
// padded q (t_q = 0 there); panel layout.  The epilogue is VALU work beside
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

// ---- the fused score tile: Z -> sigma -> G.Xd without G in HBM -----------
// With xd'_q = t_q xd_q and z' = w . xd' = t z, the score's data term is
//   sum_q t_q sigma(-t_q z_q) xd_q = sum_q sigma(-z'_q) xd'_q,
// so one block of 128 particles streams the data in chunks of kFzQ = 32 rows:
//   Z-phase  zT[q][i] = Xd'_chunk . W^T          (K = p = 256, 48 MFMAs per wave)
//   G'[q][i] = 2^15 sigma(-z'[q][i]), split into two fp16 parts in registers
//   G-phase  accT[c][i] += Xd'^T_chunk . G'      (K = 32, 8 column blocks, 48 MFMAs)
// One wave per SIMD; wave w owns particles 32 w .. +31 of the block, its
// 32 x 256 W rows held as FmtH2 B fragments in 128 VGPRs for the whole
// launch, the G-phase accumulators (256 columns x its 32 particles) in 128
// AGPRs.  G' never leaves the registers: the Z-phase's C layout (lane: one
// particle, 16 data rows q = 8 (e >> 2) + 4 h + (e & 3)) IS the G-phase's B
// operand once the k order of the G-phase is permuted to match -- the chunk
// image's A_G part is written in that q order (logreg_fused_image_kernel).
// The data images stream through two 2-slot LDS-DMA rings (A_Z of chunk
// c + 1 beside A_G of chunk c: the Z-phase of the next chunk runs with the
// sigmoid of this one spread between its MFMAs, then this chunk's G-phase).
// Replaces logreg_z_x3p_kernel + the G.Xd launch at p = 255 (pp = ldb = 256):
// no 4 n N bytes of G written and read back.

// Xd'[q][c] = t_q Xd[q][c] (padded rows: t = 0)
__global__ __launch_bounds__(256) void scale_rows_kernel(const float* __restrict__ A,
                                                         const float* __restrict__ tq,
                                                         int64_t rows, int64_t ld,
                                                         float* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e < rows * ld) out[e] = tq[e / ld] * A[e];
}

// chunk image of Xd' (N_pad x 256, ld 256), 16-byte items:
//   A_Z[part][ks][q][16 k] = parts of tz Xd'[32 ch + q][16 ks + k]   (item: ks, q, half)
//   A_G[part][kg][c][16 k] = parts of s_c Xd'[32 ch + q(kg, k)][c],
//     q(kg, 8 h + j) = 16 kg + 8 (j >> 2) + 4 h + (j & 3)          (item: kg, c, half)
// halves swapped on rows / columns with bit 3 set (x3_off); sfz: h2_colscale
// layout of Xd' ([s_c | 1/s_c | tz | 1/tz]).
__global__ __launch_bounds__(256) void logreg_fused_image_kernel(const float* __restrict__ Xt,
                                                                 const float* __restrict__ sfz,
                                                                 int64_t nchunks,
                                                                 char* __restrict__ img) {
  const int64_t item = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (item >= nchunks * 2048) return;
  const int64_t ch = item / 2048;
  const int it = (int)(item % 2048);
  char* base = img + ch * kFzChunkBytes;
  float v[8];
  int off;
  if (it < 1024) {  // A_Z
    const int ks = it >> 6, q = (it >> 1) & 31, hh = it & 1;
    const float tz = sfz[2 * 256];
    const float* src = Xt + (ch * kFzQ + q) * 256 + 16 * ks + 8 * hh;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = tz * src[j];
    off = ks * 1024 + x3_off(q, hh);
  } else {  // A_G
    const int i2 = it - 1024;
    const int kg = i2 >> 9, c = (i2 >> 1) & 255, hh = i2 & 1;
    const float sc = sfz[c];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int q = 16 * kg + 8 * (j >> 2) + 4 * hh + (j & 3);
      v[j] = sc * Xt[(ch * kFzQ + q) * 256 + c];
    }
    base += kFzHalf;
    off = kg * 8192 + x3_off(c, hh);
  }
  FmtH2::V8 p0, p1;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const _Float16 a = (_Float16)v[j];
    p0[j] = a;
    p1[j] = (_Float16)(v[j] - (float)a);
  }
  // part 1 sits half an image (16 KiB) after part 0 in both halves
  *reinterpret_cast<FmtH2::V8*>(base + off) = p0;
  *reinterpret_cast<FmtH2::V8*>(base + kFzHalf / 2 + off) = p1;
}

// Wx: logreg's FmtH2 W row image ([ks][part][row][16 k], n_img rows, per-row
// scales: riw[i] = 1 / s_i); img: the chunk images; sfz: Xd''s scales.
// GW[i][c] (ld 256) = sum_q sigma(-z'_iq) Xd'[q][c] for i < n.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void logreg_fused_kernel(
    const _Float16* __restrict__ Wx, int64_t n_img, const float* __restrict__ riw,
    const char* __restrict__ img, int nchunks, const float* __restrict__ sfz, int64_t n,
    float* __restrict__ GW) {
  using V8 = FmtH2::V8;
  __shared__ __attribute__((aligned(16))) char smem[4 * kFzHalf];  // A_Z ring, A_G ring
  char* const zring = smem;
  char* const gring = smem + 2 * kFzHalf;
  const int t = threadIdx.x, lane = t & 63, r = lane & 31, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int64_t i = (int64_t)blockIdx.x * 128 + 32 * w + r;  // this lane's particle
  // the wave's W fragments (B operand of the Z-phase): [K-step][part]
  V8 wb[16][2];
  {
    const __amdgpu_buffer_rsrc_t rW =
        __builtin_amdgcn_make_buffer_rsrc((void*)Wx, (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int ks = 0; ks < 16; ++ks)
#pragma unroll
      for (int p = 0; p < 2; ++p)
        wb[ks][p] = __builtin_bit_cast(
            V8, __builtin_amdgcn_raw_buffer_load_b128(
                    rW, (int)(((int64_t)(2 * ks + p) * n_img) * 32 + x3_off((int)i, h)), 0, 0));
  }
  // z' = acc riw_i / tz; G' = 2^15 / (1 + exp(z'))
  const float zc = kLog2e * riw[i] * sfz[2 * 256 + 1];
  f32x16 acc[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) acc[c] = f32x16{};
  const __amdgpu_buffer_rsrc_t rI =
      __builtin_amdgcn_make_buffer_rsrc((void*)img, (short)0, 0x7fffffff, 0x00020000);
  // one half (A_Z or A_G) of chunk ch -> LDS: 8 x 1 KiB per wave
  auto dma = [&](int ch, int half, char* dst) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int off = (w * 8 + u) * 1024;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rI, (__attribute__((address_space(3))) void*)(dst + off), 16, off + lane * 16,
          ch * kFzChunkBytes + half * kFzHalf, 0, 0);
    }
  };
  // G' of one z value: its two fp16 parts
  auto sig = [&](float zv, V8 (&g)[2][2], int e) {
    const float ex = __builtin_amdgcn_exp2f(zv * zc);
    const float gv = FmtH2::kAScale * __builtin_amdgcn_rcpf(1.f + ex);
    const _Float16 g0 = (_Float16)gv;
    g[e >> 3][0][e & 7] = g0;
    g[e >> 3][1][e & 7] = (_Float16)(gv - (float)g0);
  };
  // Z-phase of the chunk whose A_Z sits at az (zT[q][i], K = 256) with the
  // previous chunk's z (zp) turned into G' between its MFMAs, one value per
  // K-step -- the G-phase's B fragments g[K-step][part] (lane's value e is
  // data row 8 (e >> 2) + 4 h + (e & 3): K-step e >> 3, element e & 7)
  auto zphase = [&](const char* az, f32x16& z, const f32x16& zp, V8 (&g)[2][2]) {
    z = f32x16{};
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      const V8 a0 = *reinterpret_cast<const V8*>(az + ks * 1024 + x3_off(r, h));
      const V8 a1 = *reinterpret_cast<const V8*>(az + kFzHalf / 2 + ks * 1024 + x3_off(r, h));
      z = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, wb[ks][0], z, 0, 0, 0);
      sig(zp[ks], g, ks);
      z = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, wb[ks][1], z, 0, 0, 0);
      z = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, wb[ks][0], z, 0, 0, 0);
    }
  };
  auto gphase = [&](const char* ag, const V8 (&g)[2][2]) {
#pragma unroll
    for (int kg = 0; kg < 2; ++kg)
#pragma unroll
      for (int cb = 0; cb < 8; ++cb) {
        const V8 a0 = *reinterpret_cast<const V8*>(ag + kg * 8192 + x3_off(32 * cb + r, h));
        const V8 a1 = *reinterpret_cast<const V8*>(ag + kFzHalf / 2 + kg * 8192 + x3_off(32 * cb + r, h));
        acc[cb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, g[kg][0], acc[cb], 0, 0, 0);
        acc[cb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, g[kg][1], acc[cb], 0, 0, 0);
        acc[cb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, g[kg][0], acc[cb], 0, 0, 0);
      }
  };

  // prologue: A_Z(0) -> z = z(0); A_Z(1), A_G(0) DMA'd
  f32x16 z, zp;
  V8 g[2][2];
  dma(0, 0, zring);
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  if (nchunks > 1) dma(1, 0, zring + kFzHalf);
  dma(0, 1, gring);
  zphase(zring, z, z, g);  // (its G' values are discarded)
  // chunk c: A_Z(c+1) in zring[(c+1)&1], A_G(c) in gring[c&1], z = z(c).
  // One barrier per chunk: after it every wave's DMAs of the last iteration
  // have landed AND every wave is past the last iteration's LDS reads, so
  // the slots those reads used are refilled (for chunk c + 2's A_Z and
  // chunk c + 1's A_G) right after it, a whole iteration ahead of their use
  for (int c = 0; c < nchunks; ++c) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (c + 2 < nchunks) dma(c + 2, 0, zring + (c & 1) * kFzHalf);
    if (c + 1 < nchunks) dma(c + 1, 1, gring + ((c + 1) & 1) * kFzHalf);
    zp = z;
    if (c + 1 < nchunks) {
      zphase(zring + ((c + 1) & 1) * kFzHalf, z, zp, g);
    } else {
#pragma unroll
      for (int e = 0; e < 16; ++e) sig(zp[e], g, e);
    }
    gphase(gring + (c & 1) * kFzHalf, g);
  }
  // GW[i][c] = acc * (1 / s_c) * 2^-15: lane's column i, rows c = 32 cb + 8 g + 4 h + e
  if (i < n) {
#pragma unroll
    for (int cb = 0; cb < 8; ++cb)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int c0 = 32 * cb + 8 * gq + 4 * h;
        const f32x4 ci = *reinterpret_cast<const f32x4*>(sfz + 256 + c0);
        f32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = acc[cb][4 * gq + e] * ci[e] * (1.f / FmtH2::kAScale);
        *reinterpret_cast<f32x4*>(GW + i * 256 + c0) = o;
      }
  }
}

// one wave per particle row
__global__ __launch_bounds__(256) void logreg_finish_kernel(const float* __restrict__ X,
                                                            int64_t ldx, int64_t n, int64_t p,
                                                            const float* __restrict__ GW,
                                                            int64_t ldg, float scale,
                                                            float* __restrict__ S, int64_t lds,
                                                            int splits = 1) {
  const int lane = threadIdx.x & 63;
  const int64_t j = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j >= n) return;
  const float* x = X + j * ldx;
  const float a = expf(x[0]);
  float w2 = 0.f;
  for (int64_t c = lane; c < p; c += 64) w2 = fmaf(x[1 + c], x[1 + c], w2);
  w2 = warp_sum(w2);
  for (int64_t c = lane; c < p; c += 64) {
    float g = GW[j * ldg + c];
    for (int z = 1; z < splits; ++z) g += GW[(int64_t)z * n * ldg + j * ldg + c];  // slice order
    S[j * lds + 1 + c] = scale * (g - a * x[1 + c]);
  }
  if (lane == 0) S[j * lds] = scale * (-a + 0.5f * (float)p - 0.5f * a * w2);
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
  if (P.h2) {
    float* sxd = (float*)(P.base + w.off_sxd);
    float* sws = (float*)(P.base + w.off_sws);
    if ((rc = h2_colscale(Xdp, w.ldb, w.N_pad, w.ldb, sws, sxd, s))) return rc;
    // the tensor scale for Z's Xd image, per-column ones for G . Xd's B image
    if (fused_ok(w.pp, w.ldb)) {
      // the fused tile's chunk images of Xd' = t (.) Xd and their scales
      float* xdt = (float*)(P.base + w.off_xdt);
      float* sfz = (float*)(P.base + w.off_sfz);
      const int64_t tot2 = w.N_pad * w.ldb;
      hipLaunchKernelGGL(scale_rows_kernel, dim3((tot2 + 255) / 256), dim3(256), 0, s, Xdp, tp,
                         w.N_pad, w.ldb, xdt);
      if ((rc = check_launch("scale_rows"))) return rc;
      if ((rc = h2_colscale(xdt, w.ldb, w.N_pad, w.ldb, sws, sfz, s))) return rc;
      const int64_t nch = w.N_pad / kFzQ;
      hipLaunchKernelGGL(logreg_fused_image_kernel, dim3((unsigned)((nch * 2048 + 255) / 256)),
                         dim3(256), 0, s, xdt, sfz, nch, P.base + w.off_fimg);
      return check_launch("logreg_fused_image");
    }
    if ((rc = h2_rowsplit(Xdp, w.ldb, w.N_pad, w.pp, w.N_pad, w.pp, sxd + 2 * w.ldb,
                          P.base + w.off_xdx, s)))
      return rc;
    return h2_ysplit(Xdp, w.ldb, w.N_pad, sxd, (_Float16*)(P.base + w.off_xdy), s);
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

static int logreg_step(const float* X, int64_t ldx, int64_t n, int64_t p, float scale, float* S,
                       int64_t lds, const LogregPlan& P, hipStream_t s) {
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
    // W = X[:, 1:] in place (the row image reads its unaligned rows through
    // aligned 16-byte windows), one power-of-two scale per particle row
    if ((rc = h2_rowscale(X + 1, ldx, n, p, w.n_pad, rsw, riw, s))) return rc;
    if ((rc = h2_rowsplit_rows(X + 1, ldx, n, p, w.n_pad, w.pp, rsw, Wx, s))) return rc;
    if (fused_ok(w.pp, w.ldb)) {
      hipLaunchKernelGGL(logreg_fused_kernel, dim3((unsigned)(w.n_pad / 128)), dim3(256), 0, s,
                         (const _Float16*)Wx, w.n_pad, (const float*)riw,
                         (const char*)(base + w.off_fimg), (int)(w.N_pad / kFzQ),
                         (const float*)(base + w.off_sfz), n, GW);
      if ((rc = check_launch("logreg_fused"))) return rc;
      hipLaunchKernelGGL(logreg_finish_kernel, dim3((n + 3) / 4), dim3(256), 0, s, X, ldx, n, p, GW,
                         w.ldb, scale, S, lds, 1);
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
                      s)))
      return rc;
  }
  hipLaunchKernelGGL(logreg_finish_kernel, dim3((n + 3) / 4), dim3(256), 0, s, X, ldx, n, p, GW,
                     w.ldb, scale, S, lds, splits);
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
