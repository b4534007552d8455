// gemm_tiles.hpp -- the two fp32 MFMA tile engines every contraction of the
// SVGD step runs on (v_mfma_f32_32x32x2_f32, exact fp32: a k-ordered fmaf
// chain per output, MI355X_MICROARCH.md "Matrix cores").
//
//  * NT engine  C[BM x BN] = A[BM x K] . B[BN x K]^T, A and B row-major
//    (both operands are rows of the particle matrix: the Gram X X^T, and the
//    logistic-regression Z = W Xd^T).  Register-staged single LDS buffer, the
//    next K-tile in flight during the MFMAs (2 barriers per K-step; 3 blocks
//    per CU cover the barrier gaps).
//  * NN engine  C[BM x BC] = f(A)[BM x K] . B[K x BC], A in the "panel"
//    layout below, f = exp2(scale * a) (the fused RBF kernel) or identity.
//    Double-buffered LDS, one barrier per K-step, one 256-thread block per CU
//    holding a 128 x 512 fp32 accumulator (256 AGPRs per lane).
//
// Both read fragments with ds_read_b128: within a group of 4 consecutive
// MFMAs, lane (r = l&31, h = l>>5) feeds k = 8g + 4h + t to MFMA t, so one
// 16-byte LDS read serves 4 MFMAs (the k order inside a 8-wide group is
// permuted identically for A and B, which leaves every dot product intact).
//
// Panel layout of an M x N matrix produced by the NT engine and consumed by
// the NN engine (D and the logreg G): 128-row x 16-column panels, each a
// contiguous row-major [128][16] block, panels ordered row-panel-major:
//     off(i, j) = ((i/128) * (Npad/16) + j/16) * 2048 + (i%128) * 16 + j%16.
// One NN K-step then streams exactly one contiguous 8 KiB panel.
#pragma once
#include "common.hpp"

namespace dsvgd {

constexpr int kPanelRows = 128;
constexpr int kPanelCols = 16;
constexpr int kPanelElems = kPanelRows * kPanelCols;

__host__ __device__ inline int64_t panel_off(int64_t i, int64_t j, int64_t npad) {
  return ((i >> 7) * (npad >> 4) + (j >> 4)) * kPanelElems + (i & 127) * 16 + (j & 15);
}

// ------------------------------------------------------ tile schedules ----
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

// XCD-aware, L2-grouped tile order.  Workgroups are dispatched round-robin
// over the 8 XCDs (block b runs on XCD b % 8), each with its own 4 MiB L2.
// xcd_linear gives XCD x a contiguous range of logical tiles, and logical
// tiles run in groups of kGroup x kGroup tiles, so the rows an XCD re-reads
// (kGroup A + kGroup B blocks of 128 rows x dp, 2 MiB at dp = 256) stay in
// its L2 instead of re-streaming Y from MALL for every row panel.
constexpr int kXcds = 8;
constexpr int kGroup = 8;

__device__ __forceinline__ int64_t xcd_linear(int64_t b, int64_t total) {
  const int64_t q = total / kXcds, r = total % kXcds, x = b % kXcds;
  return x * q + min(x, r) + b / kXcds;
}

// Tile (bi, bj) of block b in a grid of `total` = groups * kGroup^2 blocks
// over Tm x Tn tiles; SYM: groups over the upper triangle, tiles bi <= bj.
// Returns false for the padding blocks of diagonal / edge groups.
__device__ __forceinline__ bool tile_at(int64_t L, int Tm, int Tn, bool sym, int& bi, int& bj);
__device__ __forceinline__ bool tile_of(int64_t b, int64_t total, int Tm, int Tn, bool sym,
                                        int& bi, int& bj) {
  return tile_at(xcd_linear(b, total), Tm, Tn, sym, bi, bj);
}

// Logical tile L (after the XCD remap) -> (bi, bj); false for padding tiles.
__device__ __forceinline__ bool tile_at(int64_t L, int Tm, int Tn, bool sym, int& bi, int& bj) {
  const int64_t g = L / (kGroup * kGroup);
  const int w = (int)(L % (kGroup * kGroup));
  int gi, gj;
  if (sym) {
    tri_decode(g, (Tn + kGroup - 1) / kGroup, gi, gj);
  } else {
    const int ngn = (Tn + kGroup - 1) / kGroup;
    gi = (int)(g / ngn);
    gj = (int)(g % ngn);
  }
  bi = gi * kGroup + w / kGroup;
  bj = gj * kGroup + w % kGroup;
  return bi < Tm && bj < Tn && (!sym || bi <= bj);
}

__host__ __device__ inline int64_t tile_grid(int64_t Tm, int64_t Tn, bool sym) {
  const int64_t ngm = (Tm + kGroup - 1) / kGroup, ngn = (Tn + kGroup - 1) / kGroup;
  return (sym ? ngn * (ngn + 1) / 2 : ngm * ngn) * kGroup * kGroup;
}

// ------------------------------------------------------------ NT engine ----
// Block = WM x WN waves, each wave TM x TN tiles of 32x32; BK = 32.
// One LDS buffer, two barriers per K-step, the next K-tile in registers
// during the MFMAs (measured: a double-buffered variant with one barrier per
// K-step was 3 % slower at dp = 256 -- it halves the blocks per CU).
template <int TM, int TN, int WM, int WN>
struct NTTile {
  static constexpr int TM_ = TM, TN_ = TN, WM_ = WM, WN_ = WN;
  static constexpr int kThreads = 64 * WM * WN;
  static constexpr int BM = 32 * TM * WM;
  static constexpr int BN = 32 * TN * WN;
  static constexpr int BK = 32;
  static constexpr int LDK = BK + 4;  // 144-B rows: 16 consecutive rows hit 16 distinct 16-B slots
  static constexpr int LA = BM * BK / 4 / kThreads;  // float4 loads per thread (A)
  static constexpr int LB = BN * BK / 4 / kThreads;
  static constexpr int kStage = (BM + BN) * LDK;
  static constexpr int kSmemFloats = kStage;

  f32x16 acc[TM][TN];
  f32x4 ra[LA], rb[LB];

  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
      for (int ni = 0; ni < TN; ++ni)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;
  }

  // Buffer loads: one per-lane byte offset (row t/8, chunk t%8) and scalar
  // offsets for the u-th 32-row group and the K-step, so the staging needs
  // no per-load 64-bit address registers (the row-block bases are uniform).
  // Offsets are 32-bit: a block touches BM (BN) rows x K columns only.
  __device__ __forceinline__ void load(const float* __restrict__ A, int64_t lda,
                                       const float* __restrict__ B, int64_t ldb, int k0) {
    const int t = threadIdx.x;
    constexpr int kRows = kThreads / 8;  // rows covered by one float4 per thread
    const __amdgpu_buffer_rsrc_t rA =
        __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rB =
        __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, 0x7fffffff, 0x00020000);
    const int voA = (int)(((t >> 3) * lda + 4 * (t & 7)) * 4);
    const int voB = (int)(((t >> 3) * ldb + 4 * (t & 7)) * 4);
#pragma unroll
    for (int u = 0; u < LA; ++u)
      ra[u] = __builtin_bit_cast(
          f32x4, __builtin_amdgcn_raw_buffer_load_b128(rA, voA, (int)((u * kRows * lda + k0) * 4), 0));
#pragma unroll
    for (int u = 0; u < LB; ++u)
      rb[u] = __builtin_bit_cast(
          f32x4, __builtin_amdgcn_raw_buffer_load_b128(rB, voB, (int)((u * kRows * ldb + k0) * 4), 0));
  }

  __device__ __forceinline__ void store(float* sA, float* sB) {
    const int t = threadIdx.x;
#pragma unroll
    for (int u = 0; u < LA; ++u) {
      const int f = t + u * kThreads, row = f >> 3, c4 = f & 7;
      *reinterpret_cast<f32x4*>(sA + row * LDK + 4 * c4) = ra[u];
    }
#pragma unroll
    for (int u = 0; u < LB; ++u) {
      const int f = t + u * kThreads, row = f >> 3, c4 = f & 7;
      *reinterpret_cast<f32x4*>(sB + row * LDK + 4 * c4) = rb[u];
    }
  }

  __device__ __forceinline__ void compute(const float* sA, const float* sB, int wm, int wn) {
    const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
#pragma unroll
    for (int g = 0; g < BK / 8; ++g) {
      f32x4 a[TM], b[TN];
#pragma unroll
      for (int mi = 0; mi < TM; ++mi)
        a[mi] = *reinterpret_cast<const f32x4*>(sA + (wm * 32 * TM + mi * 32 + r) * LDK + 8 * g +
                                                4 * h);
#pragma unroll
      for (int ni = 0; ni < TN; ++ni)
        b[ni] = *reinterpret_cast<const f32x4*>(sB + (wn * 32 * TN + ni * 32 + r) * LDK + 8 * g +
                                                4 * h);
#pragma unroll
      for (int t4 = 0; t4 < 4; ++t4)
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
          for (int ni = 0; ni < TN; ++ni) acc[mi][ni] = mfma32(a[mi][t4], b[ni][t4], acc[mi][ni]);
    }
  }

  // Full K loop: A, B point at the block's first row; K % BK == 0.
  __device__ __forceinline__ void run(const float* __restrict__ A, int64_t lda,
                                      const float* __restrict__ B, int64_t ldb, int K, float* smem) {
    const int w = threadIdx.x >> 6, wm = w / WN, wn = w % WN;
    zero();
    load(A, lda, B, ldb, 0);
    float* sA = smem;
    float* sB = smem + BM * LDK;
    for (int k0 = 0; k0 < K; k0 += BK) {
      __syncthreads();
      store(sA, sB);
      __syncthreads();
      if (k0 + BK < K) load(A, lda, B, ldb, k0 + BK);
      compute(sA, sB, wm, wn);
    }
  }
};

// ------------------------------------------------------------ NN engine ----
// Block = WM x 4 waves (256*WM threads): wave (wr, wc) owns rows
// [wr*32*TM, +32*TM) x columns [wc*32*TN, +32*TN), i.e. 16*TM*TN accumulator
// registers; BM = 32*TM*WM rows per block.  In use: WM=2 TM=2 (128 rows, two
// waves per SIMD in one block, 128 accumulators each).  (Measured and
// dropped: 1 wave/SIMD with 256 accumulators, 64-row blocks at 2 per CU, a
// transposed B image, s_setprio around the MFMA clusters -- all slower.)
// K-step = BJ columns of A (one or two 16-column panels) and BJ rows of B.
//
// BJ_ = 32: 32-deep K-steps (two D panels per step: half the barriers and
// LDS-read restarts per unit of work).  Double-buffered that is exactly
// 2 x (16 KiB A + 64 KiB B) = 160 KiB, so the A image drops its row padding
// and XOR-swizzles its 16-B chunks instead: chunk' = chunk ^ ((row >> 1) & 7)
// keeps a ds_read_b128 lane group (16 rows, 2 per 64-bank line) conflict-free.
template <int TN, bool EXP, int WM = 2, int TM_ = 4 / WM, int BJ_ = 16, bool SWZB = true>
struct NNTile {
  static constexpr int kThreads = 256 * WM;
  static constexpr int TM = TM_;
  static constexpr int BM = 32 * TM * WM;
  static constexpr int BC = 128 * TN;
  static constexpr int BJ = BJ_;
  static constexpr bool kSwz = BJ == 32;
  static constexpr int LDA = kSwz ? BJ : BJ + 4;  // 16: 80-B rows (conflict-free b128)
  static constexpr int SA = BM * LDA;
  static constexpr int SB = BJ * BC;
  static constexpr int kStage = SA + SB;
  static constexpr int kSmemFloats = 2 * kStage;
  static constexpr int LA = BM * BJ / 4 / kThreads;
  static constexpr int RPT = BM * 4 / kThreads > 1 ? BM * 4 / kThreads : 1;  // rows per thread
  static constexpr int LB = BJ * BC / 4 / kThreads;
  static_assert(LA >= 1 && LB >= 1, "tile too small for the block");
  static_assert(BM == 64 || BM == 128, "BM must divide the 128-row panel");
  static_assert(BJ == 16 || BJ == 32, "BJ is 16 or 32");
  static_assert(kSmemFloats * 4 <= 160 * 1024, "LDS budget");

  f32x16 acc[TM][TN];
  f32x4 ra[LA], rb[LB];
  float rs[RPT];  // EXP: row-sum partials of the rows this thread stages

  // A image offset of (row, 16-B chunk)
  __device__ __forceinline__ static int a_off(int row, int chunk) {
    return row * LDA + 4 * (kSwz ? (chunk ^ ((row >> 1) & 7)) : chunk);
  }
  // B image column swizzle: the two half-waves of a fragment read (k rows 4
  // apart, 4*BC floats = a multiple of 64 banks) would hit the same banks;
  // flipping column bit 5 on rows with (k >> 2) odd moves the upper half-wave
  // 32 banks over.  4-aligned column groups stay contiguous (b128 writes).
  __device__ __forceinline__ static int b_swz(int k, int col) {
    return SWZB ? (col ^ (((k >> 2) & 1) << 5)) : col;
  }
  // staged A vector u of thread t: panel p (16 columns each), row, chunk in panel
  __device__ __forceinline__ static void a_map(int t, int u, int& p, int& row, int& c4) {
    const int f = t + u * kThreads;
    p = f / (BM * 4);
    const int fi = f % (BM * 4);
    row = fi >> 2;
    c4 = fi & 3;
  }

  // Buffer loads: per-lane byte offsets are loop invariant (one 32-bit VGPR
  // each, hoisted), the K-step position is a scalar offset, so the K loop
  // carries no 64-bit address arithmetic on the VALU (every VALU instruction
  // beside the f32 MFMAs costs MFMA issue time).
  __device__ __forceinline__ void load(const float* __restrict__ Apanels, const float* __restrict__ B,
                                       int64_t ldb, int64_t j0) {
    const int t = threadIdx.x;
    const __amdgpu_buffer_rsrc_t rA =
        __builtin_amdgcn_make_buffer_rsrc((void*)Apanels, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rB =
        __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, 0x7fffffff, 0x00020000);
    const int soA = (int)((j0 >> 4) * kPanelElems * 4);
    const int soB = (int)(j0 * ldb * 4);
#pragma unroll
    for (int u = 0; u < LA; ++u) {
      int p, row, c4;
      a_map(t, u, p, row, c4);
      ra[u] = __builtin_bit_cast(
          f32x4, __builtin_amdgcn_raw_buffer_load_b128(rA, (p * kPanelElems + row * 16 + 4 * c4) * 4,
                                                       soA, 0));
    }
#pragma unroll
    for (int u = 0; u < LB; ++u) {
      const int f = t + u * kThreads, row = f / (BC / 4), c4 = f % (BC / 4);
      rb[u] = __builtin_bit_cast(
          f32x4, __builtin_amdgcn_raw_buffer_load_b128(rB, (int)((row * ldb + 4 * c4) * 4), soB, 0));
    }
  }

  // EXP: the staging thread turns its 4 D values into k = exp2(D * scale)
  // once (not once per reading wave), skips the diagonal and accumulates the
  // row-sum partial.  dgl = (global row of the block's row 0) - (global
  // column of this K-step's column 0): the diagonal k_ii is left out (phi_finish
  // adds the self term exactly) so no accumulator carries the O(1) self term
  // while it sums ~n tiny off-diagonal terms.
  __device__ __forceinline__ void store(float* st, float scale, int64_t dgl) {
    const int t = threadIdx.x;
    float* sA = st;
    float* sB = st + SA;
#pragma unroll
    for (int u = 0; u < LA; ++u) {
      int p, row, c4;
      a_map(t, u, p, row, c4);
      const int chunk = 4 * p + c4;
      if (EXP) {
        // Diagonal entry (row i, column c of this K-step) <=> c - i = dgl,
        // so only K-steps with -BM < dgl < BJ hold one; the rest skip the test.
        // (|dgl| < 2^31 for every launch the ABI accepts.)
        if (dgl > -BM && dgl < BJ) {
          const int qd = (int)dgl + row - 4 * chunk;
#pragma unroll
          for (int q = 0; q < 4; ++q)
            ra[u][q] = (qd == q) ? 0.f : __builtin_amdgcn_exp2f(ra[u][q] * scale);
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) ra[u][q] = __builtin_amdgcn_exp2f(ra[u][q] * scale);
        }
        rs[u % RPT] += (ra[u][0] + ra[u][1]) + (ra[u][2] + ra[u][3]);
      }
      *reinterpret_cast<f32x4*>(sA + a_off(row, chunk)) = ra[u];
    }
#pragma unroll
    for (int u = 0; u < LB; ++u) {
      const int f = t + u * kThreads, row = f / (BC / 4), col = 4 * (f % (BC / 4));
      *reinterpret_cast<f32x4*>(sB + row * BC + b_swz(row, col)) = rb[u];
    }
  }

  __device__ __forceinline__ void compute(const float* st, int wr, int wc) {
    const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
    const float* sA = st;
    const float* sB = st + SA;
#pragma unroll
    for (int g = 0; g < BJ / 8; ++g) {
      f32x4 a[TM];
#pragma unroll
      for (int mi = 0; mi < TM; ++mi)
        a[mi] = *reinterpret_cast<const f32x4*>(sA + a_off(wr * 32 * TM + mi * 32 + r, 2 * g + h));
      // all of this group's B fragments are read before its MFMAs (one
      // LDS wait per group instead of one per 4-MFMA cluster)
      float b[4][TN];
#pragma unroll
      for (int t4 = 0; t4 < 4; ++t4) {
        const int k = 8 * g + 4 * h + t4;
        const float* brow = sB + k * BC;
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) b[t4][ni] = brow[b_swz(k, wc * 32 * TN + ni * 32 + r)];
      }
#pragma unroll
      for (int t4 = 0; t4 < 4; ++t4) {
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
          for (int ni = 0; ni < TN; ++ni) acc[mi][ni] = mfma32(a[mi][t4], b[t4][ni], acc[mi][ni]);
      }
    }
  }

  // Apanels: the block's row-panel (128 rows x K, panel layout); B: K x BC
  // (row-major, ldb, already offset to the block's first column); the K range
  // [k0, k1) (multiples of 16) is this block's split-K slice.
  __device__ __forceinline__ void run(const float* __restrict__ Apanels, const float* __restrict__ B,
                                      int64_t ldb, int64_t k0, int64_t k1, float scale,
                                      float* smem, int64_t row_g0 = INT64_MIN / 2) {
    const int w = threadIdx.x >> 6, wr = w >> 2, wc = w & 3;
#pragma unroll
    for (int u = 0; u < RPT; ++u) rs[u] = 0.f;
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
      for (int ni = 0; ni < TN; ++ni)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[mi][ni][q] = 0.f;
    if (k0 >= k1) return;
    load(Apanels, B, ldb, k0);
    store(smem, scale, row_g0 - k0);
    __syncthreads();
    // unrolled by two so both LDS stage bases are compile-time constants
    // (immediate ds_read / ds_write offsets, no per-step address VALU)
    for (int64_t j0 = k0; j0 < k1; j0 += 2 * BJ) {
      step<0>(Apanels, B, ldb, j0, k1, scale, smem, row_g0, wr, wc);
      if (j0 + BJ < k1) step<1>(Apanels, B, ldb, j0 + BJ, k1, scale, smem, row_g0, wr, wc);
    }
  }

  template <int CUR>
  __device__ __forceinline__ void step(const float* __restrict__ Apanels,
                                       const float* __restrict__ B, int64_t ldb, int64_t j0,
                                       int64_t k1, float scale, float* smem, int64_t row_g0, int wr,
                                       int wc) {
    const bool more = j0 + BJ < k1;
    if (more) load(Apanels, B, ldb, j0 + BJ);
    compute(smem + CUR * kStage, wr, wc);
    if (more) store(smem + (CUR ^ 1) * kStage, scale, row_g0 - (j0 + BJ));
    __syncthreads();
  }

  // EXP: the full row sum of staged row a_map(t, u) (u < RPT) is the sum over
  // the 4 consecutive lanes staging that row; returned on every lane (the
  // lane with c4 == 0 is the writer).
  __device__ __forceinline__ float row_sum(int u) const {
    float v = rs[u];
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    return v;
  }
};

}  // namespace dsvgd
