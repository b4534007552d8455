/*
 * dsvgd.h -- C ABI of libdsvgd_hip.so, the MI355X (gfx950) SVGD particle-update
 * engine behind the drop-in `dsvgd.Sampler` / `dsvgd.DistSampler` Python API.
 *
 * Conventions (every entry point):
 *   - plain pointers + int64 sizes; every float buffer is caller-owned DEVICE
 *     memory, row-major fp32, with an explicit leading dimension (elements);
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream); every
 *     call only ENQUEUES work on it (no host sync, no allocation), so the whole
 *     SVGD step can be captured into a hipGraph;
 *   - return 0 on success, a negative DSVGD_E* code otherwise; the message is
 *     in dsvgd_last_error() (thread-local).  No C++ exception crosses the ABI.
 *
 * Padding contract ("padded shapes"): n_pad = roundup(n,128), m_pad =
 * roundup(m,128), dp = roundup(d,32); Y has >= n_pad+128 rows and ldy =
 * dsvgd_ldy(dp) columns; D is m_pad x n_pad (ldd >= n_pad).  The helpers
 * dsvgd_dp / dsvgd_ldy / dsvgd_pad128 compute these.
 *
 * The reference interface each call replaces is cited beside it
 * (paths relative to the Sandy4321/dist-svgd tree).
 */
#ifndef DSVGD_H_
#define DSVGD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DSVGD_ABI_VERSION 4

enum {
  DSVGD_OK = 0,
  DSVGD_E_ARG = -1,    /* bad size / pointer / alignment                    */
  DSVGD_E_LAUNCH = -2, /* hipLaunchKernel (or a HIP runtime call) failed     */
  DSVGD_E_UNSUPPORTED = -3
};

/* number of histogram bins of one radix-select pass (11-bit digits) */
#define DSVGD_RADIX_BINS 2048
/* bracketed select: the candidate buffer (cand_cap floats) is split into one
 * fixed-capacity SLOT per wave of the distance launch, written without any
 * atomic or block barrier:
 *   cand[0 : nslots)            u32 slot_cnt   (entries in [lo,hi]; bit 31 =
 *                                               weight 2, a mirrored tile)
 *   cand[nslots : 2 nslots)     u32 slot_below (entries < lo, same weight)
 *   cand[2 nslots + s*slot_cap] the slot's values (slot_cap floats each)
 * with slot_cap = (cand_cap - 2 nslots) / nslots; a slot that fills up sets
 * `overflow` and the select falls back to the passes over D (still exact). */
#define DSVGD_SLOT_WEIGHT2 0x80000000u

/* Device-resident state of the median-bandwidth radix select.  Allocate
 * dsvgd_select_state_bytes() of device memory; the histogram is the first
 * member so a distributed caller can all-reduce it in place (int64 SUM), and
 * below_total / ncand_total / overflow are adjacent for one int64[3]
 * all-reduce (between dsvgd_bracket_totals and dsvgd_bracket_check). */
typedef struct dsvgd_select_state {
  uint64_t hist[DSVGD_RADIX_BINS]; /* per-pass counts (u64: n^2 may be 2^32)  */
  uint64_t k;                      /* rank still to find inside the prefix    */
  uint64_t n_total;                /* global particle count n (matrix n x n)  */
  uint32_t prefix;                 /* key bits fixed by the passes so far     */
  uint32_t passes_done;
  float median;                    /* k-th smallest squared distance          */
  float h;                         /* bandwidth  h = median / log(n)          */
  float inv_h;                     /* 1 / h (read by the phi kernels)         */
  uint32_t fallback;               /* bracketed: 1 = select over D itself     */
  uint64_t below_total;            /* bracketed: # entries < lo      } int64[3], */
  uint64_t ncand_total;            /* bracketed: # entries in [lo,hi] } all-     */
  uint64_t overflow;               /* bracketed: # overflowed slots  } reduced  */
  float lo, hi;                    /* bracketed: the sample bracket           */
  uint64_t cand_cap;               /* bracketed: candidate buffer floats      */
  uint64_t nslots;                 /* bracketed: slots of the last sqdist     */
  uint64_t slot_cap;               /* bracketed: floats per slot              */
} dsvgd_select_state;

/* select_mode of dsvgd_sqdist */
#define DSVGD_SEL_NONE 0    /* fixed bandwidth: distances only                 */
#define DSVGD_SEL_HIST 1    /* fused radix digit-1 histogram                   */
#define DSVGD_SEL_BRACKET 2 /* count < lo, compact [lo, hi] into candidates    */

/* ---- meta ------------------------------------------------------------- */
int dsvgd_abi_version(void);
const char* dsvgd_last_error(void);
size_t dsvgd_select_state_bytes(void);
int64_t dsvgd_pad128(int64_t n);
int64_t dsvgd_dp(int64_t d);   /* padded feature width: roundup(d, 32)     */
int64_t dsvgd_ldy(int64_t dp); /* row stride of Y = [Xc | S] (phi col tile) */

/* ---- particle preparation ---------------------------------------------- */
/* mean[c] = (1/n) sum_j X[j][c]  (deterministic two-level sum; `partial`
 * is workspace of dsvgd_colmean_workspace_floats(n, d) floats).
 * Centering is exact algebra for phi (sum_j k_ij (x_i - x_j) is translation
 * invariant) and keeps ||x||^2 - 2 x.y well conditioned. */
size_t dsvgd_colmean_workspace_floats(int64_t n, int64_t d);
int dsvgd_colmean(const float* X, int64_t ldx, int64_t n, int64_t d, float* partial, float* mean,
                  void* stream);
/* center[c] = the lower median of X[:, c] over min(n, 1024) evenly spaced rows
 * (row k n / m): the centre the engine packs against.  Robust where the mean
 * is not: one diverging particle moves the mean by its distance / n and every
 * other particle's |x|^2 + |y|^2 - 2 x.y (and r x - K X) cancellation with it. */
int dsvgd_colcenter(const float* X, int64_t ldx, int64_t n, int64_t d, float* center,
                    void* stream);

/* Y[j] = [X[j]-mean | score_scale*S[j]] zero padded to (rows_pad x ldy);
 * norms[j] = ||X[j]-mean||^2.  Replaces the per-pair operand gathering of
 * dsvgd/sampler.py:37-39 and dsvgd/distsampler.py:90-99.  S may be NULL
 * (S half left zero); X may be NULL (then only the S half of rows < n is
 * written: the scores arriving after the distance stage, mean/norms unused). */
int dsvgd_pack(const float* X, int64_t ldx, const float* S, int64_t lds, float score_scale,
               const float* mean, int64_t n, int64_t d, int64_t rows_pad, float* Y, int64_t ldy,
               float* norms, void* stream);
/* dsvgd_pack + the FmtH2 statistics of what it writes (ldy <=
 * dsvgd_pack_max_ldy() = 2048, i.e. d <= 1024): partial (uint32,
 * dsvgd_pack_blocks(rows_pad) x ldy column maxima) and gmax (4 words per
 * block: [4b] / [4b+1] the largest |entry| of the X half [0, dp) / of the
 * rest; [4b+2] / [4b+3] the smallest nonzero row max of each half over the
 * block's rows < n, +inf if none -- fp32 bit patterns), the input of
 * dsvgd_h2_scales -- the scales and the range guard without a second pass
 * over Y.  With X NULL only the S half's statistics are (re)written, so
 * pack(X) then pack(NULL, S) leaves those of the whole Y.  partial = gmax =
 * NULL: dsvgd_pack.  rowscale (nullable, rows_pad floats, with X): the FmtH2
 * power-of-two scale of each row's X half (largest magnitude -> [2^14,
 * 2^15); 1 for a zero row or a row >= n) -- the Gram's per-row image scales. */
int64_t dsvgd_pack_blocks(int64_t rows_pad);
int64_t dsvgd_pack_max_ldy(void);
int dsvgd_pack_h2(const float* X, int64_t ldx, const float* S, int64_t lds, float score_scale,
                  const float* mean, int64_t n, int64_t d, int64_t rows_pad, float* Y, int64_t ldy,
                  float* norms, uint32_t* partial, uint32_t* gmax, float* rowscale,
                  void* stream);

/* ---- pairwise squared distances ---------------------------------------- */
/* D[i][j] = ||y_i - y_j||^2 for the owned row block i in [row0, row0+m) of Y
 * against all j < n, y = the first d columns of Y (centred particles).
 * d <= 2: explicit differences on the VALU (exact like the reference);
 * d > 2: max(0, |y_i|^2 + |y_j|^2 - 2 y_i.y_j) on v_mfma_f32_32x32x2_f32,
 * upper-triangle tiles only when m == n and row0 == 0 (the transpose is
 * stored too).  D[i][i] = 0 exactly, pads = +inf, panel layout (ldd = n_pad).
 * select_mode (DSVGD_SEL_*): HIST accumulates radix digit 1 of the valid
 * entries into st->hist; BRACKET counts the entries < st->lo and writes the
 * entries in [st->lo, st->hi] into the wave slots of cand (layout above;
 * st->nslots / st->slot_cap are set by the launch).
 * Replaces torch.dist(x, y, p=2)**2 inside kernel(...) at
 * experiments/logreg.py:60-61 / experiments/gmm.py:23-24 as called per pair
 * from dsvgd/sampler.py:38 and dsvgd/distsampler.py:91-97. */
int dsvgd_sqdist(const float* Y, int64_t ldy, const float* norms, int64_t row0, int64_t m,
                 int64_t n, int64_t d, float* D, int64_t ldd, int select_mode,
                 dsvgd_select_state* st, float* cand, void* stream);
/* dsvgd_sqdist's explicit-difference kernel forced for any d <= 64 (the
 * precision studies of DESIGN.md 3; dsvgd_sqdist takes it for d <= 2). */
int dsvgd_sqdist_direct(const float* Y, int64_t ldy, const float* norms, int64_t row0, int64_t m,
                        int64_t n, int64_t d, float* D, int64_t ldd, int select_mode,
                        dsvgd_select_state* st, float* cand, void* stream);

/* ---- median bandwidth: exact radix select over the n x n distances ----- */
/* (absent in the reference, whose kernel bandwidth is fixed at h=1; the
 * median heuristic is pinned in SURVEY.md a18: lower median, k=(n^2-1)//2
 * over the full matrix incl. the diagonal, h = median / log n.)
 * select_init: k = k_rank if k_rank >= 0 else (n_total^2-1)/2, prefix 0. */
int dsvgd_select_init(dsvgd_select_state* st, int64_t n_total, int64_t k_rank, void* stream);
/* histogram of key digit `pass` (1: bits 31..21, 2: 20..10, 3: 9..0) of the
 * finite entries (pads +inf / NaN skipped) whose higher digits equal
 * st->prefix, over D[0:count) -- or, when cand != NULL and the bracket holds
 * (st->fallback == 0), over the local candidate slots instead.
 * sym_npad > 0: D is the symmetric layout dsvgd_sqdist_x3 writes with
 * layout = 1 (upper-triangle tiles only; count = sym_npad^2): off-diagonal
 * tiles count twice, lower tiles are skipped. */
int dsvgd_radix_hist(const float* D, int64_t count, const float* cand, int pass,
                     dsvgd_select_state* st, int64_t sym_npad, void* stream);
/* pick the bin holding rank k, fix its digit, clear hist; after pass 3
 * writes median, h = median/log(n_total) (1 if median == 0 or n == 1), inv_h. */
int dsvgd_radix_pick(dsvgd_select_state* st, int pass, void* stream);
/* bracketed select: out[p] = ||y_i - y_j||^2 for s pairs (i,j) drawn by a
 * seeded hash (identical on every rank for the same Y) ... */
int dsvgd_sample_sqdist(const float* Y, int64_t ldy, int64_t n, int64_t d, int64_t s,
                        uint64_t seed, float* out, void* stream);
/* ... whose k_lo-th / k_hi-th order statistics (two select states run over
 * `out`) become the bracket [lo, hi] of st (k = (n_total^2-1)/2) ... */
int dsvgd_bracket_init(dsvgd_select_state* st, int64_t n_total, const dsvgd_select_state* lo_st,
                       const dsvgd_select_state* hi_st, int64_t cand_cap, void* stream);
/* ... the same three steps (sample_sqdist into `sample`, both sample
 * selects, bracket_init of st) in seven launches: the two selects share each
 * sweep over the sample and one launch picks both digits.  lo_st / hi_st:
 * histograms zero on entry (as dsvgd_select_init or a previous call leave
 * them); they end as after the three passes.  s % 4 == 0, 16-byte aligned
 * sample, 0 <= k_lo <= k_hi < s. */
int dsvgd_sample_bracket(const float* Y, int64_t ldy, int64_t n, int64_t d, int64_t s,
                         uint64_t seed, int64_t k_lo, int64_t k_hi, float* sample,
                         dsvgd_select_state* lo_st, dsvgd_select_state* hi_st,
                         dsvgd_select_state* st, int64_t n_total, int64_t cand_cap,
                         void* stream);
/* dsvgd_sample_bracket in two parts (ABI 4): a rank's share of the sample --
 * dsvgd_sample_sqdist's pairs [p0, p1) of s, the same pairs and values --
 * and, once the shares are all-gathered into the whole sample, the selects
 * and the bracket (the last six launches of dsvgd_sample_bracket). */
int dsvgd_sample_sqdist_range(const float* Y, int64_t ldy, int64_t n, int64_t d, int64_t s,
                              uint64_t seed, int64_t p0, int64_t p1, float* out, void* stream);
int dsvgd_sample_bracket_select(const float* sample, int64_t s, int64_t k_lo, int64_t k_hi,
                                dsvgd_select_state* lo_st, dsvgd_select_state* hi_st,
                                dsvgd_select_state* st, int64_t n_total, int64_t cand_cap,
                                void* stream);
/* ... then, after dsvgd_sqdist(BRACKET): bracket_totals sums the slots into
 * below_total / ncand_total / overflow (a distributed caller all-reduces
 * those three int64), and bracket_check decides exactly: below <= k <
 * below + ncand and no slot overflowed -> k -= below, the passes read the
 * candidate slots; otherwise they read D (fallback). */
int dsvgd_bracket_totals(dsvgd_select_state* st, const float* cand, void* stream);
int dsvgd_bracket_check(dsvgd_select_state* st, void* stream);
/* fixed-bandwidth mode: st->h = h, st->inv_h = 1/h */
int dsvgd_set_bandwidth(dsvgd_select_state* st, float h, void* stream);

/* dsvgd_sqdist's Gram path (d > 2) on the split engine (fp32-accurate, see
 * dsvgd_phi_mm_x3): Yg = dsvgd_rowsplit(Y, ldy, n_pad, dp, n_pad + 256, dp, 0)
 * with dp = roundup(d, 32), n_pad = roundup(n, 128) (256 rows of zero slack
 * for the 256 x 256 tiles); same outputs and select
 * modes as dsvgd_sqdist.  layout 0: the full panel-layout D; layout 1 (m ==
 * n, row0 == 0 only) the SYMMETRIC LAYOUT: tiles (I, J) with J < I are not
 * written -- consumers read them transposed (dsvgd_phi_mm_x3 with sym = 1,
 * dsvgd_radix_hist with sym_npad).  Requires dp * (n_pad + 256) * 6 < 2^31. */
int dsvgd_sqdist_x3(const void* Yg, const float* norms, int64_t row0, int64_t m, int64_t n,
                    int64_t d, float* D, int64_t ldd, int select_mode, dsvgd_select_state* st,
                    float* cand, int layout, void* stream);

/* ---- phi: K.[Xc | S] on MFMA with the fused RBF exp -------------------- */
/* KY_z[i][:] = sum_{j in slice z, j != row0+i} exp(-D[i][j]/h) Y[j][:] and
 * rowsum_z[i] = the same sum of exp(-D[i][j]/h), for split-K slices z < splits
 * of the columns (h read from st on device; row0 = index of the block's first
 * row in the interacting set; the diagonal self term is added exactly by
 * dsvgd_phi_finish instead of being summed among ~n tiny terms).  KY holds splits x m rows (ldk >= ldy,
 * slice z at KY + z*m*ldk), rowsum splits x roundup(m,128) floats.
 * Replaces the inner loop of dsvgd/sampler.py:35-40 (_phi_hat) and
 * dsvgd/distsampler.py:84-101.  dsvgd_phi_splits gives a slice count that
 * fills the 256 CUs (>= 2 blocks per CU) for an m-row block. */
int64_t dsvgd_phi_splits(int64_t m, int64_t n, int64_t ldy);
/* The symmetric layout's phi_mm form (A/B switch, returns the previous
 * setting): 1 (default) = one launch, each row block's split-K slices walking
 * contiguous K ranges ascending, transposed K-steps first (phi_w1 DS 4);
 * 0 = two launches split at each row block's diagonal tile (DS 1 + DS 2). */
int dsvgd_phi_set_symrow(int on);
/* The one-kernel FmtH2 Gram units (dsvgd_sqdist_h2, dsvgd_sqdist_h2_parts):
 * 1 (default) = gram_rs_kernel, split roles -- four waves issue only the
 * MFMAs (and stage the strip image by LDS-DMA), four waves write the
 * previous tile's epilogue (D values, bracket accounting, stores) from an
 * LDS hand-off; 0 = gram_w1_kernel, one wave per SIMD with the epilogue
 * between its MFMAs.  Identical D and candidates.  5, 6, 7: timing probes of
 * the bracketed symmetric form only (5: no epilogue, 6: no MFMAs -- D wrong;
 * 7: epilogue waves at priority 1; 8: barrier clock stamps into the buffer
 * given to dsvgd_gram_debug_stamps; 9: the MFMA waves' B ring 4 deep).
 * Returns the previous setting. */
int dsvgd_gram_set_rs(int on);
/* CUs the persistent launches issued after this call leave free (returns
 * the previous; 0 = none): the pipelined Gauss-Seidel sweep sets it around
 * its side-stream passes so the walk (one workgroup, most of a CU's LDS)
 * finds a free CU beside them.  A launch-time host setting. */
int dsvgd_set_cu_reserve(int cus);
/* Strips per unit group of the split-role Gram's walk (A/B switch, returns
 * the previous setting): 8 (default) or 16.  Each group's strip images stay
 * in an XCD's L2 while every column pair's image streams past once. */
int dsvgd_gram_set_group(int g);
/* Probe 8 of dsvgd_gram_set_rs: int64 [8 blocks][8 waves][512] shader-clock
 * stamps, on arriving at and leaving each barrier (NULL: probe off). */
int dsvgd_gram_debug_stamps(void* buf);
/* The split-K slices of the symmetric layout's phi_mm (n x n, the engine's
 * KY / rowsum hold this many): dsvgd_phi_splits, or with the one-launch form
 * half as many while each fp32 chain stays within 2 x 16384 columns and the
 * launch has >= 512 blocks (n = 65536, d = 256: 2). */
int64_t dsvgd_phi_splits_sym(int64_t n, int64_t ldy);
/* Map a phi_mm launch's split-K slices to XCDs (A/B switch, returns the
 * previous mask): the blocks of one XCD then walk one K range and share its
 * Yx K-steps in their L2.  Bits: 1 = the symmetric layout's one-launch form
 * (default), 2 = the full layout / window launches, 4 = the pair split's
 * batched forward partials; grids of one column block whose slice count
 * divides 8 and whose block count 8 divides. */
int dsvgd_phi_set_xmap(int mask);
/* logreg's G . Xd on the FmtH2 engine with 256 output columns (p <= 255):
 * phi_w1's one-wave-per-SIMD shape in 128 x 256 blocks (1; measured slower)
 * or the 8-wave 256-row NN tile (0, default).  A/B switch; returns the
 * previous setting. */
int dsvgd_phi_set_gxd_w1(int on);
int dsvgd_phi_mm(const float* D, int64_t ldd, const float* Y, int64_t ldy, int64_t row0,
                 int64_t m, int64_t n, const dsvgd_select_state* st, int64_t splits, float* KY,
                 int64_t ldk, float* rowsum, void* stream);
/* dsvgd_phi_mm gated on a device word: does nothing while *gate reads 0 --
 * the exact f32 fallback of dsvgd_phi_mm_h2 where the FmtX3 image does not
 * fit its 32-bit offsets (roundup(n,128) * ldy * 6 >= 2^31); full D layout
 * only (ABI 4). */
int dsvgd_phi_mm_gated(const float* D, int64_t ldd, const float* Y, int64_t ldy, int64_t row0,
                       int64_t m, int64_t n, const dsvgd_select_state* st, int64_t splits,
                       float* KY, int64_t ldk, float* rowsum, const float* gate, void* stream);

/* phi_mm on the bf16 MFMA at fp32 accuracy (the default engine): both
 * operands split three ways into bf16 (v = v0 + v1 + v2 to ~2^-26 |v|) and
 * the six products a_i b_j with i + j <= 2 accumulated in fp32, so the
 * result carries fp32 GEMM rounding, not bf16's.  Same arguments, outputs,
 * split-K slices and diagonal rule as dsvgd_phi_mm; Yx = dsvgd_ysplit(Y)
 * (rows >= roundup(n, 128)).  Requires roundup(n,128) * ldy * 6 < 2^31.
 * sym = 1: D is dsvgd_sqdist_x3's symmetric layout (m == n, row0 == 0,
 * ldy % 256 == 0); a K-step in a column tile J < I is read from the stored
 * tile (J, I), transposed in LDS.  m16 = 1: the v_mfma_f32_16x16x32_bf16
 * form (ldy % 256 == 0), which needs Yx built with swz = 0; m16 = 0 needs
 * swz = 1.
 * dsvgd_ysplit: Yx[kstep][part][column][16] (bf16) from the first `rows`
 * rows of Y (rows a multiple of 16; dsvgd_ysplit_bytes(rows, ldy) bytes,
 * 16-byte aligned); swz = 1: 16-byte halves swapped on columns with bit 3
 * set (the 32x32x16 engines' image), swz = 0: unswizzled (16x16x32). */
int64_t dsvgd_ysplit_bytes(int64_t rows, int64_t ldy);
/* Row image for the split NT engine (Gram, logreg Z): img[kstep][part][row]
 * [16] (bf16) = the three parts of A[row][16 kstep + k] for row < rows_pad,
 * column < kpad (zero outside rows x cols); rows_pad, kpad multiples of 16;
 * dsvgd_rowsplit_bytes(rows_pad, kpad) bytes, 16-byte aligned; swz = 1:
 * 16-byte halves swapped on rows with bit 3 set (32x32x16 engines), swz = 0:
 * unswizzled (16x16x32 engines). */
int64_t dsvgd_rowsplit_bytes(int64_t rows_pad, int64_t kpad);
int dsvgd_rowsplit(const float* A, int64_t lda, int64_t rows, int64_t cols, int64_t rows_pad,
                   int64_t kpad, void* img, int swz, void* stream);
/* gate (nullable): the FmtH2 range-guard word of a dsvgd_h2_scales output
 * over all ldy columns (&scale[2 ldy + 2]): dsvgd_ysplit and dsvgd_phi_mm_x3
 * do nothing while it reads 0 -- the FmtX3 fallback of dsvgd_phi_mm_h2,
 * launched behind it on the same stream, so exactly one of the two writes KY
 * and rowsum without a host round trip (graph-capturable). */
int dsvgd_ysplit(const float* Y, int64_t ldy, int64_t rows, void* Yx, int swz, const float* gate,
                 void* stream);
int dsvgd_phi_mm_x3(const float* D, int64_t ldd, const void* Yx, int64_t ldy, int64_t row0,
                    int64_t m, int64_t n, const dsvgd_select_state* st, int64_t splits, float* KY,
                    int64_t ldk, float* rowsum, int sym, int m16, const float* gate, void* stream);

/* ---- FmtH2: the fp16 two-part split engine (the default) ---------------
 * An operand v enters the fp16 MFMA as s v = v0 + v1, v0 = f16(s v),
 * v1 = f16(s v - v0), s a power of two putting the operand's largest
 * magnitude in [2^14, 2^15); the products a0 b0 + a0 b1 + a1 b0 are exact in
 * fp32 and the dropped a1 b1 and split remainder are <= 2^-22 relative, below
 * the fp32 accumulation rounding of any of these GEMMs: fp32-level results
 * from half the MFMAs of the X3 engine (gemm_x3.hpp, h2.hip).  The scale
 * divides out exactly inside each kernel: outputs are unscaled fp32.
 *
 * The window: an entry keeps 22 significant bits only within 2^-16 of the
 * largest magnitude sharing its scale; below it, only 2^-38 of that largest
 * (absolute).  So the NT row images (the Gram's Xc, logreg's W) take one
 * scale per ROW (dsvgd_h2_rowscale / dsvgd_pack_h2's rowscale: no particle
 * sits in another's window), and the NN B operand (phi_mm's [Xc | S], one
 * scale per column) is guarded: dsvgd_h2_scales flags a step whose particles'
 * rows span more than 2^16 in a half of Y, and that step's phi_mm runs on the
 * FmtX3 engine instead (dsvgd_phi_mm_h2 / _x3 `gate`).
 *
 * dsvgd_h2_colscale: per column c of A (rows x cols), scale[c] = s_c and
 * scale[cols + c] = 1 / s_c; scale[2 cols] = t = min s_c over the nonzero
 * finite columns (1 if a column holds an inf / NaN, which then propagate),
 * scale[2 cols + 1] = 1 / t, scale[2 cols + 2] = 0 (no range guard).
 * scale: 2 cols + 3 floats; ws: dsvgd_h2_colscale_workspace_floats(rows,
 * cols) floats.  dsvgd_h2_colscale_guarded (ABI 4; the unfused d > 1024
 * path) also writes the RANGE GUARD of dsvgd_h2_scales for the halves
 * [0, dp) and [dp, cols) (a second pass over A's rows). */
size_t dsvgd_h2_colscale_workspace_floats(int64_t rows, int64_t cols);
int dsvgd_h2_colscale(const float* A, int64_t lda, int64_t rows, int64_t cols, float* ws,
                      float* scale, void* stream);
int dsvgd_h2_colscale_guarded(const float* A, int64_t lda, int64_t rows, int64_t cols, int64_t dp,
                              float* ws, float* scale, void* stream);
/* dsvgd_h2_colscale's output over Y's first cols columns (cols = dp: the X
 * half; cols = ldy: all of Y), bit-identical, from dsvgd_pack_h2's maxima
 * (nb = dsvgd_pack_blocks(rows_pad)); scale[2 cols + 2] = the RANGE GUARD:
 * 1.0 when the X half (or, cols = ldy, the S half) has its largest magnitude
 * more than 2^16 times its smallest nonzero row max, else 0.0. */
int dsvgd_h2_scales(const uint32_t* partial, const uint32_t* gmax, int64_t nb, int64_t ldy,
                    int64_t cols, int64_t dp, float* scale, void* stream);
/* fp16 images (dsvgd_h2_image_bytes(rows, cols) bytes, 16-byte aligned):
 * ysplit: Yh[kstep][part][column][16] of colscale[c] * Y[16 kstep + k][c]
 * (the NN engine's B operand, rows a multiple of 16); rowsplit:
 * img[kstep][part][row][16] of tscale[0] * A[row][16 kstep + k] (the NT
 * engine's operands, zero outside rows x cols).  16-byte halves swapped on
 * columns / rows with bit 3 set (32x32x16 fragment reads). */
int64_t dsvgd_h2_image_bytes(int64_t rows, int64_t cols);
int dsvgd_h2_ysplit(const float* Y, int64_t ldy, int64_t rows, const float* colscale, void* Yh,
                    void* stream);
int dsvgd_h2_rowsplit(const float* A, int64_t lda, int64_t rows, int64_t cols, int64_t rows_pad,
                      int64_t kpad, const float* tscale, void* img, void* stream);
/* the same image with one scale per row: rowscale[i] * A[row i] (rows < rows) */
int dsvgd_h2_rowsplit_rows(const float* A, int64_t lda, int64_t rows, int64_t cols,
                           int64_t rows_pad, int64_t kpad, const float* rowscale, void* img,
                           void* stream);
/* rows [row_begin, row_begin + nrows) of dsvgd_h2_rowsplit_rows's image only
 * (the same arguments; ABI 4: the wide Gauss-Seidel sweep re-splits the rows a
 * block moved). */
int dsvgd_h2_rowsplit_rows_range(const float* A, int64_t lda, int64_t rows, int64_t cols,
                                 int64_t rows_pad, int64_t kpad, const float* rscale, void* img,
                                 int64_t row_begin, int64_t nrows, void* stream);
/* rowscale[i] = the FmtH2 power-of-two scale of row i of A (rows x cols) and
 * rowinv[i] = 1 / rowscale[i] (nullable), for i < rows_pad (1 past rows) */
int dsvgd_h2_rowscale(const float* A, int64_t lda, int64_t rows, int64_t cols, int64_t rows_pad,
                      float* rowscale, float* rowinv, void* stream);
/* dsvgd_h2_rowscale (rowinv required) and dsvgd_h2_rowsplit_rows with those
 * scales in one pass over A: the same bits (round 5; the logreg W image) */
int dsvgd_h2_rowimage(const float* A, int64_t lda, int64_t rows, int64_t cols, int64_t rows_pad,
                      int64_t kpad, float* rowscale, float* rowinv, void* img, void* stream);
/* dsvgd_sqdist_x3 on the FmtH2 engine: Yg = dsvgd_h2_rowsplit_rows(Y, ldy,
 * n_pad, dp, n_pad + 256, dp, rowscale) with the per-row scales of Y's X half
 * (dsvgd_pack_h2's rowscale, or dsvgd_h2_rowscale; >= n_pad floats); same
 * outputs, select modes and layouts. */
int dsvgd_sqdist_h2(const void* Yg, const float* norms, int64_t row0, int64_t m, int64_t n,
                    int64_t d, float* D, int64_t ldd, int select_mode, dsvgd_select_state* st,
                    float* cand, int layout, const float* rowscale, void* stream);
/* ---- the reference's Gauss-Seidel order for 64 < d <= 1024 (ABI 4) -----
 * dsvgd/sampler.py:64-68 / distsampler.py:194-200 move row i with phi_i of the
 * CURRENT particles.  The wide blocked sweep takes B = dsvgd_gsw_block_rows(d, kind)
 * rows at a time: their interactions with every row not moved before them in
 * the block on the f32 engines (dsvgd_sqdist of the centred Y = [X - c | S]
 * rows [r0, r0 + B); dsvgd_gs_mask: D[i][r0 + j] = +inf for j < i, the pairs
 * the walk takes; dsvgd_phi_mm into split-K slices; dsvgd_phi_partial_reduce
 * -> Q = [K Xc | K S], Qr = K 1), then dsvgd_gsw_block_sweep walks the B rows
 * in order in one workgroup: phi_i = (Q_i + s_i + sum_{j<i} k(x_i, x_j')
 * (s_j' + (2/h)(x_i - x_j'))) / n (+ extra), X[i] += step phi_i, the score
 * refreshed (score_kind as dsvgd_gs_block_sweep, or 3: the logistic
 * regression score of logreg_small_kernel on nd data rows xd (ld ldxd, d - 1
 * features) with labels td, times score_scale -- experiments/logreg.py:45-58
 * re-run per pair by distsampler.py:97-99), Y's row and norms[] kept current
 * (centre c = center, the packing centre of Y).  Any d <= 1024 for kind 3. */
int64_t dsvgd_gsw_block_rows(int64_t d, int score_kind);  /* 0 if d > 1024 */
/* The walk's form for score_kind 0 .. 2 (A/B switch, returns the previous
 * setting): 1 (default) = the incremental walk (each moved row's pair terms
 * added to every later row of the block at once, two barriers per row,
 * nothing per row on the path but the row's own phi) for roundup(d, 32) <=
 * 1024 -- 1, 2 or 4 columns per thread up to 256, 512, 1024, blocks of at
 * most 64, 32, 16 rows (B <= 64 / columns per thread), about 132 KB of LDS
 * at every shape; 0 = the four-wave walk (distances and the column loop per
 * row).  Where the incremental walk's LDS cannot be reserved the call runs
 * the four-wave walk (no error). */
int dsvgd_gsw_set_inc(int on);
/* Timing probe of the walk (scripts/walk_probe.py; results are garbage while
 * set): bit 0 skips the next row's operand loads, bit 1 the distances, bit 2
 * the column loop.  Process-wide; returns the previous mask.  0 = normal. */
int dsvgd_gsw_debug(int mask);
int dsvgd_gs_mask(float* D, int64_t ldd, int64_t r0, int64_t B, void* stream);
/* D[i][c0 + j] = +inf for i < B (<= 1024), j < nc (panel layout): the
 * pipelined wide sweep (round 6) leaves the group walking beside a wide pass
 * out of that pass; dsvgd_gsw_group_corr adds its rows at their moved
 * positions afterwards. */
int dsvgd_gs_mask_cols(float* D, int64_t ldd, int64_t B, int64_t c0, int64_t nc, void* stream);
/* Test hook: one wave holds `stream` for ns nanoseconds (the pipelined
 * sweep's forced-overlap test). */
int dsvgd_debug_spin(int64_t ns, void* stream);
/* The grouped wide sweep (round 5): one wide pass for a group of blocks
 * (dsvgd_gs_mask over the whole group, B <= 1024), then after each block's
 * walk the group's later rows [r0, r0 + nr) gain that block's moved rows
 * [p0, p0 + pB): Q += k_ij (x_j' - c | s_j'), Qr += k_ij by explicit
 * differences, j in order (Q, Qr: the later rows' first entries).  pB <= 128
 * (round 6: a whole 128-row group in one launch, the pipelined sweep's
 * correction for the group walked beside its pass). */
int dsvgd_gsw_group_corr(const float* X, int64_t ldx, const float* S, int64_t lds,
                         const float* center, int64_t n, int64_t d, int64_t r0, int64_t nr,
                         int64_t p0, int64_t pB, const dsvgd_select_state* st, float* Q,
                         int64_t ldq, float* Qr, void* stream);
int dsvgd_gsw_block_sweep(float* X, int64_t ldx, float* S, int64_t lds, float* Y, int64_t ldy,
                          float* norms, const float* center, int64_t n, int64_t d, int64_t r0,
                          int64_t B, const dsvgd_select_state* st, float step, const float* Q,
                          int64_t ldq, const float* Qr, const float* extra, int64_t lde,
                          float* phi_out, int64_t ldphi, int score_kind, const float* mu,
                          const float* lam, float score_scale, const float* xd, int64_t ldxd,
                          const float* td, int64_t nd, void* stream);

/* ---- the pair-split layout of a DistSampler rank (ABI 4) ---
 * With the scores identical on every rank (all_scores, or replicated data),
 * the S ranks split the symmetric n x n matrix by BLOCK PAIRS: rank r
 * computes its diagonal square, the forward blocks (r, r+1) .. (r, r+S/2-1)
 * (mod S) and half of the antipodal pair {(r, r+S/2), (r+S/2, r)}; for each
 * block (r, c) it holds it sends the owner of c the partial K(r,c)^T Y_r
 * (dsvgd_phi_h2_transposed), and sums the partials it receives into its own
 * phi (dsvgd_phi_finish_parts).  Replaces the interaction loop of
 * dsvgd/distsampler.py:84-101 over the all-gathered particles (:152-170).
 *
 * dsvgd_sqdist_h2_parts: dsvgd_sqdist_h2 over a list of parts of the owned
 * row block [row0, row0 + m) (host array).  kind 0: a rectangle (rows
 * [row_off, +rows) of the block x global columns [col0, +cols)) whose
 * entries count twice in the median select when weight2 (the rank holds the
 * pair for both owners); kind 1: the block's diagonal square (row_off = 0,
 * rows = cols = m, col0 = row0; upper tiles + mirror stores); kind 2: a
 * rectangle computed only while *gate != 0 (the FmtH2 range guard: the
 * fallback phi_mm reads the whole row block), without select accounting.
 * select_mode 0 or 2 (bracket); dp % 256 == 0; row0, m multiples of 256;
 * col0, cols multiples of 256, row_off, rows of 128. */
typedef struct dsvgd_gram_part {
  int64_t row_off, rows, col0, cols;
  int32_t kind, weight2;
} dsvgd_gram_part;
int dsvgd_sqdist_h2_parts(const void* Yg, const float* norms, int64_t row0, int64_t m, int64_t n,
                          int64_t d, float* D, int64_t ldd, int select_mode,
                          dsvgd_select_state* st, float* cand, const dsvgd_gram_part* parts,
                          int nparts, const float* gate, const float* rowscale, void* stream);
/* dsvgd_radix_hist with a tile weight map instead of the symmetric rule:
 * the panel of D tile (I, J) (128 x 128, panel layout, m_pad x n_pad) counts
 * wmap[I * (n_pad / 128) + J] times (0: not an entry of this rank's share). */
int dsvgd_radix_hist_wmap(const float* D, int64_t m_pad, int64_t n_pad, const float* cand,
                          int pass, dsvgd_select_state* st, const uint8_t* wmap, void* stream);
/* phi_mm (FmtH2) of rows [row0, row0 + m) of the interacting set (D: their
 * panel rows) over a CYCLIC window of columns [col0, col0 + wlen) mod
 * n_pad, into `splits` split-K slices (KY + z m ldk, rowsum + z
 * roundup(m,128)); the diagonal j == row0 + i skipped as in dsvgd_phi_mm.
 * col0, wlen multiples of 16.  gate / gate_on as dsvgd_phi_mm_h2 (run iff
 * (*gate != 0) == gate_on). */
int dsvgd_phi_h2_window(const float* D, int64_t ldd, const void* Yh, int64_t ldy, int64_t row0,
                        int64_t m, int64_t n, int64_t col0, int64_t wlen,
                        const dsvgd_select_state* st, int64_t splits, float* KY, int64_t ldk,
                        float* rowsum, const float* colinv, const float* gate, int gate_on,
                        void* stream);
/* The transposed partial of a rectangle of D: D points at the rectangle's
 * first row (a 128-row panel row; its rows are interacting-set rows yrow0 ..
 * yrow0 + krows - 1), its columns [col0, col0 + mo) (col0 a multiple of
 * 128).  P_z[i][:] = sum_{j in slice z} exp(-D[j][col0 + i]/h) Y[yrow0 + j][:]
 * and rs_z[i] the same sum of the weights, for i < mo (KY layout: P + z mo
 * ldp, rs + z roundup(mo,128)).  krows a multiple of 16. */
int dsvgd_phi_h2_transposed(const float* D, int64_t ldd, const void* Yh, int64_t ldy,
                            int64_t yrow0, int64_t krows, int64_t col0, int64_t mo, int64_t n,
                            const dsvgd_select_state* st, int64_t splits, float* P, int64_t ldp,
                            float* rs, const float* colinv, const float* gate, int gate_on,
                            void* stream);
/* dsvgd_phi_h2_transposed for `count` whole m x m blocks of the owned rows'
 * D in one launch, no split-K: block q (< count) is D's column block (first +
 * q) mod nblocks (the forward blocks of a rank), its partial [m x ldp | m row
 * sums] written at P + q pstride. */
int dsvgd_phi_h2_transposed_blocks(const float* D, int64_t ldd, const void* Yh, int64_t ldy,
                                   int64_t yrow0, int64_t m, int64_t first, int64_t nblocks,
                                   int64_t count, int64_t n, const dsvgd_select_state* st,
                                   float* P, int64_t ldp, int64_t pstride, const float* colinv,
                                   const float* gate, int gate_on, void* stream);
/* dsvgd_phi_h2_transposed_blocks with each block's K range (its m rows of D)
 * split into zsplit slices (m a multiple of 16 zsplit), so that count x
 * m/128 x zsplit workgroups fill the CUs: slice z of block q written at
 * P + (z count + q) pstride (dsvgd_phi_partial_reduce_blocks sums them). */
int dsvgd_phi_h2_transposed_blocks_split(const float* D, int64_t ldd, const void* Yh, int64_t ldy,
                                         int64_t yrow0, int64_t m, int64_t first, int64_t nblocks,
                                         int64_t count, int64_t zsplit, int64_t n,
                                         const dsvgd_select_state* st, float* P, int64_t ldp,
                                         int64_t pstride, const float* colinv, const float* gate,
                                         int gate_on, void* stream);
/* For q < count: out + q ostride = sum over z < zsplit (in slice order) of
 * the [rows x ldp | row sums] partial at P + (z count + q) pstride (row sums
 * at + rows ldp in, + rows ldo out) -- the split forward blocks' messages. */
int dsvgd_phi_partial_reduce_blocks(const float* P, int64_t ldp, int64_t pstride, int64_t zsplit,
                                    int64_t count, int64_t rows, int64_t cols, float* out,
                                    int64_t ldo, int64_t ostride, void* stream);
/* out[i][c] = sum_z P[z][i][c] (c < cols) and out_rs[i] = sum_z rs[z][i], in
 * slice order (the P / rs layout of dsvgd_phi_h2_transposed). */
int dsvgd_phi_partial_reduce(const float* P, int64_t ldp, const float* rs, int64_t splits,
                             int64_t rows, int64_t cols, float* out, int64_t ldo, float* out_rs,
                             void* stream);
/* dsvgd_phi_finish over the own split-K slices plus `nparts` partials, each
 * adding ky[z][i - row_off][:] and rs[z][i - row_off] (z < splits) to rows
 * row_off <= i < row_off + rows, summed in list order after the own slices.
 * gate (nullable): while *gate != 0 the parts are skipped and the own slices
 * are `splits_fb` (the range guard's whole-row-block fallback). */
typedef struct dsvgd_phi_part {
  const float* ky;
  const float* rs;
  int64_t ldk, row_off, rows, splits;
} dsvgd_phi_part;
int dsvgd_phi_finish_parts(const float* KY, int64_t ldk, const float* rowsum, int64_t splits,
                           const float* Y, int64_t ldy, int64_t row0, int64_t m, int64_t d,
                           int64_t dp, const dsvgd_select_state* st, float inv_n, float step,
                           const float* extra, int64_t lde, float* phi, int64_t ldphi, float* X,
                           int64_t ldx, const dsvgd_phi_part* parts, int nparts,
                           const float* gate, int64_t splits_fb, void* stream);

/* dsvgd_phi_mm_x3 on the FmtH2 engine: Yh = dsvgd_h2_ysplit(Y, ldy, n_pad,
 * scale) and colinv = &scale[ldy] of a dsvgd_h2_colscale over all ldy
 * columns of Y; same outputs (unscaled), split-K slices, diagonal rule and
 * symmetric layout (sym needs ldy % 256 == 0).  Requires n_pad * ldy * 4 <
 * 2^31.  gate (nullable, &scale[2 ldy + 2]): does nothing while it reads
 * nonzero (the range guard hands the step to dsvgd_phi_mm_x3, or to
 * dsvgd_phi_mm_gated where no FmtX3 image fits). */
int dsvgd_phi_mm_h2(const float* D, int64_t ldd, const void* Yh, int64_t ldy, int64_t row0,
                    int64_t m, int64_t n, const dsvgd_select_state* st, int64_t splits, float* KY,
                    int64_t ldk, float* rowsum, int sym, const float* colinv, const float* gate,
                    void* stream);

/* phi[i] = inv_n * (s_i + KS[i] + (2/h) (rowsum[i] xc[i] - KXc[i])) with the
 * split-K partials summed in slice order (s_i: the self term k_ii s_i), plus
 * extra[i] if extra != NULL (the h * W2-gradient row of dsvgd_w2_grad:
 * delta = phi_hat + h W, dsvgd/distsampler.py:194-198), and, if X != NULL,
 * X[i] += step * phi[i] (the update of dsvgd/sampler.py:68 /
 * dsvgd/distsampler.py:200, Jacobi order).  phi and extra may be NULL. */
int dsvgd_phi_finish(const float* KY, int64_t ldk, const float* rowsum, int64_t splits,
                     const float* Y, int64_t ldy, int64_t row0, int64_t m, int64_t d, int64_t dp,
                     const dsvgd_select_state* st, float inv_n, float step, const float* extra,
                     int64_t lde, float* phi, int64_t ldphi, float* X, int64_t ldx,
                     void* stream);
/* Process-wide A/B switch (default 1): dsvgd_phi_finish takes four columns
 * per thread (16-byte accesses) when d, dp and every leading dimension are
 * multiples of 4 and every base is 16-byte aligned; 0 keeps one element per
 * thread.  Same bits.  Returns the previous setting. */
int dsvgd_phi_set_finish_vec(int on);

/* d <= 64 (used for d <= 2): phi (and the optional X update) straight from the pairwise form
 * phi_i = inv_n sum_j k_ij (s_j + (2/h)(x_i - x_j)) on the VALU -- the
 * reference's own per-pair expression (dsvgd/sampler.py:38-40), which avoids
 * the r x - K X cancellation of the GEMM form at small d.  Replaces
 * dsvgd_phi_mm + dsvgd_phi_finish for small d (extra as in dsvgd_phi_finish).
 * partial (nullable, partial_floats long): scratch for split-J partial sums
 * (up to partial_floats / (m d) slices, summed in order by a second kernel),
 * which keeps the chip busy when m is small. */
int dsvgd_phi_direct(const float* D, int64_t ldd, const float* Y, int64_t ldy, int64_t row0,
                     int64_t m, int64_t n, int64_t d, const dsvgd_select_state* st, float inv_n,
                     float step, const float* extra, int64_t lde, float* phi, int64_t ldphi,
                     float* X, int64_t ldx, float* partial, int64_t partial_floats,
                     void* stream);

/* Gauss-Seidel single-row update (reference order): for particle i, phi_i
 * from exact differences against the CURRENT X (rows < i already moved),
 * X[i] += step * phi_i.  Reproduces dsvgd/sampler.py:64-68 and
 * dsvgd/distsampler.py:194-200 one row at a time.  n_int interacting rows
 * start at X (row i is X + i*ldx).  extra (nullable, d floats) is added to
 * phi_i before the step (the row's h * W2 gradient, distsampler.py:196-198). */
int dsvgd_phi_row(float* X, int64_t ldx, const float* S, int64_t lds, int64_t n_int, int64_t d,
                  int64_t i, const dsvgd_select_state* st, float step, const float* extra,
                  float* phi_out, void* stream);
/* The same row update with the j range split over `blocks` workgroups (two
 * launches; partial: blocks x d floats of scratch), for large n_int.
 * dsvgd_phi_row_blocks(n, d) = the split to use (1: call dsvgd_phi_row). */
int64_t dsvgd_phi_row_blocks(int64_t n, int64_t d);
int dsvgd_phi_row_split(float* X, int64_t ldx, const float* S, int64_t lds, int64_t n, int64_t d,
                        int64_t i, const dsvgd_select_state* st, float step, const float* extra,
                        float* phi_out, float* partial, int64_t blocks, void* stream);

/* Blocked Gauss-Seidel sweep (the same reference order, d <= 64): rows
 * [r0, r0 + B), B <= dsvgd_gs_block_rows() = 64, of the interacting set X
 * (n x d).  gs_block_part: Q[i][c] = the raw sum over every j outside
 * [r0, r0 + i) of k(x_i, x_j) (s_j + (2/h)(x_i - x_j)) as the block starts,
 * computed as nsplit = dsvgd_gs_splits(n) j slices (partial: nsplit x B x d
 * floats of scratch) and summed in slice order (into partial[0 .. B d) when
 * B d nsplit > 16384, else by the sweep);
 * gs_block_sweep then walks the block in order in one wave: phi_i = (Q_i +
 * the terms of the block rows already moved, at their new positions) / n
 * [+ extra row i], X[r0+i] += step phi_i, and the moved particle's score
 * refreshed in S (score_kind 1: scale * (-lam (x - mu)), 2: the
 * experiments/gmm.py mixture per coordinate; 0: S left as is -- exchanged
 * scores are frozen for the step, distsampler.py:194-200).  Two or three launches
 * per 64 rows instead of two per row (dsvgd_phi_row_split).  nsplit, B, d of
 * the sweep: those of the gs_block_part call. */
int64_t dsvgd_gs_block_rows(void);
int64_t dsvgd_gs_splits(int64_t n);
int dsvgd_gs_block_part(const float* X, int64_t ldx, const float* S, int64_t lds, int64_t n,
                        int64_t d, int64_t r0, int64_t B, const dsvgd_select_state* st,
                        float* partial, int64_t nsplit, void* stream);
int dsvgd_gs_block_sweep(float* X, int64_t ldx, float* S, int64_t lds, int64_t n, int64_t d,
                         int64_t r0, int64_t B, const dsvgd_select_state* st, float step,
                         const float* partial, int64_t nsplit, const float* extra, int64_t lde,
                         float* phi_out, int64_t ldphi, int score_kind, const float* mu,
                         const float* lam, float score_scale, void* stream);

/* ---- W2 / JKO term (dsvgd/distsampler.py:103-129, used at :190-198) ---- */
/* The reference LP  min <P,C>, P >= 0, row sums 1/m, column sums 1/n  over
 * C_ij = ||x_i - y_j||^2 (x: m owned particles, y: n previous particles) has
 * an integral optimum when n = R m: an assignment of n slots (slot s belongs
 * to row s / R) to the n columns, each of mass 1/n.
 *
 * C[i][j] (m x n, ldc >= n) from explicit fp32 differences
 * (distsampler.py:107-114). */
int dsvgd_w2_cost(const float* X, int64_t ldx, int64_t m, const float* Y, int64_t ldy, int64_t n,
                  int64_t d, float* C, int64_t ldc, void* stream);
/* The same C on the FmtH2 split-role Gram (ABI 4, round 6): C_ij = |x_i -
 * c|^2 + |y_j - c|^2 - 2 (x_i - c).(y_j - c) (c: Y's robust centre,
 * dsvgd_colcenter) on the fp16 MFMAs, fp32-accurate per the FmtH2 bound
 * (|error| ~ 2^-21 (|x_i - c|^2 + |y_j - c|^2)), and every entry below
 * tau (|x_i - c|^2 + |y_j - c|^2) -- where that form cancels, e.g. a particle
 * and its own previous position -- recomputed from explicit fp32
 * differences in dsvgd_w2_cost's order (the same bits).  C needs
 * roundup(m, 128) rows and ldc >= roundup(n, 256) (16-byte aligned rows;
 * the padding is written); ws: dsvgd_w2_cost_h2_workspace_bytes, 256-byte
 * aligned.  d <= 1024.  cstat (NULL, or 2 device words): the largest entry
 * of C (float bits) and a non-finite flag, taken while C is written --
 * dsvgd_w2_assign_stat then skips its pass over C for them. */
/* A/B switch of dsvgd_w2_cost_h2's C stores (returns the previous): 1
 * (default) non-temporal, 0 the default cache policy. */
int dsvgd_w2_set_cost_nt(int on);

/* Process-wide A/B switch (default 1): dsvgd_w2_cost_h2 writes C in whole
 * 128-byte row lines (two slices' values traded between lane pairs); 0 writes
 * each slice's half lines as it goes.  Same C bits.  Returns the previous
 * setting. */
int dsvgd_w2_set_cost_lines(int on);
size_t dsvgd_w2_cost_h2_workspace_bytes(int64_t m, int64_t n, int64_t d);
int dsvgd_w2_cost_h2(const float* X, int64_t ldx, int64_t m, const float* Y, int64_t ldy,
                     int64_t n, int64_t d, float* C, int64_t ldc, void* ws, float tau,
                     uint32_t* cstat, void* stream);
/* Device workspace of dsvgd_w2_assign (32 n + 256 bytes). */
size_t dsvgd_w2_workspace_bytes(int64_t m, int64_t n);
/* assign[s] = column of slot s in an optimal plan (replaces scipy linprog,
 * distsampler.py:115-126): epsilon-scaling auction on the GPU, final
 * eps = max C * 2^-24 / n (within one fp32 ulp of max C of the optimum).
 * BLOCKS the calling thread (polls the device between batches of rounds);
 * fails with -3 after max_rounds.  rounds_out (host, nullable) gets the
 * number of bidding rounds.  warm_phases > 0: keep the prices left in `ws`
 * by the previous call on a nearby problem (SVGD's next step) and start
 * warm_phases epsilon phases above the final eps; 0: cold start. */
int dsvgd_w2_assign(const float* C, int64_t ldc, int64_t m, int64_t n, void* ws,
                    int64_t max_rounds, int warm_phases, int32_t* assign, int64_t* rounds_out,
                    void* stream);
/* dsvgd_w2_assign warm-started from the previous call on this workspace
 * (its prices) and that call's plan prev_assign (n slots): the first epsilon
 * is the previous plan's complementary-slackness violation under the new
 * costs / 64 (so a small SVGD step starts near eps_final, a large one high),
 * then the usual phases down to eps_final -- same optimality guarantee. */
int dsvgd_w2_assign_warm(const float* C, int64_t ldc, int64_t m, int64_t n, void* ws,
                         int64_t max_rounds, const int32_t* prev_assign, int32_t* assign,
                         int64_t* rounds_out, void* stream);
/* dsvgd_w2_assign (prev_assign NULL, warm_phases as there) or
 * dsvgd_w2_assign_warm (prev_assign set) with C's largest entry and
 * finiteness taken from cstat (dsvgd_w2_cost_h2's) instead of a pass over C
 * (round 6).  The same plan. */
int dsvgd_w2_assign_stat(const float* C, int64_t ldc, int64_t m, int64_t n, void* ws,
                         int64_t max_rounds, int warm_phases, const int32_t* prev_assign,
                         int32_t* assign, int64_t* rounds_out, const uint32_t* cstat,
                         void* stream);
/* Process-wide switch of the auction's phase keep (default 0): a new
 * epsilon phase, and dsvgd_w2_assign_warm's first phase with the previous
 * plan, keep every slot whose column still meets epsilon-complementary
 * slackness; 0 re-assigns every slot each phase.  Same optimality guarantee
 * either way.  Returns the previous setting. */
int dsvgd_w2_set_keep(int keep);
/* Process-wide epsilon divisor between the auction's phases (default 8;
 * accepted in [2, 1024], otherwise ignored).  Returns the previous value. */
double dsvgd_w2_set_theta(double theta);
/* The last dsvgd_w2_assign's phase tails on this host thread: out[0] bids,
 * out[1] full row scans among them, out[2..4] microseconds spent in the
 * cached bids, the scans (with their cache refill) and the resolves, out[5]
 * tails whose scan helpers did not answer in time (the solve then finishes
 * on the bid rounds, same plan) -- as of the last control readback.
 * Returns 6 (the length of out). */
int64_t dsvgd_w2_tail_stats(int64_t* out);
/* Process-wide test switch (default 0): the phase tail's scan helpers exit
 * at once, so every tail stalls and hands its phase back to the bid rounds.
 * Returns the previous setting. */
int dsvgd_w2_set_tail_debug(int nohelp);

/* Process-wide switch (default 1): an R = 1 warm start (prev_assign given,
 * keep off) takes the violation and its first round's row scans (best value,
 * its column, second value) in one pass over C, and the first round bids from
 * them; 0 runs the violation pass and a full-scan bid round (same bids, same
 * plan; A/B).  Returns the previous setting. */
int dsvgd_w2_set_fuse_first(int on);
/* Progress of this host thread's last dsvgd_w2_assign: out[3k..3k+2] =
 * (rounds, epsilon phase, unassigned slots) at the k-th control readback
 * (every 16 rounds); copies min(count, cap) triples, returns count. */
int64_t dsvgd_w2_trace(int64_t* out, int64_t cap);
/* G[i] = h * sum_j P_ij (x_i - y_j) = h/n * sum_{slots s of i} (x_i - y_assign[s])
 * (distsampler.py:128 scaled by the JKO step h of :198); pass G as `extra`
 * to dsvgd_phi_finish / dsvgd_phi_direct / dsvgd_phi_row. */
int dsvgd_w2_grad(const float* X, int64_t ldx, int64_t m, const float* Y, int64_t ldy, int64_t n,
                  int64_t d, const int32_t* assign, float h, float* G, int64_t ldg, void* stream);

/* ---- target scores grad log p (replace the autograd _dlogp calls) ------ */
/* S = scale * (-lam * (X - mu))      (synthetic Gaussian target)            */
int dsvgd_score_gaussian(const float* X, int64_t ldx, int64_t n, int64_t d, const float* mu,
                         const float* lam, float scale, float* S, int64_t lds, void* stream);
/* S = scale * d/dx log(1/3 N(x;-2,1) + 1/3 N(x;2,1)), elementwise
 * (experiments/gmm.py:16-21) */
int dsvgd_score_gmm(const float* X, int64_t ldx, int64_t n, int64_t d, float scale, float* S,
                    int64_t lds, void* stream);
/* Bayesian logistic regression (experiments/logreg.py:45-58), x = [log a, w]:
 *   s_0 = scale*(-a + p/2 - a/2 |w|^2),  s_w = scale*(-a w + Xd^T (t * sigma(-t * Xd w)))
 * as two MFMA GEMMs (Z = W Xd^T with the sigmoid epilogue, G Xd); for
 * n <= 32 particles and N <= 8192 rows (the Gauss-Seidel order's
 * one-particle refresh) a single one-block-per-particle launch instead.
 * Xd: N x p data rows (ldxd), t: N labels (+-1).  Workspace:
 * dsvgd_logreg_workspace_bytes(n, N, p) (unused on the small path). */
/* The FmtH2 logistic-regression score as one fused kernel (1, default: Z,
 * sigma and G . Xd with G kept in registers; 224 < p <= 256 weights, the
 * bench's p = 255) or the two-GEMM path (0).  A/B switch; returns the previous
 * setting.  The prepared workspace holds both paths' data images. */
int dsvgd_logreg_set_fused(int on);
size_t dsvgd_logreg_workspace_bytes(int64_t n, int64_t N, int64_t p);
int dsvgd_score_logreg(const float* X, int64_t ldx, int64_t n, int64_t d, const float* Xd,
                       int64_t ldxd, const float* t, int64_t N, float scale, float* S, int64_t lds,
                       void* workspace, void* stream);
/* the same on a chosen GEMM engine: 0 = FmtH2 (what dsvgd_score_logreg
 * runs), 1 = FmtX3, 2 = the exact f32 MFMA engines (precision reference) */
int dsvgd_score_logreg_engine(const float* X, int64_t ldx, int64_t n, int64_t d, const float* Xd,
                              int64_t ldxd, const float* t, int64_t N, float scale, float* S,
                              int64_t lds, void* workspace, int engine, void* stream);
/* ... as two calls, for a data set scored at many particle sets (every SVGD
 * step): logreg_prepare writes the data-only part of the workspace (padded
 * Xd and t, Xd's FmtH2 scales and split images) once; score_logreg_prepared
 * then reads it every step (same n, N, d, engine and workspace).  Not for
 * the n <= 32 one-block path (EINVAL there: use dsvgd_score_logreg_engine). */
int dsvgd_logreg_prepare(const float* Xd, int64_t ldxd, const float* t, int64_t N, int64_t n,
                         int64_t d, void* workspace, int engine, void* stream);
int dsvgd_score_logreg_prepared(const float* X, int64_t ldx, int64_t n, int64_t d, int64_t N,
                                float scale, float* S, int64_t lds, void* workspace, int engine,
                                void* stream);

/* dsvgd_score_logreg_prepared with the prior weighted by prior_weight:
 * S = scale * (sum over the data - prior_weight * grad of the prior terms).
 * DistSampler's gathered-data all_scores mode scores its own particles over
 * every rank's data with prior_weight = S, which is what the reference's
 * all-reduce of S per-rank logp gradients sums to (distsampler.py:160-170:
 * each rank's logp carries the prior once).  prior_weight = 1 gives exactly
 * dsvgd_score_logreg_prepared's bits.  Replaces: the same call sites. */
int dsvgd_score_logreg_prior(const float* X, int64_t ldx, int64_t n, int64_t d, int64_t N,
                             float scale, float prior_weight, float* S, int64_t lds,
                             void* workspace, int engine, void* stream);

/* Posterior-predictive probability of the logistic-regression test set:
 * prob[q] = (1/n) sum_j sigma(xt_q . w_j), w_j = X[j][1:d] (no bias; alpha
 * unused) -- the ensemble mean of experiments/logreg_plots.py:42-50
 * (`_test_acc`), which the caller thresholds (prob > 0.5 vs t > 0) for the
 * test accuracy.  fp32 (the reference evaluates it in fp64 with numpy).
 * Xt: Nt x (d-1) row-major; workspace of
 * dsvgd_logreg_predict_workspace_bytes(n, Nt, d-1) bytes, 256-B aligned. */
size_t dsvgd_logreg_predict_workspace_bytes(int64_t n, int64_t Nt, int64_t p);
int dsvgd_logreg_predict(const float* X, int64_t ldx, int64_t n, int64_t d, const float* Xt,
                         int64_t ldxt, int64_t Nt, float* prob, void* workspace, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DSVGD_H_ */
