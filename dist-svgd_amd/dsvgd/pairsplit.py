"""The pair-split layout of a DistSampler rank: which parts of
the n x n distance / kernel matrix rank r computes, what it sends, what it
receives.

Reference semantics being sharded: every rank moves its own particles with
phi over ALL n interacting particles (dsvgd/distsampler.py:84-101, after the
all-gather of :152-158 and, for all_scores, the all-reduce of :160-170).
The matrix is symmetric, so when every rank holds the same scores (all_scores,
or replicated data) each off-diagonal block pair {(r, c), (c, r)} needs to be
computed once, by one of its two owners:

  * rank r computes its diagonal square (r, r), the S/2 - 1 FORWARD blocks
    (r, r+1) .. (r, r+S/2-1) (mod S) -- (S-1)/2 of them for odd S -- and, for
    even S, half of the antipodal pair {(r, a), (a, r)}, a = r + S/2: a rank
    r < S/2 ("low") the column half (r, a_lo), a rank r >= S/2 ("high") the
    row half (r_hi, a) -- together exactly the pair;
  * phi_r = sum_c K(r, c) Y_c: the blocks it holds give their part directly
    (one cyclic column window, plus the high rank's row half); for every
    other block it receives the partial K(c, r)^T Y_c from c's owner, who
    computes it from the same stored block read transposed;
  * the median counts forward / antipodal entries twice (each stands for
    its transpose), the diagonal square once: n^2 entries over the ranks.

Per rank at S = 8: 4 of the 8 block-equivalents of the Gram (7.5 in the
row-block layout), the same phi MFMA work, and 3-4 partials of m x ldy floats
sent and received point to point.

Pure host logic (CPU-tested: tests/test_host.py); the device work is in
dsvgd.engine.PhiEngine(pair_split=...).
"""


def _cyclic(c0, length, n):
    """[c0, c0 + length) mod n as at most two non-wrapping (start, length)."""
    c0 %= n
    if length <= 0:
        return []
    if c0 + length <= n:
        return [(c0, length)]
    return [(c0, n - c0), (0, c0 + length - n)]


class PairSplitPlan(object):
    GRAM_RECT, GRAM_DIAG, GRAM_FALLBACK = 0, 1, 2
    # the diagonal square as one full rectangle on the one-kernel Gram (both
    # triangles computed, each entry counted once) instead of its upper tiles
    # on the 8-wave kernel with mirror stores, from S = FULL_SQUARE_MIN_S
    # ranks on (round 6: Gram stage at S = 8 0.525 vs 0.615 ms, S = 4 1.125
    # vs 1.196; at S = 2 the square is half the rank's Gram and the mirror
    # kernel's half of it wins, 2.39 vs 2.66 -- profiles/r14u, r13z).
    # FULL_SQUARE: True / False forces it (A/B), None = by S.
    FULL_SQUARE = None
    FULL_SQUARE_MIN_S = 4

    @classmethod
    def full_square(cls, S):
        return cls.FULL_SQUARE if cls.FULL_SQUARE is not None else S >= cls.FULL_SQUARE_MIN_S

    @staticmethod
    def aligned(S, m):
        """Whether every part of the plan meets the kernels' alignment: the
        Gram parts' columns are 256-aligned (dsvgd_sqdist_h2_parts), and for
        even S the antipodal half-block m/2 starts or ends a Gram part, so
        m/2 must be a multiple of 256 as well (m = 256 (mod 512)
        would otherwise be rejected by the kernel mid-step)."""
        return S >= 2 and m > 0 and m % 256 == 0 and (S % 2 == 1 or m % 512 == 0)

    def __init__(self, rank, S, m):
        assert 0 <= rank < S and self.aligned(S, m), (rank, S, m)
        self.rank, self.S, self.m = rank, S, m
        n = self.n = S * m
        even = S % 2 == 0
        half = S // 2
        nf = half - 1 if even else (S - 1) // 2
        self.forward = [(rank + k) % S for k in range(1, nf + 1)]
        self.backward = [(rank - k) % S for k in range(1, nf + 1)]
        self.anti = (rank + half) % S if even else None
        self.low = even and rank < half
        self.high = even and rank >= half
        h2 = m // 2
        r0 = rank * m

        # own direct product: the diagonal square + forward blocks (+ the low
        # rank's antipodal column half), one cyclic column window
        self.window = (r0, (nf + 1) * m + (h2 if self.low else 0))
        # the high rank's row half of the antipodal pair: rows [m/2, m) x block a
        self.row_half = (h2, h2, self.anti * m, m) if self.high else None

        # Gram parts (include/dsvgd.h dsvgd_gram_part): accounted, then the
        # fallback-only complement (the range guard's whole-row-block phi)
        parts = [dict(row_off=0, rows=m, col0=r0, cols=m,
                      kind=self.GRAM_RECT if self.full_square(S) else self.GRAM_DIAG,
                      weight2=0)]
        for c0, ln in _cyclic(r0 + m, self.window[1] - m, n):
            parts.append(dict(row_off=0, rows=m, col0=c0, cols=ln, kind=self.GRAM_RECT, weight2=1))
        if self.high:
            parts.append(dict(row_off=h2, rows=h2, col0=self.anti * m, cols=m,
                              kind=self.GRAM_RECT, weight2=1))
        self.gram_parts = parts
        fb = []
        if self.high:   # rows [0, m/2) of the antipodal block, then the backward blocks
            fb.append(dict(row_off=0, rows=h2, col0=self.anti * m, cols=m,
                           kind=self.GRAM_FALLBACK, weight2=0))
            rest = (self.anti * m + m, n - self.window[1] - m)
        else:
            rest = (r0 + self.window[1], n - self.window[1])
        for c0, ln in _cyclic(rest[0], rest[1], n):
            fb.append(dict(row_off=0, rows=m, col0=c0, cols=ln, kind=self.GRAM_FALLBACK, weight2=0))
        self.fallback_parts = fb

        # partials sent: K(rows, cols)^T Y_rows of a rectangle of this rank's D
        # (row_off, krows: the rectangle's rows; col0, mo: its columns = the
        # destination's rows dst_row_off .. + mo)
        sends = [dict(dest=c, row_off=0, krows=m, col0=c * m, mo=m, dst_row_off=0)
                 for c in self.forward]
        if self.low:
            sends.append(dict(dest=self.anti, row_off=0, krows=m, col0=self.anti * m, mo=h2,
                              dst_row_off=0))
        elif self.high:
            sends.append(dict(dest=self.anti, row_off=h2, krows=h2, col0=self.anti * m, mo=m,
                              dst_row_off=0))
        self.sends = sends
        # partials received, in the order phi_finish sums them
        recvs = [dict(src=c, rows=m, row_off=0) for c in self.backward]
        if self.low:     # the high partner's row half, transposed: all m rows
            recvs.append(dict(src=self.anti, rows=m, row_off=0))
        elif self.high:  # the low partner's column half, transposed: rows [0, m/2)
            recvs.append(dict(src=self.anti, rows=h2, row_off=0))
        self.recvs = recvs

    def tile_weights(self):
        """(m/128) x (n/128) select weights of this rank's D tiles (the
        radix passes' fallback over D; dsvgd_radix_hist_wmap)."""
        m, n = self.m, self.n
        T, Tn = m // 128, n // 128
        w = [[0] * Tn for _ in range(T)]
        for p in self.gram_parts:
            wt = 1 if p["kind"] == self.GRAM_DIAG else (2 if p["weight2"] else 1)
            for I in range(p["row_off"] // 128, (p["row_off"] + p["rows"]) // 128):
                for J in range(p["col0"] // 128, (p["col0"] + p["cols"]) // 128):
                    w[I][J] = wt
        return w

    def image_rows(self):
        """The interacting-set rows whose B image (Y's FmtH2 split) the
        rank's phi products read, as sorted disjoint (start, length) ranges:
        the window's columns (its own rows among them: the transposed
        partials' B operand) and, for a high rank, the antipodal block (the
        row half's columns)."""
        spans = list(self.window_parts())
        if self.row_half:
            spans.append((self.row_half[2], self.row_half[3]))
        spans.sort()
        out = []
        for a, ln in spans:
            if out and a <= out[-1][0] + out[-1][1]:
                end = max(out[-1][0] + out[-1][1], a + ln)
                out[-1] = (out[-1][0], end - out[-1][0])
            else:
                out.append((a, ln))
        return out

    def window_parts(self):
        """The own direct product's cyclic window as non-wrapping column ranges."""
        return _cyclic(self.window[0], self.window[1], self.n)
