"""Barrier timeline of the split-role Gram (dsvgd_gram_set_rs(8): each wave
of blocks 0-7 stamps the shader clock arriving at / leaving every barrier).
Per role, the median over blocks / waves / units of: the K-step period (one
barrier release to the next), the wait at a K-step barrier, and the same at
the tile hand-off (X, Y).  S = 1 headline Gram, bracketed median.

    python scripts/gram_stamps.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dist-svgd_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import dsvgd
    from dsvgd import _native as N
    lib = N.load()
    n, d = 65536, 256
    g = torch.Generator(device="cpu").manual_seed(0)
    X = (0.1 * torch.randn(n, d, generator=g)).cuda()
    eng = dsvgd.PhiEngine(n, d, device="cuda:0")
    eng.pack(X)
    buf = torch.zeros(8 * 8 * 512, dtype=torch.int64, device="cuda:0")
    lib.dsvgd_gram_debug_stamps(N.ptr(buf))
    prev = lib.dsvgd_gram_set_rs(1)
    eng.distances(median=True)          # warm: the bracket sample, the state
    eng.median_bandwidth()
    lib.dsvgd_gram_set_rs(8)
    eng.distances(median=True)
    torch.cuda.synchronize()
    lib.dsvgd_gram_set_rs(prev)
    lib.dsvgd_gram_debug_stamps(None)
    t = buf.view(8, 8, 512).cpu().numpy().astype(np.int64)
    # per wave: stamps come in (arrive, leave) pairs; the M waves' first
    # barrier is the prologue, then 16 K-step barriers + X + Y per tile; the
    # E waves' first barrier is the same prologue one, then the same 18
    out = {}
    for role, waves in (("M", range(0, 4)), ("E", range(4, 8))):
        per, waitk, waitx, waity, tile = [], [], [], [], []
        for b in range(8):
            for w in waves:
                s = t[b, w]
                nz = int(np.count_nonzero(s))
                pairs = s[:nz - nz % 2].reshape(-1, 2)
                arr, lev = pairs[:, 0], pairs[:, 1]
                body = range(1, len(pairs) - 18, 18)     # tiles after the prologue barrier
                for u0 in body:
                    ks = list(range(u0, u0 + 16))
                    per += list(np.diff(lev[ks]))
                    waitk += list(lev[ks] - arr[ks])
                    waitx.append(lev[u0 + 16] - arr[u0 + 16])
                    waity.append(lev[u0 + 17] - arr[u0 + 17])
                    tile.append(lev[u0 + 18] - lev[u0] if u0 + 18 < len(lev) else 0)
        # per barrier index of a tile (B_0 .. B_15, X, Y): the median time from
        # the previous barrier's release to this one's release, and the wait
        seg = [[] for _ in range(18)]
        wt = [[] for _ in range(18)]
        for b in range(8):
            for w in waves:
                s = t[b, w]
                nz = int(np.count_nonzero(s))
                pairs = s[:nz - nz % 2].reshape(-1, 2)
                arr, lev = pairs[:, 0], pairs[:, 1]
                for u0 in range(1, len(pairs) - 18, 18):
                    for i in range(18):
                        seg[i].append(lev[u0 + i] - lev[u0 + i - 1])
                        wt[i].append(lev[u0 + i] - arr[u0 + i])
        med = lambda v: float(np.median(v)) if len(v) else None  # noqa: E731
        out[role + "_by_barrier"] = {"names": ["B%d" % i for i in range(16)] + ["X", "Y"],
                                     "segment_median": [med(v) for v in seg],
                                     "segment_mean": [float(np.mean(v)) if v else None for v in seg],
                                     "wait_median": [med(v) for v in wt],
                                     "wait_mean": [float(np.mean(v)) if v else None for v in wt]}
        out[role] = {"kstep_period": med(per), "kstep_wait": med(waitk),
                     "kstep_wait_p90": float(np.percentile(waitk, 90)) if waitk else None,
                     "x_wait": med(waitx), "y_wait": med(waity),
                     "tile_period": med([v for v in tile if v > 0]), "tiles": len(waitx)}
    out["unit"] = "s_memtime ticks (the shader clock)"
    print(json.dumps(out))


if __name__ == "__main__":
    main()
