"""Run-to-run determinism of the direction() stages on a row-block engine
(the S = 8 rank share, DS 0) and the whole-matrix one: two direction() calls
on the same D / Y, every intermediate buffer compared (yscale, Yx, KY slices,
rowsum, phi); prints which differ and where.

    python scripts/det_probe.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dist-svgd_amd"))

import torch  # noqa: E402


def snap(eng):
    return {k: getattr(eng, k).clone() for k in ("yscale", "Yx", "KY", "rowsum", "phi", "D", "Y")}


def diff(a, b, eng):
    out = {}
    for k in a:
        x, y = a[k], b[k]
        if x.dtype != torch.float32:
            x, y = x.view(torch.int16).int(), y.view(torch.int16).int()
        ne = (x != y)
        if k in ("KY", "rowsum", "phi", "D", "Y"):
            ne = ne & ~(torch.isnan(x) & torch.isnan(y)) if x.dtype == torch.float32 else ne
        cnt = int(ne.sum())
        rec = {"n_diff": cnt, "numel": x.numel()}
        if cnt:
            idx = ne.reshape(-1).nonzero()[:8, 0].tolist()
            rec["first"] = idx
            if k == "KY":
                m, ldy = eng.m, eng.ldy
                rec["where"] = [(i // (m * ldy), (i % (m * ldy)) // ldy, i % ldy) for i in idx]
            if k == "rowsum":
                rec["where"] = [(i // eng.m_pad, i % eng.m_pad) for i in idx]
        out[k] = rec
    return out


def main():
    import dsvgd
    n, d = 65536, 256
    g = torch.Generator(device="cpu").manual_seed(0)
    X = (0.1 * torch.randn(n, d, generator=g)).cuda()
    S = torch.randn(n, d, generator=g).cuda()
    for name, kw in (("rows_S8", dict(m=n // 8, row0=n // 2)), ("rows_S8_r0", dict(m=n // 8, row0=0)),
                     ("rows_S2", dict(m=n // 2, row0=n // 2))):
        eng = dsvgd.PhiEngine(n, d, device="cuda:0", **kw)
        eng.pack(X, S)
        eng.distances(median=True)
        eng.median_bandwidth()
        eng.KY.fill_(float("nan"))
        eng.rowsum.fill_(float("nan"))
        eng.direction(write_phi=True)
        torch.cuda.synchronize()
        a = snap(eng)
        runs = []
        for _ in range(3):
            eng.direction(write_phi=True)
            torch.cuda.synchronize()
            b = snap(eng)
            runs.append(diff(a, b, eng))
        print(json.dumps({name: {"splits": eng.splits, "runs": runs}}), flush=True)
        del eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
