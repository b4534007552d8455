"""In-process A/B of dsvgd_w2_cost_h2's stores, alternating, HIP events; C must
come out identical.  --switch nt: non-temporal vs the default cache policy
(dsvgd_w2_set_cost_nt); --switch lines: whole 128-byte lines vs half lines
(dsvgd_w2_set_cost_lines).
    python scripts/w2_cost_ab.py [--m 65536 --n 65536 --d 256] [--switch nt|lines]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dist-svgd_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=65536)
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--switch", default="nt", choices=("nt", "lines"))
    a = ap.parse_args()
    from dsvgd import _native as N
    from dsvgd.w2 import W2Term
    lib = N.load()
    setter = getattr(lib, "dsvgd_w2_set_cost_" + a.switch)
    g = torch.Generator(device="cpu").manual_seed(0)
    X = torch.randn(a.m, a.d, generator=g).cuda()
    P = (X.repeat(a.n // a.m, 1) - 1e-3 * torch.randn(a.n, a.d, generator=g).cuda()).contiguous()
    W2Term.COST = "h2"
    w = W2Term(a.m, a.n, a.d, "cuda:0")
    s = N.stream(X.device)
    ws = (N.ptr(w.cws) + 255) // 256 * 256

    def cost():
        N.call("dsvgd_w2_cost_h2", N.ptr(X), a.d, a.m, N.ptr(P), a.d, a.n, a.d, N.ptr(w.C), w.ldc,
               ws, float(w.TAU), N.ptr(w.cstat), s)

    ref = {}
    for nt in (1, 0):
        setter(nt)
        cost()
        torch.cuda.synchronize()
        ref[nt] = w.C.clone()
    same = bool(torch.equal(ref[0], ref[1]))
    del ref
    res = {1: [], 0: []}
    for _ in range(4):
        for nt in (1, 0):
            setter(nt)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                cost()
            e1.record()
            torch.cuda.synchronize()
            res[nt].append(e0.elapsed_time(e1) / 3)
    setter(1)
    print(json.dumps({"switch": a.switch, "cost_ms": res, "mean_on": sum(res[1][1:]) / 3,
                      "mean_off": sum(res[0][1:]) / 3,
                      "C_identical": same}))


if __name__ == "__main__":
    main()
