"""NT (Gram) engine efficiency vs K: times dsvgd_sqdist (no select) at
several d, symmetric (m = n) and row-block (m = n/2) shapes.

    python scripts/nt_probe.py [--n 32768]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dist-svgd_amd"))

import torch  # noqa: E402


def timed(fn, reps=3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=32768)
    ap.add_argument("--ds", default="256,512,1024,2048")
    args = ap.parse_args()
    import dsvgd
    n = args.n
    out = {}
    for d in [int(x) for x in args.ds.split(",")]:
        X = torch.randn(n, d, device="cuda") * 0.1
        for name, m, row0 in (("sym", n, 0), ("rows", n // 2, n // 2)):
            eng = dsvgd.PhiEngine(n, d, m=m, row0=row0, device="cuda:0")
            eng.pack(X)
            dp = eng.dp
            T = eng.n_pad // 128
            flops = (T * (T + 1) // 2 if name == "sym" else (eng.m_pad // 128) * T) * 2.0 * 128 * 128 * dp
            for pv in os.environ.get("PROBE_PERSIST", "1,0").split(","):
                os.environ["DSVGD_SQ_PERSIST"] = pv
                ms = timed(lambda: eng.distances(median=False))
                msb = timed(lambda: eng.distances(median=True)) if eng.bracketed else None
                out["%s_d%d_p%s" % (name, d, pv)] = {"ms": ms, "tflops": flops / ms / 1e9,
                                                     "bracket_ms": msb}
            os.environ.pop("DSVGD_SQ_PERSIST", None)
            for ev in os.environ.get("PROBE_EPI", "").split(","):
                if not ev:
                    continue
                os.environ["DSVGD_SQ_EPI"] = ev
                ms = timed(lambda: eng.distances(median=False))
                out["%s_d%d_epi%s" % (name, d, ev)] = {"ms": ms, "tflops": flops / ms / 1e9}
            os.environ.pop("DSVGD_SQ_EPI", None)
            del eng
            torch.cuda.empty_cache()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
