"""In-process interleaved A/B of phi_w1_kernel's A-fragment prefetch
(dsvgd_phi_set_prefetch 0 / 1) at the headline shape: the symmetric layout's
DS 1 + DS 2 pair (S = 1) and a full-layout row block (DS 0, the S = 8 share),
rounds interleaved in ONE process (cdna_hip_programming.md rule 24); phi of
both forms must agree bit for bit (same MFMA order).

    python scripts/phi_pf_ab.py [--rounds 5 --reps 3]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dist-svgd_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--forms", default="0,1")
    ap.add_argument("--cfgs", default="sym_S1,rows_S8")
    args = ap.parse_args()
    import dsvgd
    lib = dsvgd._native.load()
    n, d = args.n, args.d
    g = torch.Generator(device="cpu").manual_seed(0)
    X = (0.1 * torch.randn(n, d, generator=g)).cuda()
    S = torch.randn(n, d, generator=g).cuda()
    forms = [int(f) for f in args.forms.split(",")]
    cfgs = {"sym_S1": dict(m=None, row0=0), "rows_S8": dict(m=n // 8, row0=n // 2)}
    out = {}
    for name, c in cfgs.items():
        if name not in args.cfgs.split(","):
            continue
        kw = {} if c["m"] is None else dict(m=c["m"], row0=c["row0"])
        eng = dsvgd.PhiEngine(n, d, device="cuda:0", **kw)
        eng.pack(X, S)
        eng.distances(median=True)
        eng.median_bandwidth()
        times = {f: [] for f in forms}
        det = []
        phis = {}
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(args.rounds):
            for f in dict.fromkeys(forms):
                lib.dsvgd_phi_set_prefetch(f)
                eng.direction(write_phi=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(args.reps):
                    eng.direction(write_phi=True)
                e1.record()
                torch.cuda.synchronize()
                times[f].append(e0.elapsed_time(e1) / args.reps)
                if f in phis and f < 10:
                    det.append(bool(torch.equal(phis[f], eng.phi)))   # run to run
                phis[f] = eng.phi.clone()
        real = [f for f in forms if f < 10]      # 11..15: timing probes (wrong results)
        same = all(torch.equal(phis[real[0]], phis[f]) for f in real) if real else None
        res = {"sym": bool(eng.sym), "bit_equal": same, "deterministic": all(det)}
        for f in forms:
            t = sorted(times[f])
            res["pf%d_ms" % f] = {"min": t[0], "median": t[len(t) // 2], "all": t}
        out[name] = res
        print(json.dumps({name: res}), flush=True)
        del eng
        torch.cuda.empty_cache()
    lib.dsvgd_phi_set_prefetch(0)


if __name__ == "__main__":
    main()
