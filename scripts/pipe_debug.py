"""Debug the pipelined wide sweep: NaN location and per-block differences
against the serial form, with individual calls switched off."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dist-svgd_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import dsvgd  # noqa: F401
    from dsvgd import _native as N
    from dsvgd import engine as E
    from dsvgd.engine import SelectState, sequential_sweep
    n, d = int(sys.argv[1]) if len(sys.argv) > 1 else 1024, 256
    rs = np.random.RandomState(21)
    X0 = (0.3 * rs.randn(n, d)).astype(np.float32)
    S0 = (-X0 / 0.09 + 0.3 * rs.randn(n, d)).astype(np.float32)
    h = 2.0 * d * 0.09 / np.log(n)
    st = SelectState("cuda:0")
    N.call("dsvgd_set_bandwidth", st.ptr, h, N.stream("cuda:0"))
    real_call = N.call
    out = {}
    for name, pipe, skip, dbg in (("serial", False, None, 0), ("pipe", True, None, 0),
                                  ("pipe_dbgQ", True, None, 8), ("serial_dbgQ", False, None, 8)):
        E.GSW_PIPELINE = pipe
        E._GSW_DEBUG = dbg
        N.load().dsvgd_gsw_debug(8 if name.endswith("walk4") else 0)

        def call(fn, *a, skip=skip):
            if fn == skip:
                return 0
            return real_call(fn, *a)
        N.call = call
        Xg, Sg = torch.tensor(X0, device="cuda:0"), torch.tensor(S0, device="cuda:0")
        phi = torch.zeros(n, d, device="cuda:0")
        sequential_sweep(Xg, Sg, range(n), st, 1e-2, phi_out=phi)
        torch.cuda.synchronize()
        N.call = real_call
        p = phi.cpu().numpy()
        bad = np.where(~np.isfinite(p).all(1))[0]
        out[name] = p
        rec = {"nan_rows": int(len(bad)), "first_nan_rows": bad[:10].tolist()}
        if name != "serial":
            dif = np.abs(p - out["serial"]).max(1)
            rec["block_maxdiff"] = [float(np.nanmax(dif[b:b + 64])) for b in range(0, n, 64)][:16]
        if dbg == 8:
            W = list(E._WIDE.values())[0]
            qs = {k: (q.cpu().numpy(), r.cpu().numpy()) for k, q, r in W.dbg}
            out["q_" + name] = qs
            badq = [(k, np.where(~np.isfinite(q).all(1))[0][:6].tolist(),
                     np.where(~np.isfinite(r))[0][:6].tolist()) for k, (q, r) in qs.items()
                    if not (np.isfinite(q).all() and np.isfinite(r).all())]
            rec["q_nonfinite"] = badq[:4]
            if name.startswith("serial") and "q_pipe_dbgQ" in out:
                other = out["q_pipe_dbgQ"]
                dif = []
                for k in sorted(qs):
                    if k in other:
                        a, b = qs[k][0], other[k][0]
                        dq = np.abs(a - b)
                        dif.append((k, float(np.nanmax(dq)) if np.isfinite(b).any() else None,
                                    int(np.argmax(np.nanmax(np.where(np.isfinite(dq), dq, 0), 1)))))
                rec["q_vs_pipe"] = dif[:8]
        print(json.dumps({name: rec}), flush=True)


if __name__ == "__main__":
    main()
