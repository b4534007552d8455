"""Where the wide sweep's walk spends its time: one 64-row block of config D
(n = 65536, d = 256, frozen scores) walked repeatedly with parts of the row
step switched off (dsvgd_gsw_debug: 1 = no operand loads, 2 = no distances,
4 = no column loop); HIP-event time per launch.  Timing only.

    python scripts/walk_probe.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dist-svgd_amd"))

import torch  # noqa: E402


def main():
    import dsvgd
    from dsvgd import _native as N
    from dsvgd.engine import SelectState, sequential_sweep, _WIDE
    n, d = 65536, 256
    g = torch.Generator(device="cpu").manual_seed(0)
    X = (0.1 * torch.randn(n, d, generator=g)).cuda()
    S = torch.randn(n, d, generator=g).cuda()
    st = SelectState("cuda:0")
    N.call("dsvgd_set_bandwidth", st.ptr, 0.9 * d, N.stream("cuda:0"))
    sequential_sweep(X, S, range(0, 128), st, 1e-4)   # the buffers; Q of block 64
    torch.cuda.synchronize()
    W = next(iter(_WIDE.values()))
    lib = N.load()
    s = N.stream("cuda:0")
    b0, nb = 64, W.B

    def walk():
        N.call("dsvgd_gsw_block_sweep", N.ptr(X), d, N.ptr(S), d, N.ptr(W.Y), W.ldy,
               N.ptr(W.norms), N.ptr(W.mean), n, d, b0, nb, st.ptr, 1e-4, N.ptr(W.Q), W.ldy,
               N.ptr(W.Qr), None, d, None, d, 0, None, None, 1.0, None, d, None, 0, s)
    for mask in (0, 1, 2, 4, 6, 7, 0):
        lib.dsvgd_gsw_debug(mask)
        for _ in range(3):
            walk()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            walk()
        e1.record()
        torch.cuda.synchronize()
        print(json.dumps({"mask": mask, "us_per_walk": round(1e3 * e0.elapsed_time(e1) / 50, 2),
                          "rows": nb}), flush=True)
    lib.dsvgd_gsw_debug(0)


if __name__ == "__main__":
    main()
