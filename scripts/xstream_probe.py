"""Cross-stream visibility probe: a buffer read on the main stream (its lines
in the L2s), rewritten on a side stream after an event wait, then read again
on the main stream after waiting for the side's event.  Counts mismatches."""
import json
import torch


def main():
    dev = torch.device("cuda:0")
    main_s = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(device=dev)
    bad = 0
    trials = 0
    for n in (1 << 16, 1 << 20, 1 << 24):
        x = torch.zeros(n, device=dev)
        for t in range(40):
            val = float(t + 1)
            s0 = x.sum()                       # main: lines of x in the L2s
            ev = main_s.record_event()
            side.wait_event(ev)
            with torch.cuda.stream(side):
                x.fill_(val)                   # side: rewrite
                done = side.record_event()
            main_s.wait_event(done)
            s1 = x.sum()                       # main: read again
            y = x.clone()
            torch.cuda.synchronize()
            ok = bool((y == val).all())
            trials += 1
            bad += (not ok) or abs(float(s1) - val * n) > 1e-3 * val * n
            del s0
    print(json.dumps({"trials": trials, "mismatches": int(bad)}), flush=True)


if __name__ == "__main__":
    main()
