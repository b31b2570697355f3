"""Is there idle GPU capacity beside the backward's small-map kernels? Per shape of the B=128 CIFAR step: N 3x3
convs (the input-gradient's kernel class) and N weight gradients, timed one after the other on one stream and
concurrently on two streams (HIP events).

    python scripts/r6_overlap_probe.py [--iters N]
"""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from diffusion_models_collection_amd import _lib as L, kernels as K  # noqa: E402

SHAPES = {"4 256-256": (128, 4, 4, 256, 256), "8 256-256": (128, 8, 8, 256, 256),
          "16 256-256": (128, 16, 16, 256, 256), "32 128-128": (128, 32, 32, 128, 128)}


def timed(fn, streams):
    ev = []
    cur = torch.cuda.current_stream()
    for s in streams:
        s.wait_stream(cur)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for s in streams:
        s.wait_event(e0)
    fn()
    for s in streams:
        cur.wait_stream(s)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dt = torch.bfloat16
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    for name, (B, H, W, Cin, Cout) in SHAPES.items():
        x = torch.randn(B, H, W, Cin, device="cuda").to(dt)
        dy = torch.randn(B, H, W, Cout, device="cuda").to(dt)
        w = torch.randn(Cout, Cin, 3, 3, device="cuda") / (Cin * 9) ** 0.5
        Kc = L.kc_for(Cin, dt)
        wp = K.pack_weight(L.PACK_FWD, dt, w, Kc)
        d = K.make_desc(dt, B, H, W, Cin, 0, Cin, 0, Kc, H, W, Cout, K.TAPS3)
        K.set_epilogue(d, ldy1=Cout)
        ys = [torch.empty(B, H, W, Cout, dtype=dt, device="cuda") for _ in range(2)]
        dg = K.make_desc(dt, B, H, W, Cin, 0, Cin, 0, Kc, H, W, Cout, K.TAPS3)
        dws = [torch.empty(Cout, Cin, 3, 3, device="cuda") for _ in range(2)]
        n = a.iters

        def convs():
            for i in range(n):
                K.conv(d, x, None, wp, ys[i % 2])

        def wgrads():
            for i in range(n):
                K.wgrad(dg, dy, Cout, x, None, dws[i % 2])

        def seq():
            with torch.cuda.stream(sa):
                for i in range(n):
                    K.conv(d, x, None, wp, ys[i % 2])
                    K.wgrad(dg, dy, Cout, x, None, dws[i % 2])

        def par():
            with torch.cuda.stream(sa):
                convs()
            with torch.cuda.stream(sb):
                wgrads()

        for _ in range(2):
            with torch.cuda.stream(sa):
                convs()
                wgrads()
        torch.cuda.synchronize()
        res = {}
        for k in range(2):
            with torch.cuda.stream(sa):
                tc = timed(convs, [sa])
            with torch.cuda.stream(sa):
                tw = timed(wgrads, [sa])
            ts = timed(seq, [sa])
            tp = timed(par, [sa, sb])
            res = {"conv": tc / n, "wgrad": tw / n, "seq": ts / n, "par": tp / n}
        print(f"{name:11s} per pair (us): conv {res['conv']:6.1f}  wgrad {res['wgrad']:6.1f}  "
              f"one stream {res['seq']:6.1f}  two streams {res['par']:6.1f}  "
              f"saving {1 - res['par'] / res['seq']:.1%}", flush=True)


if __name__ == "__main__":
    main()
