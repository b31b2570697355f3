"""Split-count sweep of the weight-gradient launches (dmc_conv2d_wgrad = the wgrad kernel + the slab reduce) on every
weight-gradient shape of the B=128 CIFAR UNet train step: for each shape, the block targets DMC_WG_HALO_TARGET (halo
kernel) / DMC_WG_BLOCKS (generic and 1x1 kernels), HIP events around `iters` back-to-back calls.

    python scripts/wgrad_sweep.py [--iters N] [--only SUBSTR]
"""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from diffusion_models_collection_amd import _lib as L, kernels as K  # noqa: E402

# name: (B, H, W, C1, C2, Cout, taps, OH, OW, mode, stride, count per train step)
T3, T1 = K.TAPS3, K.TAPS1
SHAPES = {
    "3x3 32 128-128": (128, 32, 32, 128, 0, 128, T3, 32, 32, L.MODE_NORMAL, 1, 7),
    "3x3 32 256-128": (128, 32, 32, 128, 128, 128, T3, 32, 32, L.MODE_NORMAL, 1, 2),
    "3x3 32 384-128": (128, 32, 32, 256, 128, 128, T3, 32, 32, L.MODE_NORMAL, 1, 1),
    "3x3 16 256-256": (128, 16, 16, 256, 0, 256, T3, 16, 16, L.MODE_NORMAL, 1, 7),
    "3x3 16 512-256": (128, 16, 16, 256, 256, 256, T3, 16, 16, L.MODE_NORMAL, 1, 2),
    "3x3 16 384-256": (128, 16, 16, 256, 128, 256, T3, 16, 16, L.MODE_NORMAL, 1, 1),
    "3x3 16 128-256": (128, 16, 16, 128, 0, 256, T3, 16, 16, L.MODE_NORMAL, 1, 1),
    "3x3 8 256-256": (128, 8, 8, 256, 0, 256, T3, 8, 8, L.MODE_NORMAL, 1, 8),
    "3x3 8 512-256": (128, 8, 8, 256, 256, 256, T3, 8, 8, L.MODE_NORMAL, 1, 3),
    "3x3 4 256-256": (128, 4, 4, 256, 0, 256, T3, 4, 4, L.MODE_NORMAL, 1, 11),
    "3x3 4 512-256": (128, 4, 4, 256, 256, 256, T3, 4, 4, L.MODE_NORMAL, 1, 3),
    "3x3 in 3-128": (128, 32, 32, 3, 0, 128, T3, 32, 32, L.MODE_NORMAL, 1, 1),
    "3x3 out 128-3": (128, 32, 32, 128, 0, 3, T3, 32, 32, L.MODE_NORMAL, 1, 1),
    "3x3 down 32-16": (128, 32, 32, 128, 0, 128, T3, 16, 16, L.MODE_NORMAL, 2, 1),
    "3x3 down 8-4": (128, 8, 8, 256, 0, 256, T3, 4, 4, L.MODE_NORMAL, 2, 1),
    "3x3 up 16-32": (128, 16, 16, 128, 0, 128, T3, 32, 32, L.MODE_UPSAMPLE, 1, 1),
    "1x1 16 256-768": (128, 16, 16, 256, 0, 768, T1, 16, 16, L.MODE_NORMAL, 1, 5),
    "1x1 8 256-768": (128, 8, 8, 256, 0, 768, T1, 8, 8, L.MODE_NORMAL, 1, 5),
    "1x1 16 256-256": (128, 16, 16, 256, 0, 256, T1, 16, 16, L.MODE_NORMAL, 1, 5),
    "1x1 8 256-256": (128, 8, 8, 256, 0, 256, T1, 8, 8, L.MODE_NORMAL, 1, 5),
    "1x1 8 512-256": (128, 8, 8, 512, 0, 256, T1, 8, 8, L.MODE_NORMAL, 1, 3),
    "1x1 4 512-256": (128, 4, 4, 512, 0, 256, T1, 4, 4, L.MODE_NORMAL, 1, 3),
    "1x1 32 256-128": (128, 32, 32, 256, 0, 128, T1, 32, 32, L.MODE_NORMAL, 1, 2),
}


def time_shape(spec, iters):
    B, H, W, C1, C2, Cout, taps, OH, OW, mode, stride, _ = spec
    dt = torch.bfloat16
    dev = "cuda"
    x1 = torch.randn(B, H, W, C1, device=dev).to(dt)
    ldx = C1
    if C1 < 8:   # the input conv's packed input: 8-channel pitch
        ldx = 8
        x1 = torch.randn(B, H, W, 8, device=dev).to(dt)
    x2 = torch.randn(B, H, W, C2, device=dev).to(dt) if C2 else None
    ldy = max(Cout, 8)
    dy = torch.randn(B, OH, OW, ldy, device=dev).to(dt)
    kh = 3 if len(taps) == 9 else 1
    dw = torch.empty(Cout, C1 + C2, kh, kh, device=dev)
    db = torch.empty(Cout, device=dev)
    Kc = L.kc_for(C1 + C2, dt)
    d = K.make_desc(dt, B, H, W, C1, C2, ldx, C2, Kc, OH, OW, Cout, taps, mode, stride)
    for _ in range(2):
        K.wgrad(d, dy, ldy, x1, x2, dw, dbias=db)
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        K.wgrad(d, dy, ldy, x1, x2, dw, dbias=db)
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3, dw.clone()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    tot_def = tot_best = 0.0
    for name, spec in SHAPES.items():
        if a.only and a.only not in name:
            continue
        halo = spec[6] is T3 and spec[10] == 1 and spec[9] == L.MODE_NORMAL and spec[3] % 64 == 0 and spec[2] >= 8
        opt, vals = ("DMC_WG_HALO_TARGET", [16, 32, 64, 96, 128, 192, 256, 384]) if halo else \
                    ("DMC_WG_BLOCKS", [32, 64, 128, 192, 256, 384, 512, 768])
        L.reset_options(from_env=False)
        t_def, ref = time_shape(spec, a.iters)
        res = []
        for v in vals:
            L.set_option(opt, v)
            t, dw = time_shape(spec, a.iters)
            err = ((dw - ref).norm() / ref.norm()).item()
            res.append((t, v, err))
        L.reset_options(from_env=False)
        best = min(res)
        n = spec[-1]
        tot_def += t_def * n
        tot_best += best[0] * n
        print(f"{name:16s} x{n:2d} default {t_def:7.1f} us | " + " ".join(f"{v}:{t:.1f}" for t, v, _ in res)
              + f" | best {opt}={best[1]} {best[0]:.1f} us (rel diff {max(e for _, _, e in res):.1e})", flush=True)
    print(f"per step: default {tot_def:.0f} us, per-shape best {tot_best:.0f} us")


if __name__ == "__main__":
    main()
