"""Per-shape time of dmc_conv2d_wgrad (kernel + slab reduce) for the 3x3 weight gradients of the B=128 CIFAR train
step, under each setting of DMC_WG_PIPE (and DMC_WG_HALO_TARGET values), HIP events around back-to-back calls.

    python scripts/wgrad_probe2.py [--iters N]
"""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from diffusion_models_collection_amd import _lib as L, kernels as K  # noqa: E402

SHAPES = {   # name: (B, H, W, C1, C2, Cout, count per train step)
    "32 128-128": (128, 32, 32, 128, 0, 128, 7),
    "32 256-128": (128, 32, 32, 128, 128, 128, 2),
    "32 384-128": (128, 32, 32, 256, 128, 128, 1),
    "16 256-256": (128, 16, 16, 256, 0, 256, 7),
    "16 512-256": (128, 16, 16, 256, 256, 256, 2),
    "16 384-256": (128, 16, 16, 256, 128, 256, 1),
    "16 128-256": (128, 16, 16, 128, 0, 256, 1),
    "8 256-256": (128, 8, 8, 256, 0, 256, 8),
    "8 512-256": (128, 8, 8, 256, 256, 256, 3),
    "4 256-256": (128, 4, 4, 256, 0, 256, 11),
    "4 512-256": (128, 4, 4, 256, 256, 256, 3),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--shape", default="")
    ap.add_argument("--only", default="", help="one setting name (e.g. pipe)")
    a = ap.parse_args()
    settings = [("r4 halo", {"DMC_WG_PIPE": 0}), ("pipe", {"DMC_WG_IMG4": 0}), ("img4", {"DMC_WG_IMG4": 1}), ("pipe t128", {"DMC_WG_HALO_TARGET": 128}),
                ("pipe t192", {"DMC_WG_HALO_TARGET": 192}), ("pipe t384", {"DMC_WG_HALO_TARGET": 384}),
                ("pipe t16", {"DMC_WG_HALO_TARGET": 16}), ("pipe t32", {"DMC_WG_HALO_TARGET": 32}),
                ("pipe t64", {"DMC_WG_HALO_TARGET": 64})]
    if a.only:
        settings = [s_ for s_ in settings if s_[0] == a.only]
    tot = {n: 0.0 for n, _ in settings}
    dt = torch.bfloat16
    for name, (B, H, W, C1, C2, Cout, cnt) in SHAPES.items():
        if a.shape and a.shape != name:
            continue
        x1 = torch.randn(B, H, W, C1, device="cuda").to(dt)
        x2 = torch.randn(B, H, W, C2, device="cuda").to(dt) if C2 else None
        dy = torch.randn(B, H, W, Cout, device="cuda").to(dt)
        dw = torch.empty(Cout, C1 + C2, 3, 3, device="cuda")
        db = torch.empty(Cout, device="cuda")
        d = K.make_desc(dt, B, H, W, C1, C2, C1, C2, L.kc_for(C1 + C2, dt), H, W, Cout, K.TAPS3)
        row = []
        ref = None
        for sname, opts in settings:
            L.reset_options(from_env=False)
            for k, v in opts.items():
                L.set_option(k, v)
            for _ in range(3):
                K.wgrad(d, dy, Cout, x1, x2, dw, dbias=db)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                K.wgrad(d, dy, Cout, x1, x2, dw, dbias=db)
            e1.record()
            e1.synchronize()
            us = e0.elapsed_time(e1) / a.iters * 1e3
            if ref is None:
                ref = dw.clone()
            err = ((dw - ref).norm() / ref.norm()).item()
            tot[sname] += us * cnt
            fl = 2.0 * B * H * W * Cout * (C1 + C2) * 9
            row.append(f"{sname}: {us:6.1f} us {fl / us / 1e6:6.1f} TF/s (err {err:.1e})")
        L.reset_options(from_env=False)
        print(f"{name:11s} x{cnt}: " + " | ".join(row), flush=True)
    print("per train step: " + ", ".join(f"{k} {v:.0f} us" for k, v in tot.items()))


if __name__ == "__main__":
    main()
