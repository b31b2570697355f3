"""Time the bf16 3x3 weight-gradient (dmc_conv2d_wgrad: the halo wgrad kernel + the slab reduce) on the UNet's
layer shapes, HIP events on the launch stream; under `rocprofv3 --kernel-trace --stats` the two launches separate.

    python scripts/wgrad_probe.py [--shape NAME] [--iters N]
"""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from diffusion_models_collection_amd import _lib as L, kernels as K  # noqa: E402

# name: (B, H, W, C1, C2, Cout)
SHAPES = {
    "w128_32": (128, 32, 32, 128, 0, 128),     # ResBlock 128->128 @32x32
    "w256_32": (128, 32, 32, 128, 128, 128),   # decoder concat 256->128 @32x32
    "w384_32": (128, 32, 32, 256, 128, 128),   # decoder concat 384->128 @32x32
    "w256_16": (128, 16, 16, 256, 0, 256),
    "w512_16": (128, 16, 16, 256, 256, 256),
    "w256_8": (128, 8, 8, 256, 0, 256),
    "w512_8": (128, 8, 8, 256, 256, 256),
}


def run(name, iters):
    B, H, W, C1, C2, Cout = SHAPES[name]
    dt = torch.bfloat16
    dev = "cuda"
    x1 = torch.randn(B, H, W, C1, device=dev).to(dt)
    x2 = torch.randn(B, H, W, C2, device=dev).to(dt) if C2 else None
    dy = torch.randn(B, H, W, Cout, device=dev).to(dt)
    dw = torch.empty(Cout, C1 + C2, 3, 3, device=dev)
    db = torch.empty(Cout, device=dev)
    Kc = L.kc_for(C1 + C2, dt)
    d = K.make_desc(dt, B, H, W, C1, C2, C1, C2, Kc, H, W, Cout, K.TAPS3)
    for _ in range(3):
        K.wgrad(d, dy, Cout, x1, x2, dw, dbias=db)
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        K.wgrad(d, dy, Cout, x1, x2, dw, dbias=db)
    e1.record(s)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / iters
    flops = 2.0 * B * H * W * Cout * (C1 + C2) * 9
    print(f"{name:8s} M={B*H*W:7d} KK={(C1+C2)*9:5d} N={Cout:4d} {ms*1e3:8.1f} us (kernel + reduce) "
          f"{flops/ms/1e9:7.1f} TFLOP/s", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="all")
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    for name in (SHAPES if a.shape == "all" else [a.shape]):
        run(name, a.iters)


if __name__ == "__main__":
    main()
