"""Time the bf16 forward conv on the UNet's layer shapes (HIP events on the launch stream).

Used standalone and under `rocprofv3 --pmc ...` to read counters for one kernel at a time:
    python scripts/conv_probe.py [--shape NAME] [--iters N]
"""
import argparse
import ctypes
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from diffusion_models_collection_amd import _lib as L, kernels as K  # noqa: E402

# name: (B, H, W, C1, C2, Cout, taps)
SHAPES = {
    "r128_32": (128, 32, 32, 128, 0, 128, "3"),      # ResBlock 128->128 @32x32 (the bench roofline kernel)
    "r384_32": (128, 32, 32, 256, 128, 128, "3"),    # decoder concat 384->128 @32x32
    "r128_64": (128, 64, 64, 128, 0, 128, "3"),      # config #5 (64x64) ResBlock 128->128
    "r256_16": (128, 16, 16, 256, 0, 256, "3"),
    "r512_8": (128, 8, 8, 256, 256, 256, "3"),       # small M: split-K
    "r512_4": (128, 4, 4, 256, 256, 256, "3"),
    "qkv_16": (128, 16, 16, 256, 0, 768, "1"),
    "p1_8": (128, 8, 8, 256, 0, 256, "1"),
    "qkv_8": (128, 8, 8, 256, 0, 768, "1"),
    "p1_16": (128, 16, 16, 256, 0, 256, "1"),
    "r256_8": (128, 8, 8, 256, 0, 256, "3"),
    "r256_4": (128, 4, 4, 256, 0, 256, "3"),
    "d512_8": (128, 8, 8, 256, 0, 512, "d"),       # input gradient of the 8x8 up-block conv1 (256 -> 512)
    "d512_4": (128, 4, 4, 256, 0, 512, "d"),
    "nin_32": (128, 32, 32, 3, 0, 128, "3"),         # the UNet's first conv (3 -> 128, narrow-input kernel)
    "nout_32": (128, 32, 32, 128, 0, 3, "3"),        # the output conv (128 -> 3, narrow-output kernel)
}


def run(name, iters, epi="bias", cold=False):
    B, H, W, C1, C2, Cout, kind = SHAPES[name]
    dt = torch.bfloat16
    dev = "cuda"
    taps = K.TAPS3 if kind == "3" else K.TAPS3_DGRAD if kind == "d" else K.TAPS1
    kk = 1 if kind == "1" else 3
    ld1 = C1 if C1 >= 8 else 8    # a narrow source is stored at one 16-byte chunk per pixel
    x1 = torch.randn(B, H, W, ld1, device=dev).to(dt)
    x2 = torch.randn(B, H, W, C2, device=dev).to(dt) if C2 else None
    w = torch.randn(Cout, C1 + C2, kk, kk, device=dev) * 0.03
    Kc = L.kc_for(C1 + C2, dt)
    if kind == "d":   # the forward conv Cout -> C1 read backwards: flipped / transposed pack
        w = torch.randn(C1 + C2, Cout, kk, kk, device=dev) * 0.03
    wp = K.pack_weight(L.PACK_DGRAD if kind == "d" else L.PACK_FWD, dt, w, Kc)
    y = torch.empty(B, H, W, Cout, device=dev, dtype=dt)
    d = K.make_desc(dt, B, H, W, C1, C2, ld1, C2, Kc, H, W, Cout, taps)
    if epi == "full":   # ResBlock conv2 epilogue: bias + time embedding + residual
        resid = torch.randn(B, H, W, Cout, device=dev).to(dt)
        K.set_epilogue(d, bias=torch.randn(Cout, device=dev), addvec=torch.randn(B, Cout, device=dev), ld_add=Cout,
                       resid=resid, ld_res=Cout, ldy1=Cout)
    elif epi in ("temb", "gn"):   # conv1 epilogue: bias + time embedding (+ the next GroupNorm's partials: bench roofline)
        part = torch.empty(B * H * W // 64 * (Cout // 8) * 2, device=dev) if epi == "gn" else None
        K.set_epilogue(d, bias=torch.randn(Cout, device=dev), addvec=torch.randn(B, Cout, device=dev), ld_add=Cout,
                       ldy1=Cout, gn_part=part)
    else:
        K.set_epilogue(d, bias=torch.randn(Cout, device=dev), ldy1=Cout)
    ws = L.LIB.dmc_conv2d_workspace(ctypes.byref(d))
    for _ in range(3):
        K.conv(d, x1, x2, wp, y)
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if cold:
        # every launch with L2 and the MALL evicted (a 1 GiB write in between, outside the timed pair)
        flush = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
        small = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
        ms = 0.0
        for _ in range(iters):
            (flush if cold == "cold" else small).fill_(1)   # "hot1": the same per-launch timing, caches kept
            e0.record(s)
            K.conv(d, x1, x2, wp, y)
            e1.record(s)
            e1.synchronize()
            ms += e0.elapsed_time(e1)
        ms /= iters
    else:
        e0.record(s)
        for _ in range(iters):
            K.conv(d, x1, x2, wp, y)
        e1.record(s)
        e1.synchronize()
        ms = e0.elapsed_time(e1) / iters
    flops = 2.0 * B * H * W * Cout * (C1 + C2) * kk * kk
    print(f"{name:8s} M={B*H*W:7d} K={(C1+C2)*kk*kk:5d} N={Cout:4d} splitk_ws={ws/2**20:6.1f}MiB "
          f"{ms*1e3:8.1f} us{' ' + cold if cold else ''}  {flops/ms/1e9:7.1f} TFLOP/s", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="all")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--epi", default="bias", choices=["bias", "full", "temb", "gn"])
    ap.add_argument("--cold", default="", choices=["", "cold", "hot1"],
                    help="time launches one at a time, with L2 / MALL evicted before each (cold) or not (hot1)")
    a = ap.parse_args()
    for name in (SHAPES if a.shape == "all" else [a.shape]):
        run(name, a.iters, a.epi, a.cold)


if __name__ == "__main__":
    main()
