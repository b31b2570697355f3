"""Time the GroupNorm kernels on the UNet's shapes (HIP events on the launch stream) and report the
effective bandwidth of each pass (algorithmic bytes / time).

    python scripts/gn_probe.py [--iters N] [--shape NAME]
"""
import argparse
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from diffusion_models_collection_amd import kernels as K  # noqa: E402

SHAPES = {"c128_32": (128, 32, 32, 128), "c256_16": (128, 16, 16, 256), "c512_8": (128, 8, 8, 512),
          "c384_32": (128, 32, 32, 384), "c256_8": (128, 8, 8, 256)}


def timeit(fn, iters):
    s = torch.cuda.current_stream()
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def run(name, iters):
    N, H, W, C = SHAPES[name]
    dt = torch.bfloat16
    dev = "cuda"
    x = torch.randn(N, H, W, C, device=dev).to(dt)
    g = torch.randn(N, H, W, C, device=dev).to(dt)
    gamma = torch.rand(C, device=dev)
    beta = torch.randn(C, device=dev)
    HW = H * W
    sc, sh, mr = K.gn_stats(dt, x, None, N, HW, C, 0, C, 0, 8, 1e-5, gamma, beta)
    out = torch.empty_like(x)
    dx = torch.empty_like(x)
    dg = torch.empty(C, device=dev)
    db = torch.empty(C, device=dev)
    nc = torch.empty(N, C, device=dev)
    cs = torch.empty(C, device=dev)
    drop = (429496730, 0, 1 / 0.9)   # p = 0.1
    T = N * HW * C * 2
    r = {}
    r["stats"] = (timeit(lambda: K.gn_stats(dt, x, None, N, HW, C, 0, C, 0, 8, 1e-5, gamma, beta), iters), T)
    os.environ["DMC_GN_STATS_SPLIT"] = "1"
    r["stats_split"] = (timeit(lambda: K.gn_stats(dt, x, None, N, HW, C, 0, C, 0, 8, 1e-5, gamma, beta), iters), T)
    os.environ["DMC_GN_STATS_SPLIT"] = "0"
    r["apply"] = (timeit(lambda: K.gn_apply(dt, x, None, N, HW, C, 0, C, 0, sc, sh, out=out), iters), 2 * T)
    r["apply_drop"] = (timeit(lambda: K.gn_apply(dt, x, None, N, HW, C, 0, C, 0, sc, sh, drop=drop, out=out),
                              iters), 2 * T)
    r["bwd"] = (timeit(lambda: K.gn_bwd(dt, g, C, x, None, N, HW, C, 0, C, 0, 8, mr, gamma, beta, True, None, dx,
                                        None, C, 0, 0, 0, dg, db), iters), 5 * T)
    r["bwd_drop_sums"] = (timeit(lambda: K.gn_bwd(dt, g, C, x, None, N, HW, C, 0, C, 0, 8, mr, gamma, beta, True,
                                                  drop, dx, None, C, 0, 0, 0, dg, db, dx_sum_nc=nc, ld_sum_nc=C,
                                                  dx_sum_c=cs), iters), 5 * T)
    r["bwd_acc"] = (timeit(lambda: K.gn_bwd(dt, g, C, x, None, N, HW, C, 0, C, 0, 8, mr, gamma, beta, True, None, dx,
                                            None, C, 0, 1, 0, dg, db), iters), 6 * T)
    r["chsum"] = (timeit(lambda: K.channel_sum(dt, g, N, HW, C, C, out_c=cs), iters), T)
    for k, (us, b) in r.items():
        print(f"{name:8s} {k:14s} {us:8.1f} us  {b / us / 1e6:6.2f} TB/s (algorithmic {b / 1e6:.1f} MB)", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="all")
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    for name in (SHAPES if a.shape == "all" else [a.shape]):
        run(name, a.iters)


if __name__ == "__main__":
    main()
