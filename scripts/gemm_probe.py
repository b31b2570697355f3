"""Measurement tool (never imported by the package): the UNet's 1x1 convs / Linear GEMMs at B=128 through
dmc_conv2d (the LDS-DMA kernels, plain bias epilogue) vs torch.addmm (hipBLASLt / rocBLAS on ROCm), bf16,
HIP-event averages over back-to-back launches on the current stream.

    python scripts/gemm_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from diffusion_models_collection_amd import _lib as L, kernels as K  # noqa: E402

SHAPES = [  # (name, M pixels, K in, N out)
    ("qkv16", 128 * 256, 256, 768), ("qkv8", 128 * 64, 256, 768), ("proj16", 128 * 256, 256, 256),
    ("proj8", 128 * 64, 256, 256), ("sc32_256_128", 128 * 1024, 256, 128), ("sc16_512_256", 128 * 256, 512, 256),
    ("sc8_512_256", 128 * 64, 512, 256), ("sc4_512_256", 128 * 16, 512, 256), ("temb", 128, 512, 4992),
]


def timeit(fn, n=50):
    for _ in range(5):
        fn()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(n):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def main():
    dev = "cuda"
    dt = torch.bfloat16
    torch.manual_seed(0)
    for name, M, Kd, N in SHAPES:
        x = torch.randn(M, Kd, device=dev).to(dt)
        w = torch.randn(N, Kd, device=dev) * 0.05
        b = torch.randn(N, device=dev)
        Kc = L.kc_for(Kd, dt)
        wp = K.pack_weight(L.PACK_FWD, dt, w.view(N, Kd, 1, 1), Kc)
        y = torch.empty(M, N, device=dev, dtype=dt)
        d = K.make_desc(dt, M, 1, 1, Kd, 0, Kd, 0, Kc, 1, 1, N, K.TAPS1)
        K.set_epilogue(d, bias=b, ldy1=N)
        t_dmc = timeit(lambda: K.conv(d, x, None, wp, y))
        wt = w.to(dt).t().contiguous()   # [K][N]
        bt = b.to(dt)
        yt = torch.empty(M, N, device=dev, dtype=dt)
        t_bl = timeit(lambda: torch.addmm(bt, x, wt, out=yt))
        wn = w.to(dt)
        t_bl2 = timeit(lambda: torch.nn.functional.linear(x, wn, bt))
        torch.cuda.synchronize()
        ref = (x.float() @ w.to(dt).float().t() + b.to(dt).float())
        e1 = ((y.float() - ref).norm() / ref.norm()).item()
        e2 = ((yt.float() - ref).norm() / ref.norm()).item()
        fl = 2.0 * M * Kd * N
        print(f"{name:14s} M={M:7d} K={Kd:4d} N={N:5d}  dmc {t_dmc:7.1f} us ({fl / t_dmc / 1e6:6.1f} TF/s, err {e1:.1e})"
              f"  addmm {t_bl:7.1f} us ({fl / t_bl / 1e6:6.1f} TF/s, err {e2:.1e})  linear {t_bl2:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
