"""Measurement tool: the DiT-S/2 linear shapes (M = 256 images x 256 tokens) on the implicit-GEMM conv kernel
(1x1 taps) vs torch.nn.functional.linear (hipBLASLt), bf16, HIP-event timing. Not part of the product."""
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from diffusion_models_collection_amd import _lib as L, kernels as K  # noqa: E402

dev = "cuda"
M = int(os.environ.get("M", 65536))
SHAPES = [(1152, 384), (384, 384), (1536, 384), (384, 1536)]


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e-3


for N, Kd in SHAPES:
    x = torch.randn(M, Kd, device=dev).bfloat16()
    w = torch.randn(N, Kd, device=dev) * 0.05
    b = torch.randn(N, device=dev)
    wb = w.bfloat16()
    fl = 2.0 * M * N * Kd
    tl = timeit(lambda: torch.nn.functional.linear(x, wb, b.bfloat16()))
    Kc = L.kc_for(Kd, torch.bfloat16)
    wp = K.pack_weight(L.PACK_FWD, torch.bfloat16, w, Kc)
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    d = K.make_desc(torch.bfloat16, M, 1, 1, Kd, 0, Kd, 0, Kc, 1, 1, N, K.TAPS1)
    K.set_epilogue(d, bias=b, ldy1=N)
    tc = timeit(lambda: K.conv(d, x, None, wp, y))
    ref = torch.nn.functional.linear(x.float(), wb.float(), b)
    err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
    print(f"M={M} N={N} K={Kd}: hipBLASLt {tl * 1e6:8.1f} us {fl / tl / 1e12:7.1f} TF/s | dmc conv {tc * 1e6:8.1f} us "
          f"{fl / tc / 1e12:7.1f} TF/s (rel err {err:.1e})", flush=True)
