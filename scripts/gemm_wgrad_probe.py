"""1x1 weight gradients of the B=128 CIFAR UNet train step: dmc_conv2d_wgrad (wgrad1x1_glds_kernel + slab reduce)
against the library GEMM (torch.mm -> hipBLASLt) of the same bf16 operands, dW = dY^T X (M = Cout, N = Cin,
K = pixels). HIP events around `iters` back-to-back calls.

    python scripts/gemm_wgrad_probe.py [--iters N]
"""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from diffusion_models_collection_amd import _lib as L, kernels as K  # noqa: E402
from wgrad_sweep import SHAPES  # noqa: E402


def timeit(fn, iters):
    for _ in range(2):
        fn()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    dt, dev = torch.bfloat16, "cuda"
    tot = {"dmc": 0.0, "mm": 0.0, "mm32": 0.0}
    for name, spec in SHAPES.items():
        if not name.startswith("1x1"):
            continue
        B, H, W, C1, C2, Cout, taps, OH, OW, mode, stride, n = spec
        x = torch.randn(B, H, W, C1, device=dev).to(dt)
        dy = torch.randn(B, OH, OW, Cout, device=dev).to(dt)
        dw = torch.empty(Cout, C1, 1, 1, device=dev)
        db = torch.empty(Cout, device=dev)
        d = K.make_desc(dt, B, H, W, C1, 0, C1, 0, L.kc_for(C1, dt), OH, OW, Cout, taps, mode, stride)
        t_dmc = timeit(lambda: K.wgrad(d, dy, Cout, x, None, dw, dbias=db), a.iters)
        x2, dy2 = x.view(-1, C1), dy.view(-1, Cout)
        t_mm = timeit(lambda: torch.mm(dy2.t(), x2), a.iters)
        try:
            t_mm32 = timeit(lambda: torch.mm(dy2.t(), x2, out_dtype=torch.float32), a.iters)
            ref = torch.mm(dy2.t(), x2, out_dtype=torch.float32)
            err = ((dw.view(Cout, C1) - ref).norm() / ref.norm()).item()
        except (TypeError, RuntimeError) as e:
            t_mm32, err = float("nan"), float("nan")
            print("out_dtype:", str(e)[:80])
        fl = 2.0 * B * OH * OW * C1 * Cout
        print(f"{name:16s} x{n}: dmc {t_dmc:7.1f} us {fl / t_dmc / 1e6:6.1f} TF/s | mm bf16 {t_mm:7.1f} us "
              f"{fl / t_mm / 1e6:6.1f} TF/s | mm f32-out {t_mm32:7.1f} us (rel diff {err:.1e})", flush=True)
        tot["dmc"] += n * t_dmc
        tot["mm"] += n * t_mm
        tot["mm32"] += n * t_mm32
    print("per step: " + ", ".join(f"{k} {v:.0f} us" for k, v in tot.items()))


if __name__ == "__main__":
    main()
