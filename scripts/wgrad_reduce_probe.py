"""Time dmc_wgrad_reduce_batch alone on the weight-gradient jobs of one B=128 CIFAR train step (scripts/wgrad_sweep.py
SHAPES with their per-step counts): the partial-sum kernels run once into a WgradDefer arena, then the same job list
is reduced `iters` times (<= 32 jobs per launch, HIP events around the batches). Reports the slab bytes the
reductions read and the rate.

    DMC_LIB=... python scripts/wgrad_reduce_probe.py [--iters N]
"""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parent))
from diffusion_models_collection_amd import _lib as L, kernels as K  # noqa: E402
from wgrad_sweep import SHAPES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dt, dev = torch.bfloat16, "cuda"
    defer = K.WgradDefer()
    defer.buf = torch.empty(int(4.2e9), dtype=torch.uint8, device=dev)   # every job of the step in one arena
    keep = []
    for name, (B, H, W, C1, C2, Cout, taps, OH, OW, mode, stride, n) in SHAPES.items():
        ldx = 8 if C1 < 8 else C1
        x1 = torch.randn(B, H, W, ldx, device=dev).to(dt)
        x2 = torch.randn(B, H, W, C2, device=dev).to(dt) if C2 else None
        ldy = max(Cout, 8)
        dy = torch.randn(B, OH, OW, ldy, device=dev).to(dt)
        kh = 3 if len(taps) == 9 else 1
        d = K.make_desc(dt, B, H, W, C1, C2, ldx, C2, L.kc_for(C1 + C2, dt), OH, OW, Cout, taps, mode, stride)
        for _ in range(n):
            dw = torch.empty(Cout, C1 + C2, kh, kh, device=dev)
            db = torch.empty(Cout, device=dev)
            K.wgrad(d, dy, ldy, x1, x2, dw, dbias=db, defer=defer)
            keep.append((dw, db, d))
    jobs = list(defer.jobs)
    nbytes = sum(j.splits * (j.KK * ((j.Cout + 3) // 4) * 16 + (j.Cout * 4 if j.dbias else 0)) for j in jobs)
    wbytes = sum(j.Cout * j.Ctot * j.ntaps * 4 for j in jobs)

    def run():
        for k in range(0, len(jobs), 32):
            chunk = jobs[k:k + 32]
            arr = (L.WgradJob * len(chunk))(*chunk)
            L.check(L.LIB.dmc_wgrad_reduce_batch(arr, len(chunk), L.stream()), "reduce")

    run()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(a.iters):
        run()
    e1.record(s)
    e1.synchronize()
    t = e0.elapsed_time(e1) / a.iters * 1e3
    print(f"{len(jobs)} jobs, {(len(jobs) + 31) // 32} launches: {t:.1f} us per step; slab read {nbytes / 1e9:.3f} GB "
          f"({nbytes / t / 1e6:.2f} TB/s), dw written {wbytes / 1e6:.1f} MB", flush=True)


if __name__ == "__main__":
    main()
