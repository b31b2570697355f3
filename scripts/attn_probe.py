"""Time the fused attention kernels on the UNet's shapes (HIP events on the launch stream) and save their outputs
so two builds can be compared bitwise (DMC_LIB selects the build).

    DMC_LIB=... python scripts/attn_probe.py --save gpurun_out/attn_a.pt
    python scripts/attn_probe.py --compare gpurun_out/attn_a.pt gpurun_out/attn_b.pt
"""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

SHAPES = [(128, 256, 4, 64), (128, 64, 4, 64), (128, 16, 4, 64)]


def timeit(fn, iters=50):
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


def run(save, only=0):
    from diffusion_models_collection_amd import kernels as K
    dt, dev = torch.bfloat16, "cuda"
    out = {}
    for (N, L, heads, hd) in SHAPES:
        if only and L != only:
            continue
        C = heads * hd
        g = torch.Generator(device="cpu").manual_seed(L)
        qkv = torch.randn(N, L, 3 * C, generator=g).to(dt).to(dev)
        do = torch.randn(N, L, C, generator=g).to(dt).to(dev)
        od = torch.empty(N, L, C, dtype=dt, device=dev)
        lse = torch.empty(N * heads * L, device=dev)
        dq = torch.empty_like(qkv)
        for drop in (None, (77, 1 << 30, 4.0 / 3.0)):
            K.attn_fwd(dt, qkv, 3 * C, N, L, heads, hd, od, C, lse, drop=drop)
            K.attn_bwd(dt, qkv, 3 * C, od, do, C, lse, N, L, heads, hd, dq, 3 * C, drop=drop)
            torch.cuda.synchronize()
            tag = f"L{L}_{'drop' if drop else 'nodrop'}"
            out[tag] = [od.cpu().clone(), lse.cpu().clone(), dq.cpu().clone()]
        tf = timeit(lambda: K.attn_fwd(dt, qkv, 3 * C, N, L, heads, hd, od, C, lse))
        tb = timeit(lambda: K.attn_bwd(dt, qkv, 3 * C, od, do, C, lse, N, L, heads, hd, dq, 3 * C))
        print(f"N{N} L{L} h{heads} d{hd}: fwd {tf:7.2f} us  bwd (dq + dkdv) {tb:7.2f} us", flush=True)
    if save:
        torch.save(out, save)


def compare(a, b):
    A, B = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    bad = 0
    for k in A:
        for name, u, v in zip(("out", "lse", "dqkv"), A[k], B[k]):
            eq = torch.equal(u, v)
            bad += not eq
            print(f"{k:14s} {name:5s} {'bitwise' if eq else 'DIFFER max %.3g' % (u.float() - v.float()).abs().max()}")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--save")
    ap.add_argument("--compare", nargs=2)
    ap.add_argument("--L", type=int, default=0, help="only this sequence length")
    a = ap.parse_args()
    compare(*a.compare) if a.compare else run(a.save, a.L)
