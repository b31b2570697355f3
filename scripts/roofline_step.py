"""Measurement tool (never imported by the package): run the bench's B=128 bf16 train step EAGERLY (DMC_GRAPH=0) with
every C-ABI call of diffusion_models_collection_amd.kernels bracketed by a ROCTx range named
    dmc:<op>:<algorithmic FLOP>:<algorithmic HBM bytes>:<shape>
so that `rocprofv3 --kernel-trace --marker-trace --kernel-rename` attributes each dispatch to the op (and its
algorithmic work) that launched it. scripts/kernel_roofline.py aligns that trace by dispatch index with plain kernel
traces / PMC passes of the same command (the eager step's dispatch sequence is deterministic).

Algorithmic work per op (each tensor read or written once; fp32 weight-gradient slabs, split-K partials and re-reads
excluded): conv 2*M*Cout*taps*Cin FLOP, bytes = input + output (+ residual) + packed weights; wgrad the same FLOP,
bytes = dy + x + fp32 dw; GroupNorm stats 1 read, apply 1 read + 1 write (+ the epilogue partials when it finalises), backward x + g read, dx written (+ dx read
when accumulating); attention 4*B*h*L^2*d FLOP forward / 8*B*h*L^2*d backward; AdamW+EMA 36 B per parameter, grad
norm 4 B per parameter; weight pack 4 B read + 2 B written per element.

    rocprofv3 --kernel-trace --marker-trace --kernel-rename -d OUT -o a --output-format csv -- python3 scripts/roofline_step.py
"""
import ctypes
import os
import sys
from pathlib import Path

os.environ["DMC_GRAPH"] = "0"
import torch  # noqa: E402

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
from diffusion_models_collection_amd import _lib as L, kernels as K  # noqa: E402

# the rocprofiler-sdk ROCTx library (rocprofv3 --marker-trace intercepts it; the legacy libroctx64 is not traced)
_rx = None
for _lib in ("/opt/rocm/lib/librocprofiler-sdk-roctx.so.1", "/opt/rocm/lib/librocprofiler-sdk-roctx.so"):
    if os.path.exists(_lib):
        _rx = ctypes.CDLL(_lib)
        break
if _rx is not None:
    _rx.roctxRangePushA.argtypes = [ctypes.c_char_p]


def _esz(dt):
    return 2 if dt == L.dtype_code(torch.bfloat16) else 4


def a_conv(d, x1, x2, w, y1, y2=None):
    M, Cin, e = d.N * d.OH * d.OW, d.C1 + d.C2, _esz(d.dtype)
    f = 2.0 * M * d.Cout * d.ntaps * Cin
    b = d.N * d.H * d.W * Cin * e + M * d.Cout * (4 if d.out_f32 or d.out_nchw else e) + d.Cout * d.ntaps * d.Kc * e
    b += M * d.Cout * e if d.resid else 0
    return f, b, f"N{d.N} {d.H}x{d.W}x{Cin}->{d.OH}x{d.OW}x{d.Cout} t{d.ntaps} m{d.mode}"


def a_wgrad(d, dy, ld_dy, x1, x2, dw, scale=1.0, dbias=None, defer=None):
    M, Cin, e = d.N * d.OH * d.OW, d.C1 + d.C2, _esz(d.dtype)
    f = 2.0 * M * d.Cout * d.ntaps * Cin
    return f, M * d.Cout * e + d.N * d.H * d.W * Cin * e + d.Cout * d.ntaps * Cin * 4, \
        f"N{d.N} {d.H}x{d.W}x{Cin}->{d.OH}x{d.OW}x{d.Cout} t{d.ntaps}"


def a_gn_stats(dtype, x1, x2, N, HW, C1, C2, *a, **k):
    return 0.0, N * HW * (C1 + C2) * x1.element_size(), f"N{N} HW{HW} C{C1 + C2}"


def a_gn_finalize(p1, C1, p2, C2, N, HW, G, *a, **k):
    C = C1 + C2
    return 0.0, N * HW // 64 * C // 8 * 8 + N * C * 8, f"N{N} HW{HW} C{C}"


def a_gn_apply(dtype, x1, x2, N, HW, C1, C2, *a, **k):
    return 0.0, 2 * N * HW * (C1 + C2) * x1.element_size(), f"N{N} HW{HW} C{C1 + C2}"


def a_gn_stats_apply(dtype, x1, x2, N, HW, C1, C2, *a, **k):
    # dmc_gn_stats_apply (4x4 levels): the sample read twice (statistics, then apply) + the output written
    C = C1 + C2
    return 0.0, 3 * N * HW * C * x1.element_size(), f"N{N} HW{HW} C{C}"


def a_gn_bwd(dtype, g, ld_g, x1, x2, N, HW, C1, C2, ld1, ld2, G, mr, gamma, beta, silu, drop, dx1, dx2, ld_dx1,
             ld_dx2, acc1, acc2, *a, **k):
    e = g.element_size()
    b = 3 * N * HW * (C1 + C2) * e + (N * HW * C1 * e if acc1 else 0) + (N * HW * C2 * e if acc2 else 0)
    return 0.0, b, f"N{N} HW{HW} C{C1 + C2} silu{int(silu)} drop{int(drop is not None)}"


def a_attn_fwd(dtype, qkv, ld_qkv, N, Lq, heads, hd, out, ld_out, lse, drop=None):
    e = qkv.element_size()
    return 4.0 * N * heads * Lq * Lq * hd, N * Lq * heads * hd * 4 * e + N * heads * Lq * 4, f"N{N} L{Lq} h{heads}"


def a_attn_bwd(dtype, qkv, ld_qkv, out, dout, ld_out, lse, N, Lq, heads, hd, dqkv, ld_dqkv, drop=None):
    e = qkv.element_size()
    return 8.0 * N * heads * Lq * Lq * hd, N * Lq * heads * hd * 8 * e + N * heads * Lq * 4, f"N{N} L{Lq} h{heads}"


def a_adamw_dev(p, g, m, v, ema, coef, hyper):
    return 0.0, p.numel() * (28 + (8 if ema is not None else 0)), f"n{p.numel()}"


def a_adamw(p, g, m, v, ema, coef, *a):
    return 0.0, p.numel() * (28 + (8 if ema is not None else 0)), f"n{p.numel()}"


def a_grad_norm(g, max_norm):
    return 0.0, g.numel() * 4, f"n{g.numel()}"


def a_gn_none(*a, **k):
    return 0.0, 0.0, ""


def wrap(mod, name, alg):
    fn = getattr(mod, name, None)
    if fn is None:
        return

    def w(*a, **kw):
        f, b, shp = alg(*a, **kw)
        if _rx is not None:
            _rx.roctxRangePushA(f"dmc:{name}:{f:.6g}:{b:.6g}:{shp}".encode())
        try:
            return fn(*a, **kw)
        finally:
            if _rx is not None:
                _rx.roctxRangePop()
    setattr(mod, name, w)


for nm, alg in [("conv", a_conv), ("wgrad", a_wgrad), ("gn_stats", a_gn_stats), ("gn_finalize", a_gn_finalize),
                ("gn_apply", a_gn_apply), ("gn_stats_apply", a_gn_stats_apply), ("gn_bwd", a_gn_bwd), ("attn_fwd", a_attn_fwd), ("attn_bwd", a_attn_bwd),
                ("adamw_flat_dev", a_adamw_dev), ("adamw_flat", a_adamw), ("grad_norm_flat", a_grad_norm), ("pack_input", a_gn_none),
                ("loss_fwd", a_gn_none), ("loss_bwd", a_gn_none), ("add_", a_gn_none), ("upsample2x", a_gn_none),
                ("channel_sum", a_gn_none), ("colsum_batch", a_gn_none), ("time_embed", a_gn_none), ("unpack_output", a_gn_none)]:
    wrap(K, nm, alg)
wrap(K.WgradDefer, "flush", lambda self: (0.0, 0.0, f"jobs{len(self.jobs)}"))   # the batched slab reductions
_launch = K.PackBatch.launch


def _pack_launch(self):
    if _rx is not None:
        _rx.roctxRangePushA(b"dmc:pack_weights:0:0:")
    try:
        _launch(self)
    finally:
        if _rx is not None:
            _rx.roctxRangePop()


K.PackBatch.launch = _pack_launch


def main():
    steps = int(os.environ.get("DMC_RF_STEPS", "3"))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    model, trainer = bench.make_trainer(bench.CIFAR, "bf16", dev, 0, 1)
    gen = torch.Generator(device=dev).manual_seed(1234)
    pool = [torch.rand(128, 3, 32, 32, device=dev, generator=gen) * 2 - 1 for _ in range(2)]
    model.train()
    for i in range(steps):
        trainer.train_step(pool[i % 2], 0)
    torch.cuda.synchronize()
    print("roofline_step done", steps)


if __name__ == "__main__":
    main()
