"""A/B of the bf16 3x3 halo conv kernels on the UNet's layer shapes: round-2 4-wave kernel vs round-1 8-wave
kernel (DMC_HALO_V1), per-launch HIP-event timing and the max difference of their outputs."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from diffusion_models_collection_amd import _lib as L, kernels as K  # noqa: E402

SHAPES = {  # name: (B, H, W, C1, C2, Cout, epilogue)
    "r128_32": (128, 32, 32, 128, 0, 128, "temb"),
    "r128_32_full": (128, 32, 32, 128, 0, 128, "full"),
    "r384_32": (128, 32, 32, 256, 128, 128, "temb"),
    "r256_16": (128, 16, 16, 256, 0, 256, "temb"),
    "r512_16": (128, 16, 16, 256, 256, 256, "temb"),
    "r512_8": (128, 8, 8, 256, 256, 256, "temb"),
    "r128_64": (32, 64, 64, 128, 0, 128, "temb"),
}


def run(name, iters=30):
    B, H, W, C1, C2, Cout, epi = SHAPES[name]
    dt, dev = torch.bfloat16, "cuda"
    torch.manual_seed(0)
    x1 = torch.randn(B, H, W, C1, device=dev).to(dt)
    x2 = torch.randn(B, H, W, C2, device=dev).to(dt) if C2 else None
    w = torch.randn(Cout, C1 + C2, 3, 3, device=dev) * 0.03
    Kc = L.kc_for(C1 + C2, dt)
    wp = K.pack_weight(L.PACK_FWD, dt, w, Kc)
    d = K.make_desc(dt, B, H, W, C1, C2, C1, C2, Kc, H, W, Cout, K.TAPS3)
    resid = torch.randn(B, H, W, Cout, device=dev).to(dt) if epi == "full" else None
    K.set_epilogue(d, bias=torch.randn(Cout, device=dev), addvec=torch.randn(B, Cout, device=dev), ld_add=Cout,
                   resid=resid, ld_res=Cout if resid is not None else 0, ldy1=Cout)
    res = {}
    for v1 in (0, 1, 2):
        L.set_option("DMC_HALO_VER", {0: 5, 1: 1, 2: 4}[v1])
        y = torch.full((B, H, W, Cout), float("nan"), device=dev, dtype=dt)
        for _ in range(3):
            K.conv(d, x1, x2, wp, y)
        s = torch.cuda.current_stream()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * iters)]
        for i in range(iters):
            ev[2 * i].record(s)
            K.conv(d, x1, x2, wp, y)
            ev[2 * i + 1].record(s)
        ev[-1].synchronize()
        ms = sum(ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(iters)) / iters
        res[v1] = (ms, y.float())
    ws = L.get_option("DMC_HALO_WS")
    L.reset_options()
    L.set_option("DMC_HALO_WS", ws)
    fl = 2.0 * B * H * W * Cout * (C1 + C2) * 9
    diff = ((res[0][1] - res[1][1]).abs().max() / res[1][1].abs().max()).item()
    nan = bool(torch.isnan(res[0][1]).any())
    print(f"{name:14s} v5 {res[0][0]*1e3:7.1f} us ({fl/res[0][0]/1e9:5.0f} TF/s)  v4 {res[2][0]*1e3:6.1f} us  "
          f"r1 {res[1][0]*1e3:6.1f} us ({fl/res[1][0]/1e9:5.0f} TF/s)  rel diff {diff:.2e} nan {nan}", flush=True)


if __name__ == "__main__":
    for n in (sys.argv[1:] or SHAPES):
        run(n)
