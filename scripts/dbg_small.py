"""Debug: where does the small-map kernel differ from the split-K path (4x4 shapes)."""
import math, sys
from pathlib import Path
import torch
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from diffusion_models_collection_amd import _lib as L, kernels as K  # noqa: E402

dt = torch.bfloat16
DEV = "cuda"
for (H, Cin, Cout, dg) in [(4, 256, 512, True), (4, 256, 256, True), (4, 256, 512, False), (8, 256, 512, True)]:
    torch.manual_seed(9)
    N = 128
    taps, pm = (K.TAPS3_DGRAD, L.PACK_DGRAD) if dg else (K.TAPS3, L.PACK_FWD)
    x = torch.randn(N, H, H, Cin, device=DEV).to(dt)
    w = (torch.randn(Cin, Cout, 3, 3) if dg else torch.randn(Cout, Cin, 3, 3)) / math.sqrt(Cin * 9)
    wp = K.pack_weight(pm, dt, w.to(DEV), L.kc_for(Cin, dt))
    outs = []
    for ns in (0, 1):
        L.set_option("DMC_NO_SMALL", ns)
        d = K.make_desc(dt, N, H, H, Cin, 0, Cin, 0, L.kc_for(Cin, dt), H, H, Cout, taps)
        K.set_epilogue(d, ldy1=Cout)
        y = torch.full((N, H, H, Cout), float("nan"), dtype=dt, device=DEV)
        K.conv(d, x, None, wp, y)
        torch.cuda.synchronize()
        outs.append(y.float().cpu())
    diff = (outs[0] - outs[1]).abs()
    bad = diff > 0.05 * outs[1].abs().max()
    print(H, Cin, Cout, "dgrad" if dg else "fwd", "bad", int(bad.sum()), "of", bad.numel(), "nan", int(outs[0].isnan().sum()))
    if bad.any():
        idx = bad.nonzero()
        print("  images", sorted(set(idx[:, 0].tolist()))[:20], "rows", sorted(set(idx[:, 1].tolist())),
              "cols", sorted(set(idx[:, 2].tolist())), "ch", sorted(set((idx[:, 3] // 64).tolist())))
        print("  ch mod 64", sorted(set((idx[:, 3] % 64).tolist()))[:70])
L.reset_options(from_env=False)
