"""Debug the DMC_PRO_GN_SILU small-map conv: NaN pattern by image / channel / pixel on the 4x4 case."""
import math
import sys
import torch
import torch.nn.functional as F
sys.path.insert(0, ".")
from diffusion_models_collection_amd import _lib as L, kernels as K  # noqa: E402

dt = torch.bfloat16
torch.manual_seed(41)
H, N, C1, Cout, G = int(sys.argv[1]) if len(sys.argv) > 1 else 4, 128, 256, 256, 8
x1 = torch.randn(N, C1, H, H) * 1.7 + 0.3
for mode in ("ones", "rand"):
    gamma = torch.ones(C1) if mode == "ones" else torch.rand(C1) + 0.5
    beta = torch.zeros(C1) if mode == "ones" else torch.randn(C1) * 0.3
    xr = x1.to(dt).float()
    a = F.silu(F.group_norm(xr, G, gamma, beta, 1e-5)).to(dt).float()
    w = torch.randn(Cout, C1, 3, 3) / math.sqrt(C1 * 9)
    yr = F.conv2d(a, w.to(dt).float(), padding=1)
    Kc = L.kc_for(C1, dt)
    wp = K.pack_weight(L.PACK_FWD, dt, w.cuda(), Kc)
    d = K.make_desc(dt, N, H, H, C1, 0, C1, 0, Kc, H, H, Cout, K.TAPS3)
    K.set_prologue(d, L.PRO_GN_SILU, gamma.cuda(), beta.cuda(), C1)
    d.pro_groups, d.pro_eps = G, 1e-5
    print("prologue taken", K.conv_halo_prologue(d), "groups", d.pro_groups, "eps", d.pro_eps)
    K.set_epilogue(d, ldy1=Cout)
    y = torch.full((N, H, H, Cout), 7.0, dtype=dt, device="cuda")
    K.conv(d, x1.permute(0, 2, 3, 1).contiguous().to(dt).cuda(), None, wp, y)
    torch.cuda.synchronize()
    got = y.float().cpu().permute(0, 3, 1, 2)
    nan = torch.isnan(got)
    print(mode, "nan frac", nan.float().mean().item(), "per image nan", nan.flatten(1).any(1).sum().item(),
          "err", ((got - yr).abs().max() / yr.abs().max()).item() if not nan.any() else None)
    if nan.any():
        print(" nan images", torch.nonzero(nan.flatten(1).any(1)).flatten()[:20].tolist())
        print(" nan channels", torch.nonzero(nan.transpose(0, 1).flatten(1).any(1)).flatten()[:20].tolist())
