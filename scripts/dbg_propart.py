"""Debug tool (never imported by the package): DMC_PRO_GN_SILU vs dmc_gn_finalize + DMC_PRO_AFFINE_SILU on the
UNet's shapes at B=128, and the model output with the executor switch on / off."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from diffusion_models_collection_amd import _lib as L, kernels as K  # noqa: E402


def kernel_case(N, H, C1, C2, Cout, G=8):
    dt, dev = torch.bfloat16, "cuda"
    torch.manual_seed(3)
    Cin = C1 + C2
    x1 = (torch.randn(N, H, H, C1, device=dev) * 1.3 + 0.2).to(dt)
    x2 = (torch.randn(N, H, H, C2, device=dev) * 0.7 - 0.1).to(dt) if C2 else None
    gamma, beta = torch.rand(Cin, device=dev) + 0.5, torch.randn(Cin, device=dev)
    w = torch.randn(Cout, Cin, 3, 3, device=dev) * 0.02
    Kc = L.kc_for(Cin, dt)
    wp = K.pack_weight(L.PACK_FWD, dt, w, Kc)

    def parts(t, C_):
        v = t.float().reshape(N * H * H // 64, 64, C_ // 8, 8).permute(0, 2, 1, 3).reshape(-1, C_ // 8, 512)
        mu = v.mean(-1)
        return torch.stack([mu, ((v - mu[..., None]) ** 2).sum(-1)], -1).contiguous()
    p1 = parts(x1, C1)
    p2 = parts(x2, C2) if C2 else None
    sc, sh, _ = K.gn_finalize(p1, C1, p2, C2, N, H * H, G, 1e-5, gamma, beta)
    outs = []
    for mode in (0, 1):
        d = K.make_desc(dt, N, H, H, C1, C2, C1, C2, Kc, H, H, Cout, K.TAPS3)
        if mode == 0:
            K.set_prologue(d, L.PRO_AFFINE_SILU, sc, sh, Cin)
        else:
            K.set_prologue_gn(d, p1, p2, G, 1e-5, gamma, beta)
        K.set_epilogue(d, bias=torch.zeros(Cout, device=dev), ldy1=Cout)
        y = torch.full((N, H, H, Cout), float("nan"), device=dev).to(dt)
        K.conv(d, x1, x2, wp, y)
        outs.append(y)
    torch.cuda.synchronize()
    diff = (outs[0].float() - outs[1].float()).abs()
    print(f"kernel N{N} {H}x{H} {C1}+{C2}->{Cout}: equal={torch.equal(outs[0], outs[1])} maxdiff={diff.max().item():.3e} "
          f"bad_frac={(diff > 0).float().mean().item():.2e}", flush=True)
    if not torch.equal(outs[0], outs[1]):
        bad = (diff > 0).nonzero()
        print("   first bad (n, y, x, co):", bad[:4].tolist(), " images with diffs:", bad[:, 0].unique().numel(),
              " rows:", bad[:, 1].unique().tolist()[:20], flush=True)


def main():
    for case in ((128, 32, 128, 128, 128), (128, 32, 128, 0, 128), (128, 32, 256, 0, 128), (128, 32, 128, 128, 256),
                 (128, 16, 256, 128, 256), (128, 16, 128, 256, 256), (128, 32, 256, 128, 256)):
        kernel_case(*case)


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def model_bisect():
    """Allow the in-conv GroupNorm combine for one eligible conv at a time; report which ones change the output."""
    from diffusion_models_collection_amd.models import UNet
    from diffusion_models_collection_amd.models import _unet_exec as E
    L.set_option("DMC_REG_EPI", 2)
    torch.manual_seed(42)
    cfg = dict(image_size=(32, 32), in_channels=3, model_channels=128, out_channels=3, num_res_blocks=2,
               attention_resolutions=(16, 8), dropout=0.1, channel_mult=(1, 2, 2, 2), num_classes=None,
               use_attention=True)
    m = UNet(**cfg, compute_dtype="bf16").cuda().eval()
    x = torch.randn(128, 3, 32, 32, device="cuda")
    t = torch.randint(0, 1000, (128,), device="cuda")
    orig = E.UNetExecutor._pro_gn
    state = {"i": 0, "allow": -1, "info": []}

    def limited(self, srcs, gn, Cout):
        r = orig(self, srcs, gn, Cout)
        if r is None:
            return None
        i = state["i"]
        state["i"] += 1
        state["info"].append((i, srcs[0].H, srcs[0].C, srcs[1].C if len(srcs) > 1 else 0, Cout))
        return r if i == state["allow"] else None
    E.UNetExecutor._pro_gn = limited
    with torch.no_grad():
        ref = m(x, t).clone()
    n = state["i"]
    info = list(state["info"])
    print("eligible convs:", n, flush=True)
    for k in range(n):
        state.update(i=0, allow=k, info=[])
        with torch.no_grad():
            out = m(x, t)
        d = (out - ref).abs().max().item()
        print(f"  allow #{k} {info[k]}: maxdiff {d:.3e}", flush=True)
    E.UNetExecutor._pro_gn = orig


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "model":
    model_bisect()
