"""Debug tool (never imported by the package): isolate gn_bwd_fused's accumulate / pixel-sum paths."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from diffusion_models_collection_amd import _lib as L, kernels as K  # noqa: E402


def rel(a, b):
    return ((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-12)).item()


def main():
    dev, dt = "cuda", torch.bfloat16
    N, H, W, C, G = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[2]), int(sys.argv[3]), 8
    HW = H * W
    torch.manual_seed(0)
    x = (torch.randn(N, H, W, C, device=dev) * 1.3 + 0.4).to(dt)
    g = torch.randn(N, H, W, C, device=dev).to(dt)
    gamma = torch.rand(C, device=dev) + 0.5
    beta = torch.randn(C, device=dev)
    _, _, mr = K.gn_stats(dt, x, None, N, HW, C, 0, C, 0, G, 1e-5, gamma, beta)
    prev = torch.randn(N, H, W, C, device=dev).to(dt)
    for fused in (4, 0):
        L.set_option("DMC_GN_BWD_FUSED", fused)
        dg, db = torch.empty(C, device=dev), torch.empty(C, device=dev)
        dx0 = torch.empty_like(x)
        K.gn_bwd(dt, g, C, x, None, N, HW, C, 0, C, 0, G, mr, gamma, beta, True, None, dx0, None, C, 0, 0, 0, dg, db)
        for acc in (0, 1):
            for sums in (0, 1):
                dx = prev.clone() if acc else torch.empty_like(x)
                snc = torch.full((N, C), -7.0, device=dev) if sums else None
                sc_ = torch.empty(C, device=dev) if sums else None
                K.gn_bwd(dt, g, C, x, None, N, HW, C, 0, C, 0, G, mr, gamma, beta, True, None, dx, None, C, 0, acc, 0,
                         dg, db, dx_sum_nc=snc, ld_sum_nc=C, dx_sum_c=sc_)
                torch.cuda.synchronize()
                want = dx0.float() + (prev.float() if acc else 0)
                line = f"fused={fused} acc={acc} sums={sums}: dx {rel(dx, want):.2e}"
                if sums:
                    line += f"  snc {rel(snc, dx.float().sum((1, 2))):.2e}  sc {rel(sc_, dx.float().sum((0, 1, 2))):.2e}"
                print(line, flush=True)


if __name__ == "__main__":
    main()
