import math, os, sys, ctypes
sys.path.insert(0, os.getcwd())
import torch
from diffusion_models_collection_amd import _lib as L, kernels as K

dev = "cuda"
dt = torch.bfloat16


def run(N, H, W, C1, Cout, stride, split, taps=None):
    torch.manual_seed(0)
    OH, OW = H // stride, W // stride
    x1 = torch.randn(N, H, W, C1, device=dev).to(dt)
    w = torch.randn(Cout, C1, 3, 3, device=dev) / math.sqrt(C1 * 9)
    Kc = L.kc_for(C1, dt)
    wp = K.pack_weight(L.PACK_FWD, dt, w, Kc)
    d = K.make_desc(dt, N, H, W, C1, 0, C1, 0, Kc, OH, OW, Cout, K.TAPS3, L.MODE_NORMAL, stride)
    K.set_epilogue(d, ldy1=Cout)
    y = torch.zeros(N, OH, OW, Cout, dtype=dt, device=dev)
    if split:
        os.environ.pop("DMC_NO_SPLITK", None)
    else:
        os.environ["DMC_NO_SPLITK"] = "1"
    ws = L.LIB.dmc_conv2d_workspace(ctypes.byref(d))
    K.conv(d, x1, None, wp, y)
    torch.cuda.synchronize()
    ref = torch.nn.functional.conv2d(x1.permute(0, 3, 1, 2).float(), w.to(dt).float(), stride=stride, padding=1)
    got = y.permute(0, 3, 1, 2).float()
    err = (got - ref).abs()
    print(f"N={N} H={H} C1={C1} Cout={Cout} s={stride} split={split} ws={ws} maxerr={err.max().item():.4f} "
          f"rel={(err.max() / ref.abs().max()).item():.4f}")
    if err.max() > 0.05 * ref.abs().max():
        bad = err > 0.05 * ref.abs().max()
        print("  bad per oy:", bad.sum(dim=(0, 1, 3)).tolist(), " per ox:", bad.sum(dim=(0, 1, 2)).tolist())
        print("  bad per n:", bad.sum(dim=(1, 2, 3)).tolist(), " per c (first 16):", bad.sum(dim=(0, 2, 3))[:16].tolist())


for split in (False, True):
    run(2, 8, 8, 32, 48, 2, split)
    run(2, 8, 8, 32, 48, 1, split)
    run(2, 8, 8, 64, 48, 2, split)
    run(8, 8, 8, 32, 48, 2, split)
    run(2, 16, 16, 32, 48, 2, split)
    run(2, 8, 8, 32, 128, 2, split)
