"""Ablation of the round-2 halo conv (conv3x3_halo4_kernel PROBE instantiations) on the roofline layer."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from diffusion_models_collection_amd import _lib as L, kernels as K  # noqa: E402
L.set_option("DMC_HALO_VER", 5)

B, H, W, C, Cout = 128, 32, 32, 128, 128
dt, dev = torch.bfloat16, "cuda"
x = torch.randn(B, H, W, C, device=dev).to(dt)
w = torch.randn(Cout, C, 3, 3, device=dev) * 0.03
wp = K.pack_weight(L.PACK_FWD, dt, w, C)
d = K.make_desc(dt, B, H, W, C, 0, C, 0, C, H, W, Cout, K.TAPS3)
K.set_epilogue(d, bias=torch.randn(Cout, device=dev), addvec=torch.randn(B, Cout, device=dev), ld_add=Cout, ldy1=Cout)
y = torch.empty(B, H, W, Cout, device=dev, dtype=dt)
names = {0: "full", 1: "no MFMA", 2: "no epilogue stores", 4: "no loop DMA", 3: "no MFMA, no stores"}
_unused = {0: "full", 1: "no MFMA", 2: "no epilogue stores", 4: "no loop DMA", 8: "no loop barrier",
         3: "no MFMA, no stores", 5: "no MFMA, no DMA", 7: "no MFMA/stores/DMA", 16: "no LDS reads",
         23: "no reads/MFMA/stores/DMA", 32: "no main loop", 34: "no main loop/stores"}
for p in [int(a) for a in sys.argv[1:]] or (0, 1, 2, 4, 8, 3, 5, 7, 16, 23, 32, 34):
    L.set_option("DMC_HALO_PROBE", p)
    for _ in range(3):
        K.conv(d, x, None, wp, y)
    s = torch.cuda.current_stream()
    n = 20
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * n)]
    for i in range(n):
        ev[2 * i].record(s)
        K.conv(d, x, None, wp, y)
        ev[2 * i + 1].record(s)
    ev[-1].synchronize()
    ms = sum(ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(n)) / n
    print(f"probe {p} ({names[p]:22s}): {ms*1e3:7.1f} us", flush=True)
L.set_option("DMC_HALO_PROBE", 0)
