"""In-kernel s_memtime stamps of conv3x3_halo5_kernel (PROBE 16 / 17 = no MFMA) on the roofline layer."""
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
for probe in (18, 19):
    L.set_option("DMC_HALO_PROBE", probe)
    for _ in range(10):
        y = torch.zeros(B, H, W, Cout, device=dev, dtype=dt)
        K.conv(d, x, None, wp, y)
    torch.cuda.synchronize()
    st = y.view(-1).view(torch.int64)[: 256 * 8 * 4].view(256, 8, 4).double()
    m = st.mean(dim=(0, 1))
    print(f"probe {probe}: cycles per wave: prologue {m[0]:.0f}, stage waits {m[1]:.0f}, main loop {m[2]:.0f} "
          f"(waits {100*m[1]/m[2]:.0f}%), epilogue {m[3]:.0f};  loop max {st[:, :, 2].max():.0f} min {st[:, :, 2].min():.0f}",
          flush=True)
L.set_option("DMC_HALO_PROBE", 0)
