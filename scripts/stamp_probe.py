"""Phase clocks of conv3x3_halo2_kernel's tap loop on the roofline layer (3x3 128->128 @32x32, B=128), from the
DMC_STAMP measurement build (scripts/stamp_build.sh). Per wave: clocks spent waiting for the weight slice / halo,
in the block barrier, issuing the next slice's LDS-DMA, issuing the fragment reads + MFMAs, and the tail."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["DMC_LIB"] = os.path.join(ROOT, "stamp_lib", "libdmc_stamp.so")
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from diffusion_models_collection_amd import _lib as L, kernels as K  # noqa: E402

dt = torch.bfloat16
B, H, W, C, Cout = 128, 32, 32, 128, 128
x = torch.randn(B, H, W, C, device="cuda").to(dt)
w = torch.randn(Cout, C, 3, 3, device="cuda") * 0.03
Kc = L.kc_for(C, dt)
wp = K.pack_weight(L.PACK_FWD, dt, w, Kc)
y = torch.empty(B, H, W, Cout, device="cuda", dtype=dt)
nblk = B * H * W // 128
stamp = torch.zeros(nblk * 4 * 8, dtype=torch.int64, device="cuda")
for _ in range(3):
    d = K.make_desc(dt, B, H, W, C, 0, C, 0, Kc, H, W, Cout, K.TAPS3)
    K.set_epilogue(d, bias=torch.zeros(Cout, device="cuda"), ldy1=Cout)
    K.conv(d, x, None, wp, y)
L.set_option("DMC_STAMP_PTR", stamp.data_ptr())
d = K.make_desc(dt, B, H, W, C, 0, C, 0, Kc, H, W, Cout, K.TAPS3)
K.set_epilogue(d, bias=torch.zeros(Cout, device="cuda"), ldy1=Cout)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
K.conv(d, x, None, wp, y)
e1.record()
torch.cuda.synchronize()
L.set_option("DMC_STAMP_PTR", 0)
ms = e0.elapsed_time(e1)
s = stamp.view(nblk * 4, 8).cpu().double()
ph = s[:, :5]
life = s[:, 6] - s[:, 5]
t0, t1 = s[:, 5].min(), s[:, 6].max()
print(f"kernel {ms * 1e3:.1f} us (events); s_memtime span {t1 - t0:.0f} ticks -> {(t1 - t0) / (ms * 1e3):.1f} ticks/us")
tot = ph.sum(1)
names = ["wait (slice/halo)", "barrier", "DMA issue", "reads+MFMA issue", "tail+epi barrier"]
for i, n in enumerate(names):
    print(f"  {n:20s} mean {ph[:, i].mean():9.1f} ticks  {100 * (ph[:, i] / tot).mean():5.1f} % of the loop")
print(f"  wave lifetime (loop + tail) mean {life.mean():.0f} ticks, taps per wave {int(s[0, 7])}")
