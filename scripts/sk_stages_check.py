"""Split-K ring depth (DMC_SK_STAGES 0 / 4 / 5): the small-map convs give bitwise the same output (same split
ranges and summation order, only the DMA lookahead differs); prints the per-launch time of each."""
import ctypes
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from diffusion_models_collection_amd import _lib as L, kernels as K  # noqa: E402


def main():
    dt, dev = torch.bfloat16, "cuda"
    for (B, H, C1, C2, Cout) in ((128, 4, 256, 0, 256), (128, 4, 256, 256, 256), (128, 8, 256, 256, 256)):
        torch.manual_seed(0)
        x1 = torch.randn(B, H, H, C1, device=dev).to(dt)
        x2 = torch.randn(B, H, H, C2, device=dev).to(dt) if C2 else None
        w = torch.randn(Cout, C1 + C2, 3, 3, device=dev) * 0.03
        Kc = L.kc_for(C1 + C2, dt)
        wp = K.pack_weight(L.PACK_FWD, dt, w, Kc)
        d = K.make_desc(dt, B, H, H, C1, C2, C1, C2, Kc, H, H, Cout, K.TAPS3)
        K.set_epilogue(d, bias=torch.randn(Cout, device=dev), ldy1=Cout)
        outs = {}
        for st in (0, 4, 5):
            L.set_option("DMC_SK_STAGES", st)
            y = torch.full((B, H, H, Cout), float("nan"), device=dev).to(dt)
            K.conv(d, x1, x2, wp, y)
            s = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(50):
                K.conv(d, x1, x2, wp, y)
            e1.record(s)
            e1.synchronize()
            outs[st] = y.clone()
            print(f"B{B} {H}x{H} {C1}+{C2}->{Cout} SK_STAGES={st}: {e0.elapsed_time(e1) / 50 * 1e3:.1f} us", flush=True)
        L.set_option("DMC_SK_STAGES", 0)
        for st in (4, 5):
            assert torch.equal(outs[st], outs[0]), st
            assert not torch.isnan(outs[st].float()).any()
    print("bitwise OK")


if __name__ == "__main__":
    main()
