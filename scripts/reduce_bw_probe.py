"""Bandwidth of dmc_wgrad_reduce_batch (dw-shaped slab, layout 1) against torch's sum over the split dimension and
a plain copy, on synthetic slabs of the step's typical shapes: [splits][Cout * Ctot * ntaps] fp32.

    python scripts/reduce_bw_probe.py
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from diffusion_models_collection_amd import _lib as L  # noqa: E402


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    dev = "cuda"
    for splits, Cout, Ctot, ntaps, njobs in [(64, 128, 128, 9, 1), (16, 256, 256, 9, 1), (8, 256, 512, 9, 1),
                                             (16, 256, 256, 9, 8), (64, 128, 128, 9, 8), (32, 256, 256, 1, 8)]:
        n = Cout * Ctot * ntaps
        slabs = [torch.randn(splits, n, device=dev) for _ in range(njobs)]
        dws = [torch.empty(n, device=dev) for _ in range(njobs)]
        arr = (L.WgradJob * njobs)()
        for i in range(njobs):
            j = arr[i]
            j.slab, j.bslab, j.dw, j.dbias = slabs[i].data_ptr(), None, dws[i].data_ptr(), None
            j.splits, j.KK, j.Cpad, j.Cout, j.Ctot, j.ntaps, j.Kc = splits, ntaps * Ctot, Cout, Cout, Ctot, ntaps, Ctot
            j.scale, j.layout = 1.0, 1

        def ours():
            L.check(L.LIB.dmc_wgrad_reduce_batch(arr, njobs, L.stream()), "reduce")

        def tsum():
            for i in range(njobs):
                torch.sum(slabs[i], 0, out=dws[i])

        big = torch.empty(splits * n * njobs, device=dev)
        big2 = torch.empty_like(big)
        nb = splits * n * 4 * njobs
        t0, t1, t2 = timeit(ours), timeit(tsum), timeit(lambda: big2.copy_(big))
        ours()
        ref = slabs[0].sum(0)
        err = ((dws[0] - ref).abs().max() / ref.abs().max()).item()
        print(f"splits {splits:3d} x {n:8d} x{njobs}: ours {t0:7.1f} us {nb / t0 / 1e6:5.2f} TB/s | torch.sum "
              f"{t1:7.1f} us {nb / t1 / 1e6:5.2f} TB/s | copy {t2:7.1f} us {2 * nb / t2 / 1e6:5.2f} TB/s r+w "
              f"(max rel diff {err:.1e})", flush=True)
        del slabs, big, big2


if __name__ == "__main__":
    main()
