"""DDIM-50 sampling throughput of the CIFAR UNet (bf16) per batch size, eager step loop vs the step graph.

    python scripts/ddim_probe.py [--batches 8,32,128]
"""
import argparse
import os
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from bench import CIFAR  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="8,32,128")
    ap.add_argument("--host", action="store_true", help="also time the host enqueue of one UNet forward (no sync)")
    a = ap.parse_args()
    from diffusion_models_collection_amd.models import UNet
    from diffusion_models_collection_amd.diffusion import DDIM
    torch.manual_seed(0)
    m = UNet(**CIFAR, compute_dtype="bf16").cuda().eval()
    ddim = DDIM(1000, 50, device="cuda")
    for B in [int(b) for b in a.batches.split(",")]:
        for mode in ("0", "1"):
            os.environ["DMC_GRAPH"] = mode
            els = []
            with torch.no_grad():
                for _ in range(3):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    ddim.sample(m, (B, 3, 32, 32))
                    torch.cuda.synchronize()
                    els.append(time.perf_counter() - t0)
            print(f"B={B:4d} graph={mode}  calls " + " ".join(f"{e * 1e3:7.1f}" for e in els)
                  + f" ms  (last {B / els[-1]:7.1f} img/s)", flush=True)
        if a.host:
            x = torch.randn(B, 3, 32, 32, device="cuda")
            t = torch.full((B,), 500, dtype=torch.long, device="cuda")
            with torch.no_grad():
                for _ in range(3):
                    m(x, t[:1], None)
                torch.cuda.synchronize()
                hs = []
                for _ in range(5):
                    t0 = time.perf_counter()
                    m(x, t[:1], None)
                    hs.append(time.perf_counter() - t0)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(10):
                    m(x, t[:1], None)
                torch.cuda.synchronize()
                gpu = (time.perf_counter() - t0) / 10
            print(f"B={B:4d} forward: host enqueue {min(hs) * 1e3:.3f} ms (min of 5), back-to-back {gpu * 1e3:.3f} ms",
                  flush=True)


if __name__ == "__main__":
    main()
