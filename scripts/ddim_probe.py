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
    a = ap.parse_args()
    from diffusion_models_collection_amd.models import UNet
    from diffusion_models_collection_amd.diffusion import DDIM
    torch.manual_seed(0)
    m = UNet(**CIFAR, compute_dtype="bf16").cuda().eval()
    ddim = DDIM(1000, 50, device="cuda")
    for B in [int(b) for b in a.batches.split(",")]:
        for mode in ("0", "1"):
            os.environ["DMC_GRAPH"] = mode
            with torch.no_grad():
                ddim.sample(m, (B, 3, 32, 32))
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                ddim.sample(m, (B, 3, 32, 32))
                torch.cuda.synchronize()
            el = time.perf_counter() - t0
            print(f"B={B:4d} graph={mode}  {el * 1e3:8.1f} ms  {B / el:8.1f} img/s", flush=True)


if __name__ == "__main__":
    main()
