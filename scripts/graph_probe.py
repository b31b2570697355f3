"""Per-step cost of DDIM sampling at B=128: eager vs HIP-graph replay, from the difference of 100- and 50-step runs
(the capture and the first eager step cancel out). Run with DMC_GRAPH=0 / 1."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import CIFAR  # noqa: E402
from diffusion_models_collection_amd.models import UNet  # noqa: E402
from diffusion_models_collection_amd.diffusion import DDIM  # noqa: E402

torch.manual_seed(0)
m = UNet(**CIFAR, compute_dtype="bf16").cuda().eval()
res = {}
with torch.no_grad():
    for S in (50, 100, 50, 100):
        d = DDIM(1000, S, device="cuda")
        d.sample(m, (128, 3, 32, 32))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d.sample(m, (128, 3, 32, 32))
        torch.cuda.synchronize()
        res[S] = time.perf_counter() - t0
print(f"DMC_GRAPH={os.environ.get('DMC_GRAPH')} 50: {res[50]*1e3:.1f} ms 100: {res[100]*1e3:.1f} ms "
      f"per step {(res[100]-res[50])/50*1e3:.3f} ms")
