"""Per-layer conv timing of the bench training step (DMC_LAYER_PROF=1): forward convs, input-gradient convs
(dgrad, tagged conv too: taps/mode tell them apart) and weight gradients, with achieved TF/s.

    DMC_LAYER_PROF=1 python scripts/layer_prof.py [--steps N] [--sample]
"""
import argparse
import os
import sys
from pathlib import Path

os.environ.setdefault("DMC_LAYER_PROF", "1")
os.environ["DMC_GRAPH"] = "0"     # eager steps: the per-call events must not be graph-captured
import torch  # noqa: E402

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from diffusion_models_collection_amd import kernels as K  # noqa: E402
from diffusion_models_collection_amd.models import UNet  # noqa: E402
from diffusion_models_collection_amd.diffusion import DDPM, DDIM  # noqa: E402
from diffusion_models_collection_amd.utils.trainer import DiffusionTrainer  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=3)
ap.add_argument("--sample", action="store_true")
a = ap.parse_args()
dev = torch.device("cuda", 0)
torch.manual_seed(0)
m = UNet(**bench.CIFAR, compute_dtype="bf16").to(dev)
ddpm = DDPM(device=dev)
opt = torch.optim.AdamW(m.parameters(), lr=2e-4, weight_decay=1e-4)
cfg = {"epochs": 1, "save_dir": "/tmp/dmc_lp", "sample_dir": "/tmp/dmc_lp", "use_ema": True, "model_params": dict(bench.CIFAR)}
tr = DiffusionTrainer(m, ddpm, None, opt, None, device=dev, config=cfg)
x = torch.rand(128, 3, 32, 32, device=dev) * 2 - 1
for _ in range(2):
    tr.train_step(x, 0)
torch.cuda.synchronize()
K.PROF.pending = []
if a.sample:
    m.eval()
    with torch.no_grad():
        DDIM(1000, a.steps, device=dev).sample(m, (128, 3, 32, 32))
else:
    for _ in range(a.steps):
        tr.train_step(x, 0)
print(K.PROF.report(a.steps))
