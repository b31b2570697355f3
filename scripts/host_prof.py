"""Host-side cost of one bench training step: cProfile over K steps of DiffusionTrainer.train_step.

bench.py reports host_enqueue_ms_per_step next to ms_per_step; when the two are close the step is bound by
Python/ctypes launch work, and this shows where it goes.
    python scripts/host_prof.py [--steps K] [--top N]
"""
import argparse
import cProfile
import io
import pstats
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from bench import CIFAR  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--top", type=int, default=45)
    a = ap.parse_args()
    from diffusion_models_collection_amd.models import UNet
    from diffusion_models_collection_amd.diffusion import DDPM
    from diffusion_models_collection_amd.utils.trainer import DiffusionTrainer
    dev = torch.device("cuda", 0)
    torch.manual_seed(42)
    model = UNet(**CIFAR, compute_dtype="bf16").to(dev)
    ddpm = DDPM(1000, 1e-4, 0.02, "linear", device=dev)
    opt = torch.optim.AdamW(model.parameters(), lr=2e-4, weight_decay=1e-4)
    cfg = {"epochs": 1, "save_dir": "/tmp/dmc_hp_ckpt", "sample_dir": "/tmp/dmc_hp_smp", "loss_type": "l2",
           "use_ema": True, "ema_decay": 0.9999, "model_type": "unet", "model_params": dict(CIFAR)}
    tr = DiffusionTrainer(model, ddpm, None, opt, None, device=dev, config=cfg)
    x = torch.rand(128, 3, 32, 32, device=dev) * 2 - 1
    model.train()
    for _ in range(5):
        tr.train_step(x, 0)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.steps):
        tr.train_step(x, 0)
    pr.disable()
    torch.cuda.synchronize()
    for key in ("tottime", "cumulative"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(a.top)
        print(s.getvalue(), flush=True)


if __name__ == "__main__":
    main()
