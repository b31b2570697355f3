"""Narrow down the capture_end segfault of test_dropped_model_frees_without_cyclic_gc[unet] (round 6).

python scripts/r6_drop_repro.py <gc:on|off> <presample:0|1> <drop:0|1>
Prints a line per phase, so the last line before a crash names the phase."""
import gc
import sys
import weakref

import ctypes
import torch

ctypes.CDLL('scripts/probe/segv_bt.so')   # native backtrace on a crash
sys.path.insert(0, ".")
from diffusion_models_collection_amd.models import UNet  # noqa: E402
from diffusion_models_collection_amd.diffusion import DDIM, DDPM  # noqa: E402
from diffusion_models_collection_amd.utils.trainer import DiffusionTrainer  # noqa: E402

gc_mode, presample, drop = sys.argv[1], sys.argv[2] == "1", sys.argv[3] == "1"
DEV = "cuda"
up = dict(image_size=(16, 16), in_channels=3, model_channels=32, out_channels=3, num_res_blocks=1,
          attention_resolutions=(8,), dropout=0.1, channel_mult=(1, 2), use_attention=True)


def make():
    torch.manual_seed(0)
    return UNet(**up, compute_dtype="bf16").to(DEV)


def say(*a):
    print(*a, flush=True)


if gc_mode == "off":
    gc.disable()
ddim = DDIM(1000, 4, device=DEV)
m = make().eval()
if presample:
    with torch.no_grad():
        ddim.sample(m, (4, 3, 16, 16))
    torch.cuda.synchronize()
    say("presampled, graphs", len(getattr(ddim, "_step_graphs", {})))
if drop:
    wm = weakref.ref(m)
    del m
    say("dropped, alive:", wm() is not None)
m2 = make()
opt = torch.optim.AdamW(m2.parameters(), lr=1e-4)
cfg = {"epochs": 1, "save_dir": "/tmp/r6c", "sample_dir": "/tmp/r6s", "loss_type": "l2",
       "use_ema": True, "ema_decay": 0.99, "model_type": "unet", "model_params": dict(up)}
tr = DiffusionTrainer(m2, DDPM(device=DEV), None, opt, None, device=DEV, config=cfg)
m2.train()
gen = torch.Generator().manual_seed(3)
for i in range(4):
    say("step", i)
    loss = tr.train_step((torch.rand(4, 3, 16, 16, generator=gen) * 2 - 1).to(DEV), i)
    torch.cuda.synchronize()
    say("step", i, "done", float(loss))
say("OK", gc_mode, presample, drop)
