import sys, torch
sys.path.insert(0, '.')
from diffusion_models_collection_amd.models import UNet
from diffusion_models_collection_amd.diffusion import DDPM
DEV = "cuda"
cfg = dict(image_size=(32, 32), in_channels=3, model_channels=128, out_channels=3, num_res_blocks=2,
           attention_resolutions=(16, 8), dropout=0.0, channel_mult=(1, 2, 2, 2), num_classes=None, use_attention=True)
gen = torch.Generator().manual_seed(17)
x0 = (torch.rand(128, 3, 32, 32, generator=gen) * 2 - 1).to(DEV)
t = torch.randint(0, 1000, (128,), generator=gen).to(DEV)
noise = torch.randn(128, 3, 32, 32, generator=gen).to(DEV)
ddpm = DDPM(device=DEV)
for dtype in sys.argv[1:]:
    for B in (128, 64, 32):
        torch.manual_seed(42)
        m = UNet(**cfg, compute_dtype=dtype).to(DEV).train()
        loss = ddpm.p_losses(m, x0[:B], t[:B], noise=noise[:B])
        loss.backward()
        bad = [k for k, p in m.named_parameters() if not torch.isfinite(p.grad).all()]
        print(dtype, B, 'loss', loss.item(), 'nonfinite grads', len(bad), bad[:6], flush=True)
        del m
