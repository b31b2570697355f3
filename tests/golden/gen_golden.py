"""Generate the golden fixtures under tests/golden/ from the REFERENCE implementation.

Run ONLY in the build container (where /root/reference exists):

    python tests/golden/gen_golden.py

It imports sunyzhi55/Diffusion_Models_Collection from /root/reference (read-only, never shipped),
runs it on CPU in fp32 and writes small .npz fixtures: inputs and expected outputs only.
The GPU box never runs this script; the tests only read the .npz files it wrote.

Fixture list (every array is float32 / int64 data, loaded with numpy.load(allow_pickle=False)):
  schedules.npz      DDPM/DDIM tables for linear/cosine/quadratic (diffusion/ddpm.py:38-71)
                     and DDIM inference timesteps (diffusion/ddim.py:71-85)
  unet_tiny_*.npz    tiny UNet (models/unet.py) weights, input, output, and the gradients of
                     sum(out * cot) w.r.t. every parameter and x
  diffusion_ops.npz  q_sample, p_losses (l1/l2/huber), DDPM p_sample (injected noise),
                     DDIM p_sample / sample trajectory (injected x_T), CFG+dynamic-threshold step
  trainer_traj.npz   5 DiffusionTrainer steps (dropout 0, injected t/noise), per-step loss,
                     final parameters and EMA
  ddpm_sample.npz    DDPM.sample and DDPM.sample_with_cfg (diffusion/ddpm.py:222-332) on the tiny
                     conditional UNet, T=1000, injected x_T and per-step z (numpy PCG64 standard normals,
                     regenerated from their seeds by the tests); snapshots every 100 steps + final
  unet_mnist.npz     full-width UNet at the MNIST shape (1x28x28, channel_mult=(1,2,2), 128 channels,
                     BASELINE config #1) and
  unet_64.npz        the CIFAR UNet params at 64x64 (BASELINE config #5): weights are NOT stored (the
                     build's UNet reproduces the reference's initialisation from torch.manual_seed(1234);
                     per-parameter checksums pin that), input, output, grad_x in full, and per parameter
                     gradient sum / sum of squares / absmax plus 32 sampled entries
  trainer_ckpt.pth   the reference's own save_checkpoint() dict after 2 trainer steps (tensors, numbers,
                     strings and the config dict only: loads with torch.load(weights_only=True))
  ckpt_resume.npz    the inputs of a 3rd step and the reference's loss / parameters / EMA after resuming
                     from trainer_ckpt.pth and running it
  dit_tiny_*.npz     tiny DiTs (models/dit.py; patch 2 conditional, patch 4 unconditional), parameters
                     perturbed away from the zero adaLN init, input, output (and the y=None output), the
                     gradients of sum(out * cot) w.r.t. every parameter and x
  dit_s2.npz         DiT-S/2 at 32x32 (BASELINE config #4): weights NOT stored (seed + perturbation are
                     reproduced, per-tensor checksums pin them), output, grad_x, gradient summaries
  trainer_1k.npz     north_star "p_losses ... over 1k steps": the reference DiffusionTrainer for 1000 steps on the
                     tiny unconditional UNet (dropout 0; inputs = numpy PCG64 draws from stored seeds), every
                     step's loss, theta_k at k = 0/250/500/750 with the step-k gradient summaries, AdamW moments
                     at k = 500, final parameter / EMA sums, and the same run on one host thread (losses_alt)
"""
import os
import sys
import types
from pathlib import Path

import numpy as np
import torch

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent

# utils/trainer.py imports swanlab and torchvision.utils.save_image (both absent here; ordinary
# ImportError). Stub them so the trainer module imports.
sys.modules.setdefault("swanlab", types.ModuleType("swanlab"))
if "torchvision" not in sys.modules:
    tv = types.ModuleType("torchvision")
    tvu = types.ModuleType("torchvision.utils")
    tvu.save_image = lambda *a, **k: None
    tv.utils = tvu
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.utils"] = tvu
sys.path.insert(0, str(REF))

from models.unet import UNet  # noqa: E402  (reference)
from diffusion.ddpm import DDPM  # noqa: E402
from diffusion.ddim import DDIM  # noqa: E402

torch.set_num_threads(8)
torch.use_deterministic_algorithms(False)

TINY_CFGS = {
    # 16x16, 2 levels: covers 3x3/1x1/stride-2/upsample convs, concat with a GN group that
    # straddles the two sources (96 = 64 + 32 channels, 12 per group), attention at 8x8.
    "unet_tiny_uncond": dict(image_size=(16, 16), in_channels=3, model_channels=16, out_channels=3,
                             num_res_blocks=1, attention_resolutions=(8,), dropout=0.0,
                             channel_mult=(1, 2), num_classes=None, use_attention=True),
    "unet_tiny_cond": dict(image_size=(16, 16), in_channels=3, model_channels=16, out_channels=3,
                           num_res_blocks=1, attention_resolutions=(8,), dropout=0.0,
                           channel_mult=(1, 2), num_classes=10, use_attention=True),
    # 3 levels down to 4x4 (attention at 8x8 and at 4x4 in the middle), 1 input channel
    "unet_tiny_l3": dict(image_size=(16, 16), in_channels=1, model_channels=16, out_channels=1,
                         num_res_blocks=2, attention_resolutions=(8, 4), dropout=0.0,
                         channel_mult=(1, 2, 2), num_classes=None, use_attention=True),
}


def npz(path, **arrs):
    clean = {}
    for k, v in arrs.items():
        if isinstance(v, torch.Tensor):
            v = v.detach().cpu().numpy()
        clean[k] = np.ascontiguousarray(v)
    np.savez_compressed(path, **clean)
    print("wrote", path, sum(a.nbytes for a in clean.values()) / 1e6, "MB raw")


def gen_schedules():
    out = {}
    for sched in ("linear", "cosine", "quadratic"):
        d = DDPM(1000, 1e-4, 0.02, sched, device="cpu")
        for name in ("betas", "alphas", "alphas_cumprod", "alphas_cumprod_prev", "sqrt_alphas_cumprod",
                     "sqrt_one_minus_alphas_cumprod", "sqrt_recip_alphas", "sqrt_recipm1_alphas_cumprod",
                     "posterior_variance", "posterior_log_variance_clipped", "posterior_mean_coef1",
                     "posterior_mean_coef2"):
            out[f"{sched}/{name}"] = getattr(d, name)
    for T in (1000, 100):
        for S in (10, 20, 50, 100, 250):
            if S > T:
                continue
            d = DDIM(T, S, device="cpu")
            out[f"ddim_ts/{T}/{S}"] = d.inference_timesteps
    npz(OUT / "schedules.npz", **out)


def gen_unet(name, cfg, B=2):
    torch.manual_seed(1234)
    m = UNet(**cfg).float()
    m.train()  # dropout 0.0 -> deterministic
    g = torch.Generator().manual_seed(7)
    C, (H, W) = cfg["in_channels"], cfg["image_size"]
    x = torch.randn(B, C, H, W, generator=g).requires_grad_(True)
    t = torch.tensor([17, 903][:B], dtype=torch.long)
    y = None
    if cfg["num_classes"] is not None:
        # label 0 = null class (CFG); 11 > num_classes exercises the clamp (models/unet.py:256-257)
        y = torch.tensor([0, 11][:B], dtype=torch.long)
    out = m(x, t, y)
    cot = torch.randn(out.shape, generator=g)
    (out * cot).sum().backward()
    arrs = {"x": x.detach(), "t": t, "out": out.detach(), "cot": cot}
    if y is not None:
        arrs["y"] = y
    for k, v in m.state_dict().items():
        arrs["param/" + k] = v
    for k, p in m.named_parameters():
        if p.grad is not None:
            arrs["grad/" + k] = p.grad
    arrs["grad_x"] = x.grad
    npz(OUT / f"{name}.npz", **arrs)


def gen_diffusion_ops():
    cfg = TINY_CFGS["unet_tiny_cond"]
    torch.manual_seed(1234)
    m = UNet(**cfg).float().eval()
    g = torch.Generator().manual_seed(11)
    B, C, H, W = 3, 3, 16, 16
    x0 = torch.rand(B, C, H, W, generator=g) * 2 - 1
    noise = torch.randn(B, C, H, W, generator=g)
    t = torch.tensor([0, 499, 999])
    y = torch.tensor([1, 5, 0])
    ddpm = DDPM(1000, 1e-4, 0.02, "linear", device="cpu")
    arrs = {"x0": x0, "noise": noise, "t": t, "y": y}
    arrs["q_sample"] = ddpm.q_sample(x0, t, noise)
    with torch.no_grad():
        for lt in ("l1", "l2", "huber"):
            arrs[f"p_losses/{lt}"] = ddpm.p_losses(m, x0, t, y, noise=noise, loss_type=lt).reshape(1)
    # DDPM p_sample with injected noise: patch randn_like for this one call
    xt = arrs["q_sample"]
    z = torch.randn(B, C, H, W, generator=g)
    arrs["ddpm_z"] = z
    orig = torch.randn_like
    torch.randn_like = lambda a, *k, **kw: z.clone()
    try:
        with torch.no_grad():
            arrs["ddpm_p_sample"] = ddpm.p_sample(m, xt, t, y)
    finally:
        torch.randn_like = orig
    # DDIM single step and a full 10-step trajectory from an injected x_T
    ddim = DDIM(1000, 10, 1e-4, 0.02, "linear", eta=0.0, device="cpu")
    t_next = torch.tensor([-1, 479, 979])
    with torch.no_grad():
        arrs["ddim_p_sample"] = ddim.p_sample(m, xt, t, torch.tensor([-1, -1, -1]), y)
        # the reference takes the alpha_next branch only when every t_next >= 0
        arrs["ddim_p_sample_next"] = ddim.p_sample(m, xt, torch.tensor([20, 499, 999]),
                                                   torch.tensor([0, 479, 979]), y)
    xT = torch.randn(B, C, H, W, generator=g)
    arrs["ddim_xT"] = xT
    orig_randn = torch.randn
    torch.randn = lambda *a, **kw: xT.clone()
    try:
        with torch.no_grad():
            arrs["ddim_sample"] = ddim.sample(m, (B, C, H, W), y)
            arrs["ddim_sample_all"] = ddim.sample(m, (B, C, H, W), y, return_all_timesteps=True)
            arrs["ddim_sample_cfg"] = ddim.sample_with_cfg(m, (B, C, H, W), y, cfg_scale=3.0)
            arrs["ddim_sample_cfg_nothr"] = ddim.sample_with_cfg(m, (B, C, H, W), y, cfg_scale=2.0,
                                                                 p_threshold=None)
    finally:
        torch.randn = orig_randn
    # DDIM with eta > 0 (stochastic): inject both x_T and the per-step noise
    ddim_eta = DDIM(1000, 5, 1e-4, 0.02, "linear", eta=0.5, device="cpu")
    zs = torch.randn(5, B, C, H, W, generator=g)
    arrs["ddim_eta_z"] = zs
    it = iter(list(zs))
    torch.randn = lambda *a, **kw: xT.clone()
    torch.randn_like = lambda a, *k, **kw: next(it).clone()
    try:
        with torch.no_grad():
            arrs["ddim_eta_sample"] = ddim_eta.sample(m, (B, C, H, W), y)
    finally:
        torch.randn = orig_randn
        torch.randn_like = orig
    npz(OUT / "diffusion_ops.npz", **arrs)
    del t_next


def gen_trainer_traj():
    from utils import trainer as trainer_mod  # reference utils/trainer.py
    cfg = dict(TINY_CFGS["unet_tiny_uncond"])
    torch.manual_seed(1234)
    m = UNet(**cfg).float()
    init = {k: v.clone() for k, v in m.state_dict().items()}
    g = torch.Generator().manual_seed(21)
    steps, B = 5, 4
    images = [torch.rand(B, 3, 16, 16, generator=g) * 2 - 1 for _ in range(steps)]
    ts = [torch.randint(0, 1000, (B,), generator=g) for _ in range(steps)]
    noises = [torch.randn(B, 3, 16, 16, generator=g) for _ in range(steps)]
    ddpm = DDPM(1000, 1e-4, 0.02, "linear", device="cpu")
    opt = torch.optim.AdamW(m.parameters(), lr=2e-4, weight_decay=1e-4)
    config = {"epochs": 1, "save_dir": "/tmp/gg_ckpt", "sample_dir": "/tmp/gg_smp", "loss_type": "l2",
              "use_ema": True, "ema_decay": 0.9, "model_type": "unet",
              "model_params": {k: v for k, v in cfg.items() if k != "num_classes"}}
    tr = trainer_mod.DiffusionTrainer(m, ddpm, images, opt, None, device="cpu", config=config)
    # inject t and noise in order
    t_it, n_it = iter(ts), iter(noises)
    orig_randint, orig_randn_like = torch.randint, torch.randn_like
    losses = []
    orig_pl = ddpm.p_losses

    def p_losses(model, x, t, y=None, noise=None, loss_type="l2"):
        loss = orig_pl(model, x, t, y, noise=noise, loss_type=loss_type)
        losses.append(loss.item())
        return loss

    ddpm.p_losses = p_losses
    torch.randint = lambda *a, **kw: next(t_it)
    torch.randn_like = lambda a, *k, **kw: next(n_it).clone()
    try:
        tr.train_epoch(1)
    finally:
        torch.randint, torch.randn_like = orig_randint, orig_randn_like
    arrs = {"images": torch.stack(images), "ts": torch.stack(ts), "noises": torch.stack(noises),
            "losses": torch.tensor(losses)}
    for k, v in init.items():
        arrs["init/" + k] = v
    for k, v in m.state_dict().items():
        arrs["final/" + k] = v
    for k, v in tr.ema_model.state_dict().items():
        arrs["ema/" + k] = v
    npz(OUT / "trainer_traj.npz", **arrs)


def np_normal(seed, shape):
    """Host-independent Gaussian draws (numpy PCG64 ziggurat, fp32): the tests regenerate them from the seed."""
    return torch.from_numpy(np.random.default_rng(seed).standard_normal(shape, dtype=np.float32))


def gen_ddpm_sample():
    cfg = TINY_CFGS["unet_tiny_cond"]
    torch.manual_seed(1234)
    m = UNet(**cfg).float().eval()
    B, shape = 2, (2, 3, 16, 16)
    y = torch.tensor([3, 7])
    ddpm = DDPM(1000, 1e-4, 0.02, "linear", device="cpu")
    arrs = {"y": y, "xT_seed": np.array([100]), "z_seed": np.array([101]), "xT_seed_cfg": np.array([102]),
            "z_seed_cfg": np.array([103])}
    snap = list(range(99, 1000, 100))
    arrs["snap_steps"] = np.array(snap)
    orig_randn, orig_randn_like = torch.randn, torch.randn_like
    for tag, xs, zsd, call in (
            ("sample", 100, 101, lambda: ddpm.sample(m, shape, y, return_all_timesteps=True)),
            ("cfg", 102, 103, lambda: ddpm.sample_with_cfg(m, shape, y, cfg_scale=3.0, return_all_timesteps=True))):
        xT = np_normal(xs, shape)
        zs = np_normal(zsd, (1000,) + shape)
        it = iter(list(zs))
        torch.randn = lambda *a, **kw: xT.clone()
        torch.randn_like = lambda a, *k, **kw: next(it).clone()
        try:
            with torch.no_grad():
                allt = call()
        finally:
            torch.randn, torch.randn_like = orig_randn, orig_randn_like
        arrs[f"{tag}/snap"] = allt[snap]
        arrs[f"{tag}/final"] = allt[-1]
    npz(OUT / "ddpm_sample.npz", **arrs)


BIG_CFGS = {
    # BASELINE config #1 shape class: 28 -> 14 -> 7 maps, 1 channel, attention only in the 7x7 middle (L=49)
    "unet_mnist": dict(image_size=(28, 28), in_channels=1, model_channels=128, out_channels=1, num_res_blocks=2,
                       attention_resolutions=(16, 8), dropout=0.0, channel_mult=(1, 2, 2), num_classes=None,
                       use_attention=True),
    # BASELINE config #5: the CIFAR network at 64x64 (attention at 16 and 8, i.e. levels 2 and 3)
    "unet_64": dict(image_size=(64, 64), in_channels=3, model_channels=128, out_channels=3, num_res_blocks=2,
                    attention_resolutions=(16, 8), dropout=0.0, channel_mult=(1, 2, 2, 2), num_classes=None,
                    use_attention=True),
}
NSAMP = 32


def grad_summary(name, v, arrs, prefix):
    v = v.detach().double().reshape(-1)
    arrs[f"{prefix}sum/{name}"] = v.sum().reshape(1)
    arrs[f"{prefix}sumsq/{name}"] = (v * v).sum().reshape(1)
    arrs[f"{prefix}absmax/{name}"] = v.abs().max().reshape(1)
    idx = np.random.default_rng(5).integers(0, v.numel(), NSAMP)
    arrs[f"{prefix}idx/{name}"] = idx
    arrs[f"{prefix}val/{name}"] = v[torch.from_numpy(idx)].float()


def gen_big_unet(name, cfg, B=2):
    torch.manual_seed(1234)
    m = UNet(**cfg).float()
    m.train()
    g = torch.Generator().manual_seed(7)
    C, (H, W) = cfg["in_channels"], cfg["image_size"]
    x = torch.randn(B, C, H, W, generator=g).requires_grad_(True)
    t = torch.tensor([17, 903][:B], dtype=torch.long)
    out = m(x, t, None)
    cot = torch.randn(out.shape, generator=g)
    (out * cot).sum().backward()
    arrs = {"x": x.detach(), "t": t, "out": out.detach(), "cot": cot, "grad_x": x.grad}
    for k, v in m.state_dict().items():
        arrs[f"psum/{k}"] = v.double().sum().reshape(1)
        arrs[f"pabs/{k}"] = v.double().abs().sum().reshape(1)
    for k, p in m.named_parameters():
        grad_summary(k, p.grad, arrs, "g")
    npz(OUT / f"{name}.npz", **arrs)


def gen_checkpoint():
    """reference save_checkpoint (utils/trainer.py:328-365) after 2 steps, then resume (:120-154) + 1 step."""
    from utils import trainer as trainer_mod
    cfg = dict(TINY_CFGS["unet_tiny_uncond"])
    g = torch.Generator().manual_seed(31)
    B = 4
    images = [torch.rand(B, 3, 16, 16, generator=g) * 2 - 1 for _ in range(3)]
    ts = [torch.randint(0, 1000, (B,), generator=g) for _ in range(3)]
    noises = [torch.randn(B, 3, 16, 16, generator=g) for _ in range(3)]
    ddpm = DDPM(1000, 1e-4, 0.02, "linear", device="cpu")
    save_dir = Path("/tmp/gg_ckpt2")
    config = {"epochs": 1, "save_dir": str(save_dir), "sample_dir": "/tmp/gg_smp2", "loss_type": "l2",
              "use_ema": True, "ema_decay": 0.9, "model_type": "unet", "save_interval": 1000,
              "model_params": {k: v for k, v in cfg.items() if k != "num_classes"}}
    losses = []

    def run(tr, imgs, tt, nn_):
        t_it, n_it = iter(tt), iter(nn_)
        orig_randint, orig_randn_like = torch.randint, torch.randn_like
        orig_pl = ddpm.p_losses

        def p_losses(model, x, t, y=None, noise=None, loss_type="l2"):
            loss = orig_pl(model, x, t, y, noise=noise, loss_type=loss_type)
            losses.append(loss.item())
            return loss

        ddpm.p_losses = p_losses
        torch.randint = lambda *a, **kw: next(t_it)
        torch.randn_like = lambda a, *k, **kw: next(n_it).clone()
        try:
            tr.train_loader = imgs
            tr.train_epoch(1)
        finally:
            torch.randint, torch.randn_like = orig_randint, orig_randn_like
            ddpm.p_losses = orig_pl

    torch.manual_seed(1234)
    m = UNet(**cfg).float()
    opt = torch.optim.AdamW(m.parameters(), lr=2e-4, weight_decay=1e-4)
    tr = trainer_mod.DiffusionTrainer(m, ddpm, images[:2], opt, None, device="cpu", config=config)
    run(tr, images[:2], ts[:2], noises[:2])
    tr.best_loss = 0.5
    tr.save_checkpoint(1)
    import shutil
    shutil.copy(save_dir / "current_model.pth", OUT / "trainer_ckpt.pth")
    # resume in a fresh trainer exactly as train.py would (new model + optimizer, resume_path)
    torch.manual_seed(999)
    m2 = UNet(**cfg).float()
    opt2 = torch.optim.AdamW(m2.parameters(), lr=2e-4, weight_decay=1e-4)
    tr2 = trainer_mod.DiffusionTrainer(m2, ddpm, images[2:], opt2, None, device="cpu", config=config,
                                       resume_path=str(OUT / "trainer_ckpt.pth"))
    run(tr2, images[2:], ts[2:], noises[2:])
    arrs = {"images": torch.stack(images), "ts": torch.stack(ts), "noises": torch.stack(noises),
            "losses": torch.tensor(losses), "start_epoch": np.array([tr2.start_epoch])}
    for k, v in m2.state_dict().items():
        arrs["final/" + k] = v
    for k, v in tr2.ema_model.state_dict().items():
        arrs["ema/" + k] = v
    arrs["step_after"] = np.array([float(opt2.state[p]["step"]) for p in m2.parameters()])
    npz(OUT / "ckpt_resume.npz", **arrs)


DIT_CFGS = {
    # 8x8 tokens of 2x2 patches, 2 heads of 32, conditional (label 0 = null, 11 exercises the clamp)
    "dit_tiny_cond": dict(img_size=(16, 16), patch_size=2, in_channels=3, hidden_size=64, depth=2, num_heads=2,
                          mlp_ratio=4.0, num_classes=10, dropout=0.0),
    # 4x4 patches (16 taps), 1 channel, 4 heads of 16, unconditional, non-square image
    "dit_tiny_p4": dict(img_size=(16, 32), patch_size=4, in_channels=1, hidden_size=64, depth=2, num_heads=4,
                        mlp_ratio=2.0, num_classes=None, dropout=0.0),
}
# BASELINE config #4: DiT-S/2 at 32x32, 10 classes
DIT_S2 = dict(img_size=(32, 32), patch_size=2, in_channels=3, hidden_size=384, depth=12, num_heads=6, mlp_ratio=4.0,
              num_classes=10, dropout=0.0)


def perturb_dit(m, std, seed=11):
    """The reference zero-initialises every adaLN projection and the final linear (models/dit.py:239-247), which
    makes a fresh DiT output exactly 0 and most gradients vanish: add seeded N(0, std) to every parameter (in
    named_parameters order) so that the fixture exercises every path. The build's DiT applies the same
    perturbation (tests/test_oracle.py: perturb_dit)."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for _, p in m.named_parameters():
            p.add_(std * torch.randn(p.shape, generator=g))


def _dit_inputs(cfg, B):
    g = torch.Generator().manual_seed(7)
    C, (H, W) = cfg["in_channels"], cfg["img_size"]
    x = torch.randn(B, C, H, W, generator=g).requires_grad_(True)
    t = torch.tensor([17, 903, 500, 0][:B], dtype=torch.long)
    y = torch.tensor([0, 11, 3, 10][:B], dtype=torch.long) if cfg["num_classes"] is not None else None
    return g, x, t, y


def gen_dit(name, cfg, B=2):
    from models.dit import DiT
    torch.manual_seed(1234)
    m = DiT(**cfg).float()
    perturb_dit(m, 0.05)
    m.train()   # dropout 0.0 -> deterministic
    g, x, t, y = _dit_inputs(cfg, B)
    out = m(x, t, y)
    cot = torch.randn(out.shape, generator=g)
    (out * cot).sum().backward()
    arrs = {"x": x.detach(), "t": t, "out": out.detach(), "cot": cot, "grad_x": x.grad}
    if y is not None:
        arrs["y"] = y
        with torch.no_grad():
            arrs["out_ynone"] = m(x.detach(), t, None)
    for k, v in m.state_dict().items():
        arrs["param/" + k] = v
    for k, p in m.named_parameters():
        arrs["grad/" + k] = p.grad
    npz(OUT / f"{name}.npz", **arrs)


def gen_dit_s2(B=2):
    """Weights not stored: torch.manual_seed(1234) + perturb_dit(std 0.02) is reproduced by the tests and pinned by
    the per-tensor checksums."""
    from models.dit import DiT
    torch.manual_seed(1234)
    m = DiT(**DIT_S2).float()
    perturb_dit(m, 0.02)
    m.train()
    g, x, t, y = _dit_inputs(DIT_S2, B)
    out = m(x, t, y)
    cot = torch.randn(out.shape, generator=g)
    (out * cot).sum().backward()
    arrs = {"x": x.detach(), "t": t, "y": y, "out": out.detach(), "cot": cot, "grad_x": x.grad}
    for k, v in m.state_dict().items():
        arrs[f"psum/{k}"] = v.double().sum().reshape(1)
        arrs[f"pabs/{k}"] = v.double().abs().sum().reshape(1)
    for k, p in m.named_parameters():
        grad_summary(k, p.grad, arrs, "g")
    npz(OUT / "dit_s2.npz", **arrs)


K1_STEPS, K1_B = 1000, 4
K1_SNAP = (0, 250, 500, 750)      # theta_k stored (weights BEFORE step k, i.e. the ones step k's loss sees)
K1_OPT = 500                      # AdamW exp_avg / exp_avg_sq stored here too (teacher-forced window restart)
K1_SEEDS = (41, 42, 43)           # numpy PCG64 seeds of x0 / t / noise; the tests regenerate the draws


def k1_inputs():
    """The 1000 steps' inputs, host-independent (tests/k1_draws.py, shared with the tests): numpy PCG64 draws in
    step order (x0 ~ U(-1,1), t ~ U{0..999}, noise ~ N(0,1), float32)."""
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    from k1_draws import k1_draws
    return k1_draws(K1_SEEDS, K1_B, K1_STEPS)


def _run_ref_1k(threads, capture):
    """The reference DiffusionTrainer (utils/trainer.py:221-273) for 1000 steps on the tiny unconditional UNet
    (dropout 0, l2, clip 1.0, AdamW lr 2e-4 wd 1e-4, EMA 0.9999), t and noise injected per step."""
    from utils import trainer as trainer_mod
    torch.set_num_threads(threads)
    cfg = dict(TINY_CFGS["unet_tiny_uncond"])
    torch.manual_seed(1234)
    m = UNet(**cfg).float()
    xs, ts, ns = k1_inputs()
    ddpm = DDPM(1000, 1e-4, 0.02, "linear", device="cpu")
    opt = torch.optim.AdamW(m.parameters(), lr=2e-4, weight_decay=1e-4)
    config = {"epochs": 1, "save_dir": "/tmp/gg_ckpt1k", "sample_dir": "/tmp/gg_smp1k", "loss_type": "l2",
              "use_ema": True, "ema_decay": 0.9999, "model_type": "unet",
              "model_params": {k: v for k, v in cfg.items() if k != "num_classes"}}
    tr = trainer_mod.DiffusionTrainer(m, ddpm, xs, opt, None, device="cpu", config=config)
    t_it, n_it = iter(ts), iter(ns)
    losses = []
    snaps = {}
    step = [0]
    orig_pl, orig_clip = ddpm.p_losses, torch.nn.utils.clip_grad_norm_
    orig_randint, orig_randn_like = torch.randint, torch.randn_like

    def p_losses(model, x, t, y=None, noise=None, loss_type="l2"):
        k = step[0]
        if capture and k in K1_SNAP:
            snaps[f"theta/{k}"] = {n: v.detach().clone() for n, v in m.state_dict().items()}
            if k == K1_OPT:
                snaps["m"] = {n: opt.state[p]["exp_avg"].clone() for n, p in m.named_parameters()}
                snaps["v"] = {n: opt.state[p]["exp_avg_sq"].clone() for n, p in m.named_parameters()}
        loss = orig_pl(model, x, t, y, noise=noise, loss_type=loss_type)
        losses.append(loss.item())
        return loss

    def clip(params, max_norm, *a, **kw):
        k = step[0]
        if capture and k in K1_SNAP:
            snaps[f"grad/{k}"] = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
        step[0] += 1
        return orig_clip(params, max_norm, *a, **kw)

    ddpm.p_losses = p_losses
    torch.nn.utils.clip_grad_norm_ = clip
    torch.randint = lambda *a, **kw: next(t_it)
    torch.randn_like = lambda a, *k, **kw: next(n_it).clone()
    try:
        tr.train_epoch(1)
    finally:
        torch.randint, torch.randn_like = orig_randint, orig_randn_like
        torch.nn.utils.clip_grad_norm_ = orig_clip
        ddpm.p_losses = orig_pl
        torch.set_num_threads(8)
    assert len(losses) == K1_STEPS
    return losses, snaps, m, tr


def gen_trainer_1k():
    """north_star "p_losses matching reference to 1e-4 over 1k steps" (SURVEY §7 protocol (ii)): the reference's
    1000-step training run with every step's loss, the weights theta_k at K1_SNAP (with the step-k gradient as a
    per-tensor summary), AdamW state at K1_OPT, and the same run on ONE host thread (`losses_alt`: the spread a
    mere change of summation order produces, which calibrates the free-running band of the GPU test)."""
    losses, snaps, m, tr = _run_ref_1k(8, True)
    alt, _, _, _ = _run_ref_1k(1, False)
    arrs = {"losses": np.array(losses, dtype=np.float64), "losses_alt": np.array(alt, dtype=np.float64),
            "snap_steps": np.array(K1_SNAP), "opt_step": np.array([K1_OPT]), "seeds": np.array(K1_SEEDS),
            "batch": np.array([K1_B])}
    for k in K1_SNAP:
        for n, v in snaps[f"theta/{k}"].items():
            arrs[f"theta/{k}/{n}"] = v
        for n, v in snaps[f"grad/{k}"].items():
            grad_summary(n, v, arrs, f"g{k}/")
    for n in snaps["m"]:
        arrs[f"exp_avg/{n}"] = snaps["m"][n]
        arrs[f"exp_avg_sq/{n}"] = snaps["v"][n]
    for n, v in m.state_dict().items():
        arrs[f"psum_final/{n}"] = v.double().sum().reshape(1)
    for n, v in tr.ema_model.state_dict().items():
        arrs[f"esum_final/{n}"] = v.double().sum().reshape(1)
    npz(OUT / "trainer_1k.npz", **arrs)


GENERATORS = {"schedules": gen_schedules, "tiny": lambda: [gen_unet(n, c) for n, c in TINY_CFGS.items()],
              "diffusion_ops": gen_diffusion_ops, "trainer_traj": gen_trainer_traj,
              "ddpm_sample": gen_ddpm_sample, "big": lambda: [gen_big_unet(n, c) for n, c in BIG_CFGS.items()],
              "checkpoint": gen_checkpoint, "dit": lambda: [gen_dit(n, c) for n, c in DIT_CFGS.items()],
              "dit_s2": gen_dit_s2, "trainer_1k": gen_trainer_1k}


if __name__ == "__main__":
    # python tests/golden/gen_golden.py [name ...]   (default: every fixture)
    for name in (sys.argv[1:] or list(GENERATORS)):
        GENERATORS[name]()
