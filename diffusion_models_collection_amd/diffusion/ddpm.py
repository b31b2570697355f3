"""DDPM scheduler with the reference API (diffusion/ddpm.py of sunyzhi55/Diffusion_Models_Collection).

Same constructor (:27-34), attributes (betas, alphas_cumprod, ... :38-71) and methods (q_sample :84,
p_losses :106, _extract :142, p_mean_variance :151, p_sample :197, sample :222, sample_with_cfg :254).
Arithmetic runs in fused HIP kernels (libdmc.so):
  q_sample            -> dmc_q_sample
  p_losses loss       -> dmc_loss_fwd / dmc_loss_bwd (deterministic reduction), via _LossFn
  p_sample / mean     -> dmc_ddpm_step (x0 prediction, clip, posterior mean, noise, one launch)
  CFG + threshold     -> dmc_cfg_x0 (combine, x0, per-row quantile, clamp, one launch)
The cond/uncond forwards of CFG are batched into ONE 2B forward.

Schedule tables are built on the host with the reference's exact fp32 op sequence (so they are
bit-identical to the reference's), then uploaded once.

Extra optional keyword arguments (not in the reference, all default to the reference behaviour):
p_sample(noise=...), sample(x_T=...), sample_with_cfg(x_T=...) inject the Gaussian draws for parity tests.
"""
import torch
import torch.nn.functional as F
from tqdm import tqdm

from .. import kernels as K


def _cosine_betas(timesteps, s=0.008):
    # diffusion/ddpm.py:73-82, on the host in fp32
    steps = timesteps + 1
    x = torch.linspace(0, timesteps, steps)
    ac = torch.cos(((x / timesteps) + s) / (1 + s) * torch.pi * 0.5) ** 2
    ac = ac / ac[0]
    betas = 1 - (ac[1:] / ac[:-1])
    return torch.clip(betas, 0.0001, 0.9999)


def make_betas(num_timesteps, beta_start, beta_end, beta_schedule):
    if beta_schedule == "linear":
        return torch.linspace(beta_start, beta_end, num_timesteps)
    if beta_schedule == "cosine":
        return _cosine_betas(num_timesteps)
    if beta_schedule == "quadratic":
        return torch.linspace(beta_start ** 0.5, beta_end ** 0.5, num_timesteps) ** 2
    raise ValueError(f"Unknown beta schedule: {beta_schedule}")


def _require_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("the diffusion hot path runs on the MI355X HIP kernels only: use cuda tensors")


class _LossFn(torch.autograd.Function):
    """F.l1_loss / F.mse_loss / F.smooth_l1_loss(noise, pred) with a fused fwd/bwd (ddpm.py:130-139)."""

    @staticmethod
    def forward(ctx, pred, target, loss_type):
        pred = pred.contiguous().float()
        target = target.contiguous().float()
        ctx.save_for_backward(pred, target)
        ctx.loss_type = loss_type
        return K.loss_fwd(loss_type, pred, target)

    @staticmethod
    def backward(ctx, g):
        pred, target = ctx.saved_tensors
        g = g.contiguous().float()
        dpred = K.loss_bwd(ctx.loss_type, pred, target, g)
        dtarget = -dpred if ctx.needs_input_grad[1] else None
        return dpred, dtarget, None


def diffusion_loss(pred, target, loss_type):
    if loss_type not in ("l1", "l2", "huber"):
        raise ValueError(f"Unknown loss type: {loss_type}")
    return _LossFn.apply(pred, target, loss_type)


class DDPM:
    """DDPM diffusion process (diffusion/ddpm.py:15-332)."""

    def __init__(self, num_timesteps=1000, beta_start=0.0001, beta_end=0.02, beta_schedule='linear', device='cuda'):
        self.num_timesteps = num_timesteps
        self.device = device
        betas = make_betas(num_timesteps, beta_start, beta_end, beta_schedule)
        alphas = 1.0 - betas
        ac = torch.cumprod(alphas, dim=0)
        ac_prev = F.pad(ac[:-1], (1, 0), value=1.0)
        tabs = {
            "betas": betas,
            "alphas": alphas,
            "alphas_cumprod": ac,
            "alphas_cumprod_prev": ac_prev,
            "sqrt_alphas_cumprod": torch.sqrt(ac),
            "sqrt_one_minus_alphas_cumprod": torch.sqrt(1.0 - ac),
            "sqrt_recip_alphas": torch.sqrt(1.0 / alphas),
            "sqrt_recipm1_alphas_cumprod": torch.sqrt(1.0 / ac - 1),
            "posterior_variance": betas * (1.0 - ac_prev) / (1.0 - ac),
        }
        tabs["posterior_log_variance_clipped"] = torch.log(torch.clamp(tabs["posterior_variance"], min=1e-20))
        tabs["posterior_mean_coef1"] = betas * torch.sqrt(ac_prev) / (1.0 - ac)
        tabs["posterior_mean_coef2"] = (1.0 - ac_prev) * torch.sqrt(alphas) / (1.0 - ac)
        # recomputed by the reference on every p_mean_variance call (:170-171); identical values
        tabs["sqrt_recip_alphas_cumprod"] = torch.sqrt(1.0 / ac)
        for k, v in tabs.items():
            setattr(self, k, v.to(device))

    def _cosine_beta_schedule(self, timesteps, s=0.008, device='cuda'):
        return _cosine_betas(timesteps, s).to(device)

    def _tab(self, name, dev):
        v = getattr(self, name)
        if v.device != dev:
            v = v.to(dev)
            setattr(self, name, v)
        return v

    def q_sample(self, x_start, t, noise=None):
        """q(x_t | x_0) = sqrt(ac[t]) x_0 + sqrt(1 - ac[t]) noise (diffusion/ddpm.py:84-104)."""
        if noise is None:
            noise = torch.randn_like(x_start)
        _require_cuda(x_start, noise)
        dev = x_start.device
        return K.q_sample(x_start.float(), noise.float(), t.to(dev).long().contiguous(),
                          self._tab("sqrt_alphas_cumprod", dev), self._tab("sqrt_one_minus_alphas_cumprod", dev))

    def p_losses(self, model, x_start, t, y=None, noise=None, loss_type='l2'):
        """Training loss (diffusion/ddpm.py:106-140)."""
        if noise is None:
            noise = torch.randn_like(x_start)
        x_noisy = self.q_sample(x_start, t, noise)
        predicted_noise = model(x_noisy, t, y)
        return diffusion_loss(predicted_noise, noise, loss_type)

    def _extract(self, a, t, x_shape):
        batch_size = t.shape[0]
        a = a.to(t.device)
        out = a[t]
        return out.reshape(batch_size, *((1,) * (len(x_shape) - 1)))

    def _step(self, x, eps, t, clip, x0_pred, z):
        dev = x.device
        return K.ddpm_step(x.contiguous().float(), eps.contiguous().float(), t.to(dev).long().contiguous(),
                           self._tab("sqrt_recip_alphas_cumprod", dev), self._tab("sqrt_recipm1_alphas_cumprod", dev),
                           self._tab("posterior_mean_coef1", dev), self._tab("posterior_mean_coef2", dev),
                           self._tab("posterior_log_variance_clipped", dev), clip=clip,
                           x0=None if x0_pred is None else x0_pred.contiguous().float(),
                           z=None if z is None else z.contiguous().float())

    def p_mean_variance(self, model, x, t, y=None, clip_denoised=True, eps=None, x0_pred=None):
        """Posterior mean / variance / log-variance (diffusion/ddpm.py:151-195)."""
        if eps is None:
            eps = model(x, t, y)
        _require_cuda(x, eps)
        mean = self._step(x, eps, t, clip_denoised, x0_pred, None)
        var = self._extract(self.posterior_variance, t, x.shape)
        logvar = self._extract(self.posterior_log_variance_clipped, t, x.shape)
        return mean, var, logvar

    @torch.no_grad()
    def p_sample(self, model, x, t, y=None, clip_denoised=True, eps=None, x0_pred=None, noise=None):
        """x_{t-1} ~ p(x_{t-1} | x_t) (diffusion/ddpm.py:197-220), one fused kernel after the model call."""
        if eps is None:
            eps = model(x, t, y)
        if noise is None:
            noise = torch.randn_like(x)
        _require_cuda(x, eps, noise)
        return self._step(x, eps, t, clip_denoised, x0_pred, noise)

    @torch.no_grad()
    def sample(self, model, shape, y=None, return_all_timesteps=False, x_T=None):
        """Ancestral sampling over all timesteps (diffusion/ddpm.py:222-252)."""
        batch_size = shape[0]
        device = self.device
        img = torch.randn(shape, device=device) if x_T is None else x_T.to(device).float()
        imgs = []
        ts = torch.arange(self.num_timesteps, device=img.device).view(-1, 1).expand(-1, batch_size).contiguous()
        for i in tqdm(reversed(range(0, self.num_timesteps)), desc='Sampling', total=self.num_timesteps):
            img = self.p_sample(model, img, ts[i], y)
            if return_all_timesteps:
                imgs.append(img.cpu())
        if return_all_timesteps:
            return torch.stack(imgs, dim=0)
        return img

    @staticmethod
    def _cfg_eps(model, img, t, y):
        """eps_cond and eps_uncond from ONE batched forward (cond rows first, null label 0 second)."""
        B = img.shape[0]
        both = model(torch.cat([img, img], 0), torch.cat([t, t], 0), torch.cat([y, torch.zeros_like(y)], 0))
        return both[:B], both[B:]

    @torch.no_grad()
    def sample_with_cfg(self, model, shape, y, cfg_scale=3.0, p_threshold=0.995, return_all_timesteps=False,
                        x_T=None):
        """Classifier-free guidance + dynamic thresholding (diffusion/ddpm.py:254-332)."""
        if y is None:
            raise ValueError("CFG sampling requires class labels y.")
        if p_threshold is not None and not (0.0 < float(p_threshold) < 1.0):
            raise ValueError("p_threshold must be in (0, 1) or None")
        batch_size = shape[0]
        device = self.device
        img = torch.randn(shape, device=device) if x_T is None else x_T.to(device).float()
        imgs = []
        y = y.to(img.device)
        dev = img.device
        ts = torch.arange(self.num_timesteps, device=dev).view(-1, 1).expand(-1, batch_size).contiguous()
        for i in tqdm(reversed(range(0, self.num_timesteps)), desc=f'DDPM Sampling with CFG scale {cfg_scale}',
                      total=self.num_timesteps):
            t = ts[i]
            eps_c, eps_u = self._cfg_eps(model, img, t, y)
            eps_g, x0 = K.cfg_x0(img.contiguous(), eps_c.contiguous(), eps_u.contiguous(), cfg_scale, t,
                                 self._tab("sqrt_recip_alphas_cumprod", dev),
                                 self._tab("sqrt_recipm1_alphas_cumprod", dev), 1, p_threshold)
            img = self.p_sample(model, img, t, y=None, clip_denoised=False, eps=eps_g, x0_pred=x0)
            if return_all_timesteps:
                imgs.append(img.cpu())
        if return_all_timesteps:
            return torch.stack(imgs, dim=0)
        return img
