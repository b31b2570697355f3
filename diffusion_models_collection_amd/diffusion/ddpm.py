"""DDPM scheduler with the reference API (diffusion/ddpm.py of sunyzhi55/Diffusion_Models_Collection).

Same constructor (:27-34), attributes (betas, alphas_cumprod, ... :38-71) and methods (q_sample :84,
p_losses :106, _extract :142, p_mean_variance :151, p_sample :197, sample :222, sample_with_cfg :254).
Arithmetic runs in fused HIP kernels (libdmc.so):
  q_sample            -> dmc_q_sample
  p_losses loss       -> dmc_loss_fwd / dmc_loss_bwd (deterministic reduction), via _LossFn
  p_sample / mean     -> dmc_ddpm_step (x0 prediction, clip, posterior mean, noise, one launch)
  CFG + threshold     -> dmc_cfg_x0 (combine, x0, per-row quantile, clamp, one launch)
The cond/uncond forwards of CFG are batched into ONE 2B forward.

Schedule tables are built on the host by _schedule.py: the reference's op sequence as explicit IEEE fp32
numpy arithmetic (the same bits on any host whose libm log/cos are accurate to 64 double ulps: _schedule.py),
then uploaded once.

Extra optional keyword arguments (not in the reference, all default to the reference behaviour):
p_sample(noise=...), sample(x_T=...), sample_with_cfg(x_T=...) inject the Gaussian draws for parity tests.
"""
import torch
import torch.nn.functional as F
from tqdm import tqdm

from .. import kernels as K
from . import _schedule
from ._graph import StepGraph, run_loop


def make_betas(num_timesteps, beta_start, beta_end, beta_schedule):
    """Beta schedule (diffusion/ddpm.py:39-46, cosine :73-82) as an fp32 CPU tensor (see _schedule.py)."""
    return torch.from_numpy(_schedule.make_betas(num_timesteps, beta_start, beta_end, beta_schedule))


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
        tabs = _schedule.build_tables(num_timesteps, beta_start, beta_end, beta_schedule)
        for k, v in tabs.items():
            setattr(self, k, torch.from_numpy(v).to(device))

    def _cosine_beta_schedule(self, timesteps, s=0.008, device='cuda'):
        return make_betas(timesteps, 0, 0, "cosine").to(device)

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

    def _noise(self, noise, i, x):
        """Loop step i's Gaussian draw: the injected noise[i] (parity tests) or torch.randn_like(x)."""
        if noise is None:
            return torch.randn_like(x)
        return noise(i) if callable(noise) else noise[i].to(x.device)

    @torch.no_grad()
    def sample(self, model, shape, y=None, return_all_timesteps=False, x_T=None, noise=None):
        """Ancestral sampling over all timesteps (diffusion/ddpm.py:222-252). Optional (not in the reference):
        x_T, and noise = [T, B, C, H, W] tensor or callable i -> tensor, the z of loop step i (t = T-1-i).
        Steps after the first replay one captured HIP graph (diffusion/_graph.py)."""
        batch_size = shape[0]
        device = self.device
        img = torch.randn(shape, device=device) if x_T is None else x_T.to(device).float()
        T = self.num_timesteps
        ts = torch.arange(T, device=img.device).view(-1, 1).expand(-1, batch_size).contiguous()
        imgs = []
        bar = tqdm(total=T, desc='Sampling')

        def inputs(i, x):
            return x, ts[T - 1 - i], self._noise(noise, i, x)

        def fn(x, t, z):
            return self.p_sample(model, x, t, y, noise=z)

        def record(i, x):
            bar.update(1)
            if return_all_timesteps:
                imgs.append(x.cpu())

        img = run_loop(img, T, inputs, fn, StepGraph.eligible(model, img, True, False), record)
        bar.close()
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
                        x_T=None, noise=None):
        """Classifier-free guidance + dynamic thresholding (diffusion/ddpm.py:254-332); x_T / noise as sample()."""
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
        T = self.num_timesteps
        ts = torch.arange(T, device=dev).view(-1, 1).expand(-1, batch_size).contiguous()
        bar = tqdm(total=T, desc=f'DDPM Sampling with CFG scale {cfg_scale}')

        def inputs(i, x):
            return x, ts[T - 1 - i], self._noise(noise, i, x)

        def fn(x, t, z):
            eps_c, eps_u = self._cfg_eps(model, x, t, y)
            eps_g, x0 = K.cfg_x0(x.contiguous(), eps_c.contiguous(), eps_u.contiguous(), cfg_scale, t,
                                 self._tab("sqrt_recip_alphas_cumprod", dev),
                                 self._tab("sqrt_recipm1_alphas_cumprod", dev), 1, p_threshold)
            return self.p_sample(model, x, t, y=None, clip_denoised=False, eps=eps_g, x0_pred=x0, noise=z)

        def record(i, x):
            bar.update(1)
            if return_all_timesteps:
                imgs.append(x.cpu())

        img = run_loop(img, T, inputs, fn, StepGraph.eligible(model, img, True, False), record)
        bar.close()
        if return_all_timesteps:
            return torch.stack(imgs, dim=0)
        return img
