"""DDIM scheduler with the reference API (diffusion/ddim.py of sunyzhi55/Diffusion_Models_Collection).

Same constructor (:27-36), attributes, inference timesteps (linspace(T-1, 0, S).round().long(), :71-85,
built on the host so they are bit-identical) and methods (q_sample :87, p_losses :109, _extract :145,
p_sample :154, sample :210, sample_with_cfg :251, set_inference_steps :348).

Sampling loops replay one captured HIP graph per step after the first (diffusion/_graph.py).
The per-step update is ONE fused kernel (dmc_ddim_step): alpha gathers on device, x0 prediction,
clamp, sigma, direction term and the eta>0 noise. The reference's `t_next.min() >= 0` host sync (:176)
is done on device: if any t_next < 0, alpha_next = 1 for the whole batch, exactly as the reference.
CFG batches the cond/uncond forwards into one 2B forward and fuses combine + x0 + dynamic threshold
(per-row torch.quantile restatement) into dmc_cfg_x0.
"""
import os

import torch
from tqdm import tqdm

from .. import kernels as K
from . import _schedule
from ._graph import StepGraph, cache_for, run_loop
from .ddpm import DDPM, _require_cuda, diffusion_loss, make_betas


class DDIM:
    """DDIM diffusion process with accelerated sampling (diffusion/ddim.py:13-351)."""

    def __init__(self, num_timesteps=1000, num_inference_steps=50, beta_start=0.0001, beta_end=0.02,
                 beta_schedule='linear', eta=0.0, device='cuda'):
        self.num_timesteps = num_timesteps
        self.num_inference_steps = num_inference_steps
        self.eta = eta
        self.device = device
        tabs = _schedule.build_tables(num_timesteps, beta_start, beta_end, beta_schedule)
        for k in ("betas", "alphas", "alphas_cumprod", "sqrt_alphas_cumprod", "sqrt_one_minus_alphas_cumprod"):
            setattr(self, k, torch.from_numpy(tabs[k]).to(device))
        self._setup_inference_timesteps()

    def _cosine_beta_schedule(self, timesteps, s=0.008, device='cuda'):
        return make_betas(timesteps, 0, 0, "cosine").to(device)

    def _setup_inference_timesteps(self):
        ts = _schedule.ddim_timesteps(self.num_timesteps, self.num_inference_steps)
        self.inference_timesteps = torch.from_numpy(ts).to(self.device)

    def _tab(self, name, dev):
        v = getattr(self, name)
        if v.device != dev:
            v = v.to(dev)
            setattr(self, name, v)
        return v

    def q_sample(self, x_start, t, noise=None):
        if noise is None:
            noise = torch.randn_like(x_start)
        _require_cuda(x_start, noise)
        dev = x_start.device
        return K.q_sample(x_start.float(), noise.float(), t.to(dev).long().contiguous(),
                          self._tab("sqrt_alphas_cumprod", dev), self._tab("sqrt_one_minus_alphas_cumprod", dev))

    def p_losses(self, model, x_start, t, y=None, noise=None, loss_type='l2'):
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

    @torch.no_grad()
    def p_sample(self, model, x, t, t_next, y=None, clip_denoised=True, eps=None, x0_pred=None, noise=None):
        """x_t -> x_{t_next} (diffusion/ddim.py:154-208), one fused kernel after the model call."""
        if eps is None:
            eps = model(x, t, y)
        _require_cuda(x, eps)
        dev = x.device
        z = None
        if self.eta > 0:
            z = noise if noise is not None else torch.randn_like(x)
        return K.ddim_step(x.contiguous().float(), eps.contiguous().float(), t.to(dev).long().contiguous(),
                           t_next.to(dev).long().contiguous(), self._tab("alphas_cumprod", dev), eta=self.eta,
                           clip=clip_denoised, x0=None if x0_pred is None else x0_pred.contiguous().float(),
                           z=None if z is None else z.contiguous().float())

    def _ts_table(self, batch_size, dev):
        """[S+1, B] device table: row i = t_i for every sample, last row = -1 (t_next of the last step)."""
        ts = self.inference_timesteps.to(dev)
        tab = torch.cat([ts, torch.full((1,), -1, dtype=torch.long, device=dev)])
        return tab.view(-1, 1).expand(-1, batch_size).contiguous()

    def _noise(self, noise, i, x):
        if self.eta <= 0:
            return None
        if noise is None:
            return torch.randn_like(x)
        return noise(i) if callable(noise) else noise[i].to(x.device)

    @torch.no_grad()
    def sample(self, model, shape, y=None, return_all_timesteps=False, x_T=None, noise=None):
        """DDIM sampling loop (diffusion/ddim.py:210-249). Optional (not in the reference): x_T, and for eta > 0
        noise = [S, B, C, H, W] tensor or callable i -> tensor. Steps after the first replay one captured HIP
        graph (diffusion/_graph.py)."""
        batch_size = shape[0]
        device = self.device
        img = torch.randn(shape, device=device) if x_T is None else x_T.to(device).float()
        imgs = []
        tab = self._ts_table(batch_size, img.device)
        S = len(self.inference_timesteps)
        bar = tqdm(total=S, desc='DDIM Sampling')

        if y is not None:
            y = y.to(img.device)
        has_y, has_z = y is not None, self.eta > 0

        def inputs(i, x):
            # the labels are a step input (not captured by fn), so a graph kept across calls reads the new ones
            z = self._noise(noise, i, x)
            return (x, tab[i], tab[i + 1]) + ((y,) if has_y else ()) + ((z,) if z is not None else ())

        # every sample shares the step's timestep: a model that takes a length-1 t (UNet.shared_timestep) runs its
        # time-embedding MLPs once per step instead of once per image
        shared_t = (y is None and getattr(model, "shared_timestep", False)
                    and os.environ.get("DMC_SHARED_T", "1") != "0")   # A/B switch

        def fn(x, t, tn, *rest):
            yy = rest[0] if has_y else None
            z = rest[-1] if len(rest) > has_y else None
            eps = model(x, t[:1], None) if shared_t else None
            return self.p_sample(model, x, t, tn, yy, eps=eps, noise=z)

        def record(i, x):
            bar.update(1)
            if return_all_timesteps:
                imgs.append(x.cpu())

        cache = None if return_all_timesteps else cache_for(
            model, ("ddim", self.eta, shared_t, has_y, has_z, self.alphas_cumprod.data_ptr()), self, img)
        img = run_loop(img, S, inputs, fn, StepGraph.eligible(model, img, True, False),
                       record, cache=cache, const=(3,) if has_y else ())
        bar.close()
        if return_all_timesteps:
            return torch.stack(imgs, dim=0)
        return img

    @torch.no_grad()
    def sample_with_cfg(self, model, shape, y, cfg_scale=3.0, p_threshold=0.995, return_all_timesteps=False,
                        x_T=None, noise=None):
        """DDIM + classifier-free guidance + dynamic thresholding (diffusion/ddim.py:251-346)."""
        if y is None:
            raise ValueError("CFG sampling requires class labels y.")
        if p_threshold is not None and not (0.0 < float(p_threshold) < 1.0):
            raise ValueError("p_threshold must be in (0, 1) or None")
        batch_size = shape[0]
        device = self.device
        img = torch.randn(shape, device=device) if x_T is None else x_T.to(device).float()
        imgs = []
        dev = img.device
        y = y.to(dev)
        tab = self._ts_table(batch_size, dev)
        ac = self._tab("alphas_cumprod", dev)
        S = len(self.inference_timesteps)
        bar = tqdm(total=S, desc=f"DDIM sampling with CFG scale {cfg_scale}")

        has_z = self.eta > 0

        def inputs(i, x):
            z = self._noise(noise, i, x)
            return (x, tab[i], tab[i + 1], y) + ((z,) if z is not None else ())

        def fn(x, t, tn, yy, z=None):
            eps_c, eps_u = DDPM._cfg_eps(model, x, t, yy)
            eps_g, x0 = K.cfg_x0(x.contiguous(), eps_c.contiguous(), eps_u.contiguous(), cfg_scale, t, ac, None, 0,
                                 p_threshold)
            return self.p_sample(model, x, t, tn, y=None, clip_denoised=False, eps=eps_g, x0_pred=x0, noise=z)

        def record(i, x):
            bar.update(1)
            if return_all_timesteps:
                imgs.append(x.cpu())

        cache = None if return_all_timesteps else cache_for(
            model, ("ddim_cfg", self.eta, has_z, float(cfg_scale), p_threshold, ac.data_ptr()), self, img)
        img = run_loop(img, S, inputs, fn, StepGraph.eligible(model, img, True, False),
                       record, cache=cache, const=(3,))
        bar.close()
        if return_all_timesteps:
            return torch.stack(imgs, dim=0)
        return img

    def set_inference_steps(self, num_inference_steps):
        self.num_inference_steps = num_inference_steps
        self._setup_inference_timesteps()
