"""CPU ORACLE — test infrastructure only. Never imported by the product path.

fp32 CPU restatement of the reference's diffusion math (diffusion/ddpm.py, diffusion/ddim.py,
utils/trainer.py of sunyzhi55/Diffusion_Models_Collection), written from the equations:
  schedules         ddpm.py:38-71 (cosine :73-82)
  ddim timesteps    ddim.py:71-85
  q_sample          ddpm.py:84-104
  losses            ddpm.py:130-139
  DDPM posterior    ddpm.py:151-220
  DDIM update       ddim.py:154-208
  CFG + threshold   ddim.py:300-325, ddpm.py:284-303
  DDPM sample loops ddpm.py:222-332
  train step        utils/trainer.py:221-265 (clip 1.0 -> AdamW -> zero_grad -> EMA)
Pinned by tests/test_oracle.py against tests/golden/ (fixtures produced by the reference itself).
"""
import torch
import torch.nn.functional as F


def schedule(T=1000, beta_start=1e-4, beta_end=0.02, kind="linear"):
    if kind == "linear":
        b = torch.linspace(beta_start, beta_end, T)
    elif kind == "quadratic":
        b = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, T) ** 2
    elif kind == "cosine":
        x = torch.linspace(0, T, T + 1)
        ac = torch.cos(((x / T) + 0.008) / 1.008 * torch.pi * 0.5) ** 2
        ac = ac / ac[0]
        b = torch.clip(1 - ac[1:] / ac[:-1], 0.0001, 0.9999)
    else:
        raise ValueError(kind)
    a = 1.0 - b
    ac = torch.cumprod(a, 0)
    acp = F.pad(ac[:-1], (1, 0), value=1.0)
    pv = b * (1.0 - acp) / (1.0 - ac)
    return {
        "betas": b, "alphas": a, "alphas_cumprod": ac, "alphas_cumprod_prev": acp,
        "sqrt_alphas_cumprod": ac.sqrt(), "sqrt_one_minus_alphas_cumprod": (1.0 - ac).sqrt(),
        "sqrt_recip_alphas": (1.0 / a).sqrt(), "sqrt_recipm1_alphas_cumprod": (1.0 / ac - 1).sqrt(),
        "posterior_variance": pv, "posterior_log_variance_clipped": torch.log(torch.clamp(pv, min=1e-20)),
        "posterior_mean_coef1": b * acp.sqrt() / (1.0 - ac),
        "posterior_mean_coef2": (1.0 - acp) * a.sqrt() / (1.0 - ac),
    }


def ddim_timesteps(T, S):
    return torch.linspace(T - 1, 0, S).round().long()


def bcast(v, t, ndim):
    return v[t].reshape(-1, *([1] * (ndim - 1)))


def q_sample(tab, x0, t, noise):
    return bcast(tab["sqrt_alphas_cumprod"], t, x0.dim()) * x0 + bcast(tab["sqrt_one_minus_alphas_cumprod"], t,
                                                                      x0.dim()) * noise


def loss(kind, noise, pred):
    if kind == "l1":
        return F.l1_loss(noise, pred)
    if kind == "l2":
        return F.mse_loss(noise, pred)
    if kind == "huber":
        return F.smooth_l1_loss(noise, pred)
    raise ValueError(kind)


def ddpm_step(tab, x, eps, t, z, clip=True, x0=None):
    nd = x.dim()
    if x0 is None:
        x0 = bcast((1.0 / tab["alphas_cumprod"]).sqrt(), t, nd) * x - bcast(tab["sqrt_recipm1_alphas_cumprod"], t,
                                                                              nd) * eps
    if clip:
        x0 = x0.clamp(-1, 1)
    mean = bcast(tab["posterior_mean_coef1"], t, nd) * x0 + bcast(tab["posterior_mean_coef2"], t, nd) * x
    nz = (t != 0).float().view(-1, *([1] * (nd - 1)))
    return mean + nz * torch.exp(0.5 * bcast(tab["posterior_log_variance_clipped"], t, nd)) * z


def ddim_step(ac_tab, x, eps, t, t_next, eta=0.0, z=None, clip=True, x0=None):
    nd = x.dim()
    at = bcast(ac_tab, t, nd)
    an = bcast(ac_tab, t_next, nd) if bool((t_next >= 0).all()) else torch.ones_like(at)
    if x0 is None:
        x0 = (x - (1 - at).sqrt() * eps) / at.sqrt()
    if clip:
        x0 = x0.clamp(-1, 1)
    sigma = eta * torch.sqrt(torch.clamp((1 - an) / (1 - at) * (1 - at / an), min=0.0))
    out = an.sqrt() * x0 + torch.sqrt(torch.clamp(1 - an - sigma ** 2, min=0.0)) * eps
    if eta > 0:
        out = out + sigma * z
    return out


def dynamic_threshold(x0, p):
    B = x0.shape[0]
    s = torch.quantile(x0.reshape(B, -1).abs(), p, dim=1)
    s = torch.maximum(s, torch.ones_like(s)).view(B, *([1] * (x0.dim() - 1)))
    return torch.clamp(x0, -s, s) / s


def ddim_sample(model_fn, ac_tab, ts, xT, y=None, eta=0.0, zs=None, cfg_scale=None, p_threshold=0.995):
    """DDIM loop (ddim.py:210-249) and its CFG variant (:251-346). model_fn(x, t, y) -> eps."""
    img = xT
    B = xT.shape[0]
    ts = list(ts.tolist())
    for i, t in enumerate(ts):
        tb = torch.full((B,), t, dtype=torch.long)
        tn = torch.full((B,), ts[i + 1] if i + 1 < len(ts) else -1, dtype=torch.long)
        if cfg_scale is None:
            eps = model_fn(img, tb, y)
            img = ddim_step(ac_tab, img, eps, tb, tn, eta, None if zs is None else zs[i])
        else:
            ec = model_fn(img, tb, y)
            eu = model_fn(img, tb, torch.zeros_like(y))
            eps = eu + cfg_scale * (ec - eu)
            at = bcast(ac_tab, tb, img.dim())
            x0 = (img - torch.sqrt(1 - at) * eps) / torch.sqrt(at)
            x0 = dynamic_threshold(x0, p_threshold) if p_threshold is not None else x0.clamp(-1, 1)
            img = ddim_step(ac_tab, img, eps, tb, tn, eta, None if zs is None else zs[i], clip=False, x0=x0)
    return img


def ddpm_sample(model_fn, tab, xT, zs, y=None, cfg_scale=None, p_threshold=0.995, snap=()):
    """DDPM ancestral loop (ddpm.py:222-252) and its CFG variant (:254-332); zs[i] is the noise of loop step i
    (t = T-1-i). Returns (final, [x after loop step s for s in snap])."""
    img = xT
    B = xT.shape[0]
    T = tab["betas"].numel()
    snaps = []
    for i, ti in enumerate(reversed(range(T))):
        t = torch.full((B,), ti, dtype=torch.long)
        if cfg_scale is None:
            img = ddpm_step(tab, img, model_fn(img, t, y), t, zs[i])
        else:
            ec = model_fn(img, t, y)
            eu = model_fn(img, t, torch.zeros_like(y))
            eps = eu + cfg_scale * (ec - eu)
            nd = img.dim()
            x0 = bcast((1.0 / tab["alphas_cumprod"]).sqrt(), t, nd) * img - bcast(
                tab["sqrt_recipm1_alphas_cumprod"], t, nd) * eps
            x0 = dynamic_threshold(x0, p_threshold) if p_threshold is not None else x0.clamp(-1, 1)
            img = ddpm_step(tab, img, eps, t, zs[i], clip=False, x0=x0)
        if i in snap:
            snaps.append(img)
    return img, snaps


def ema_update(ema_sd, sd, decay):
    for k in ema_sd:
        ema_sd[k].mul_(decay).add_(sd[k], alpha=1 - decay)
