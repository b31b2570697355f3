"""Pin the CPU oracle (oracle/) against the golden fixtures produced by the reference (tests/golden/)."""
import pytest
import torch

from conftest import load_golden
from oracle import diffusion_oracle as DO
from oracle.unet_oracle import make_oracle

TINY = {
    "unet_tiny_uncond": dict(image_size=(16, 16), in_channels=3, model_channels=16, out_channels=3,
                             num_res_blocks=1, attention_resolutions=(8,), dropout=0.0, channel_mult=(1, 2),
                             num_classes=None, use_attention=True),
    "unet_tiny_cond": dict(image_size=(16, 16), in_channels=3, model_channels=16, out_channels=3,
                           num_res_blocks=1, attention_resolutions=(8,), dropout=0.0, channel_mult=(1, 2),
                           num_classes=10, use_attention=True),
    "unet_tiny_l3": dict(image_size=(16, 16), in_channels=1, model_channels=16, out_channels=1,
                         num_res_blocks=2, attention_resolutions=(8, 4), dropout=0.0, channel_mult=(1, 2, 2),
                         num_classes=None, use_attention=True),
}


def split_params(g, prefix):
    return {k[len(prefix):]: v for k, v in g.items() if k.startswith(prefix)}


def test_schedules_bit_exact():
    g = load_golden("schedules")
    for kind in ("linear", "cosine", "quadratic"):
        tab = DO.schedule(1000, 1e-4, 0.02, kind)
        for name, v in tab.items():
            assert torch.equal(v, g[f"{kind}/{name}"]), (kind, name)


def test_ddim_timesteps_bit_exact():
    g = load_golden("schedules")
    for k, v in g.items():
        if k.startswith("ddim_ts/"):
            _, T, S = k.split("/")
            assert torch.equal(DO.ddim_timesteps(int(T), int(S)), v), k
    assert DO.ddim_timesteps(1000, 50)[:4].tolist() == [999, 979, 958, 938]


@pytest.mark.parametrize("name", list(TINY))
def test_oracle_unet_fwd_bwd(name):
    g = load_golden(name)
    params = split_params(g, "param/")
    orc, sd = make_oracle(params, TINY[name], requires_grad=True)
    x = g["x"].clone().requires_grad_(True)
    out = orc.forward(x, g["t"], g.get("y"))
    torch.testing.assert_close(out, g["out"], rtol=1e-5, atol=1e-5)
    (out * g["cot"]).sum().backward()
    torch.testing.assert_close(x.grad, g["grad_x"], rtol=1e-4, atol=1e-5)
    grads = split_params(g, "grad/")
    for k, ref in grads.items():
        torch.testing.assert_close(sd[k].grad, ref, rtol=1e-4, atol=1e-5, msg=k)


def test_oracle_diffusion_ops():
    g = load_golden("diffusion_ops")
    params = split_params(load_golden("unet_tiny_cond"), "param/")
    orc, _ = make_oracle(params, TINY["unet_tiny_cond"])
    tab = DO.schedule()
    f = lambda x, t, y: orc.forward(x, t, y)  # noqa: E731
    x0, noise, t, y = g["x0"], g["noise"], g["t"], g["y"]
    xt = DO.q_sample(tab, x0, t, noise)
    assert torch.equal(xt, g["q_sample"])
    with torch.no_grad():
        pred = f(xt, t, y)
        for lt in ("l1", "l2", "huber"):
            torch.testing.assert_close(DO.loss(lt, noise, pred).reshape(1), g[f"p_losses/{lt}"], rtol=1e-5,
                                       atol=1e-6)
        torch.testing.assert_close(DO.ddpm_step(tab, xt, pred, t, g["ddpm_z"]), g["ddpm_p_sample"], rtol=1e-5,
                                   atol=1e-5)
        ac = tab["alphas_cumprod"]
        torch.testing.assert_close(DO.ddim_step(ac, xt, pred, t, torch.tensor([-1, -1, -1])), g["ddim_p_sample"],
                                   rtol=1e-5, atol=1e-5)
        t2, tn2 = torch.tensor([20, 499, 999]), torch.tensor([0, 479, 979])
        torch.testing.assert_close(DO.ddim_step(ac, xt, f(xt, t2, y), t2, tn2), g["ddim_p_sample_next"], rtol=1e-5,
                                   atol=1e-5)
        ts = DO.ddim_timesteps(1000, 10)
        torch.testing.assert_close(DO.ddim_sample(f, ac, ts, g["ddim_xT"], y), g["ddim_sample"], rtol=1e-4,
                                   atol=1e-4)
        torch.testing.assert_close(DO.ddim_sample(f, ac, ts, g["ddim_xT"], y, cfg_scale=3.0), g["ddim_sample_cfg"],
                                   rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(DO.ddim_sample(f, ac, ts, g["ddim_xT"], y, cfg_scale=2.0, p_threshold=None),
                                   g["ddim_sample_cfg_nothr"], rtol=1e-4, atol=1e-4)
        ts5 = DO.ddim_timesteps(1000, 5)
        torch.testing.assert_close(DO.ddim_sample(f, ac, ts5, g["ddim_xT"], y, eta=0.5, zs=g["ddim_eta_z"]),
                                   g["ddim_eta_sample"], rtol=1e-4, atol=1e-4)


def train_oracle(g, cfg, steps, ema_decay=0.9):
    """utils/trainer.py:221-265 step order on the oracle UNet."""
    init = split_params(g, "init/")
    orc, sd = make_oracle(init, cfg, requires_grad=True)
    params = list(sd.values())
    opt = torch.optim.AdamW(params, lr=2e-4, weight_decay=1e-4)
    ema = {k: v.detach().clone() for k, v in sd.items()}
    tab = DO.schedule()
    losses = []
    for i in range(steps):
        x0, t, noise = g["images"][i], g["ts"][i], g["noises"][i]
        xt = DO.q_sample(tab, x0, t, noise)
        loss = DO.loss("l2", noise, orc.forward(xt, t, None, training=True))
        loss.backward()
        torch.nn.utils.clip_grad_norm_(params, 1.0)
        opt.step()
        opt.zero_grad()
        DO.ema_update(ema, {k: v.detach() for k, v in sd.items()}, ema_decay)
        losses.append(loss.item())
    return losses, sd, ema


def test_oracle_trainer_trajectory():
    g = load_golden("trainer_traj")
    cfg = dict(TINY["unet_tiny_uncond"])
    losses, sd, ema = train_oracle(g, cfg, g["losses"].numel())
    torch.testing.assert_close(torch.tensor(losses), g["losses"].float(), rtol=1e-5, atol=1e-6)
    for k, v in split_params(g, "final/").items():
        torch.testing.assert_close(sd[k].detach(), v, rtol=1e-4, atol=1e-6, msg=k)
    for k, v in split_params(g, "ema/").items():
        torch.testing.assert_close(ema[k], v, rtol=1e-4, atol=1e-6, msg=k)


def np_normal(seed, shape):
    """The fixture generator's host-independent Gaussian draws (tests/golden/gen_golden.py::np_normal)."""
    import numpy as np
    return torch.from_numpy(np.random.default_rng(seed).standard_normal(shape, dtype=np.float32))


def test_oracle_ddpm_sample_loops():
    """DDPM.sample / sample_with_cfg, 1000 steps, injected x_T and z (diffusion/ddpm.py:222-332)."""
    g = load_golden("ddpm_sample")
    orc, _ = make_oracle(split_params(load_golden("unet_tiny_cond"), "param/"), TINY["unet_tiny_cond"])
    tab = DO.schedule()
    f = lambda x, t, y: orc.forward(x, t, y)  # noqa: E731
    shape = (2, 3, 16, 16)
    snap = [int(s) for s in g["snap_steps"]]
    with torch.no_grad():
        for tag, cfg in (("sample", None), ("cfg", 3.0)):
            xs, zs = (int(g["xT_seed"]), int(g["z_seed"])) if tag == "sample" else (int(g["xT_seed_cfg"]),
                                                                                     int(g["z_seed_cfg"]))
            fin, snaps = DO.ddpm_sample(f, tab, np_normal(xs, shape), np_normal(zs, (1000,) + shape), g["y"],
                                        cfg_scale=cfg, snap=snap)
            torch.testing.assert_close(fin, g[f"{tag}/final"], rtol=1e-4, atol=1e-4)
            torch.testing.assert_close(torch.stack(snaps), g[f"{tag}/snap"], rtol=1e-4, atol=1e-4)


BIG = {
    "unet_mnist": dict(image_size=(28, 28), in_channels=1, model_channels=128, out_channels=1, num_res_blocks=2,
                       attention_resolutions=(16, 8), dropout=0.0, channel_mult=(1, 2, 2), num_classes=None,
                       use_attention=True),
    "unet_64": dict(image_size=(64, 64), in_channels=3, model_channels=128, out_channels=3, num_res_blocks=2,
                    attention_resolutions=(16, 8), dropout=0.0, channel_mult=(1, 2, 2, 2), num_classes=None,
                    use_attention=True),
}


def check_checksum(k, v, g):
    """fp64 sum and abs-sum of a parameter vs the fixture's: 1e-12 relative (the fp64 reduction order of
    torch.sum differs between hosts by an ulp; a different fp32 value moves the sum by far more)."""
    for tag, got in (("psum", v.double().sum()), ("pabs", v.double().abs().sum())):
        ref = float(g[f"{tag}/{k}"])
        assert abs(float(got) - ref) <= 1e-12 * max(1.0, abs(ref)), (k, tag, float(got), ref)


def big_init_state_dict(name):
    """The build's UNet initialised from torch.manual_seed(1234), as the fixture generator initialised the
    reference's; pinned against the fixture's per-tensor checksums."""
    from diffusion_models_collection_amd.models import UNet
    g = load_golden(name)
    torch.manual_seed(1234)
    sd = UNet(**BIG[name]).state_dict()
    for k, v in sd.items():
        check_checksum(k, v, g)
    return sd, g


def check_grad_summary(name, grad, g, tol):
    v = grad.detach().double().reshape(-1).cpu()
    amax = float(g[f"gabsmax/{name}"])
    scale = max(amax, 1e-12)
    assert abs(float(v.abs().max()) - amax) <= tol * scale, (name, float(v.abs().max()), amax)
    ref_n = float(g[f"gsumsq/{name}"]) ** 0.5
    assert abs(float((v * v).sum()) ** 0.5 - ref_n) <= tol * max(ref_n, 1e-12) * 4, name
    got = v[g[f"gidx/{name}"]].float()
    assert (got - g[f"gval/{name}"]).abs().max().item() <= tol * scale, name


@pytest.mark.parametrize("name", list(BIG))
def test_oracle_big_unet_fwd_bwd(name):
    """BASELINE configs #1 (MNIST 28x28, channel_mult (1,2,2)) and #5 (64x64) shapes, full width, B=2."""
    sd0, g = big_init_state_dict(name)
    orc, sd = make_oracle(sd0, BIG[name], requires_grad=True)
    x = g["x"].clone().requires_grad_(True)
    out = orc.forward(x, g["t"], None)
    torch.testing.assert_close(out, g["out"], rtol=1e-4, atol=1e-4)
    (out * g["cot"]).sum().backward()
    torch.testing.assert_close(x.grad, g["grad_x"], rtol=1e-3, atol=1e-4)
    for k, p in sd.items():
        if p.grad is not None:
            check_grad_summary(k, p.grad, g, 1e-3)


def test_oracle_checkpoint_resume():
    """utils/trainer.py:120-154 resume + one step (:221-265) from the reference's own checkpoint dict."""
    from pathlib import Path
    ck = torch.load(Path(__file__).parent / "golden" / "trainer_ckpt.pth", weights_only=True)
    g = load_golden("ckpt_resume")
    assert ck["epoch"] == 1 and int(g["start_epoch"]) == 2
    cfg = dict(TINY["unet_tiny_uncond"])
    orc, sd = make_oracle(ck["model_state_dict"], cfg, requires_grad=True)
    params = list(sd.values())
    opt = torch.optim.AdamW(params, lr=2e-4, weight_decay=1e-4)
    opt.load_state_dict(ck["optimizer_state_dict"])
    ema = {k: v.clone() for k, v in ck["ema_model_state_dict"].items()}
    tab = DO.schedule()
    x0, t, noise = g["images"][2], g["ts"][2], g["noises"][2]
    loss = DO.loss("l2", noise, orc.forward(DO.q_sample(tab, x0, t, noise), t, None, training=True))
    loss.backward()
    torch.nn.utils.clip_grad_norm_(params, 1.0)
    opt.step()
    DO.ema_update(ema, {k: v.detach() for k, v in sd.items()}, 0.9)
    torch.testing.assert_close(loss.reshape(1), g["losses"][2:3].float(), rtol=1e-5, atol=1e-6)
    for k, v in split_params(g, "final/").items():
        torch.testing.assert_close(sd[k].detach(), v, rtol=1e-4, atol=1e-6, msg=k)
    for k, v in split_params(g, "ema/").items():
        torch.testing.assert_close(ema[k], v, rtol=1e-4, atol=1e-6, msg=k)
    assert all(float(s) == 3.0 for s in g["step_after"])


# ---- DiT (models/dit.py) ----
DIT = {
    "dit_tiny_cond": dict(img_size=(16, 16), patch_size=2, in_channels=3, hidden_size=64, depth=2, num_heads=2,
                          mlp_ratio=4.0, num_classes=10, dropout=0.0),
    "dit_tiny_p4": dict(img_size=(16, 32), patch_size=4, in_channels=1, hidden_size=64, depth=2, num_heads=4,
                        mlp_ratio=2.0, num_classes=None, dropout=0.0),
}
DIT_S2 = dict(img_size=(32, 32), patch_size=2, in_channels=3, hidden_size=384, depth=12, num_heads=6, mlp_ratio=4.0,
              num_classes=10, dropout=0.0)


def perturb_dit(m, std, seed=11):
    """tests/golden/gen_golden.py perturb_dit: seeded N(0, std) added to every parameter in named_parameters
    order (the reference zero-initialises adaLN and the final linear)."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for _, p in m.named_parameters():
            p.add_(std * torch.randn(p.shape, generator=g))
    return m


def dit_s2_state_dict():
    """The build's DiT-S/2 from torch.manual_seed(1234) + perturbation, pinned on the fixture's checksums."""
    from diffusion_models_collection_amd.models import DiT
    g = load_golden("dit_s2")
    torch.manual_seed(1234)
    m = perturb_dit(DiT(**DIT_S2), 0.02)
    sd = m.state_dict()
    for k, v in sd.items():
        check_checksum(k, v, g)
    return m, g


@pytest.mark.parametrize("name", list(DIT))
def test_oracle_dit_fwd_bwd(name):
    from oracle.dit_oracle import make_oracle as make_dit
    g = load_golden(name)
    orc, sd = make_dit(split_params(g, "param/"), DIT[name], requires_grad=True)
    x = g["x"].clone().requires_grad_(True)
    out = orc.forward(x, g["t"], g.get("y"))
    torch.testing.assert_close(out, g["out"], rtol=1e-5, atol=1e-5)
    if "out_ynone" in g:
        torch.testing.assert_close(orc.forward(g["x"], g["t"], None), g["out_ynone"], rtol=1e-5, atol=1e-5)
    (out * g["cot"]).sum().backward()
    torch.testing.assert_close(x.grad, g["grad_x"], rtol=1e-4, atol=1e-5)
    for k, ref in split_params(g, "grad/").items():
        torch.testing.assert_close(sd[k].grad, ref, rtol=1e-4, atol=1e-5, msg=k)


def test_dit_module_tree_matches_reference_fixture():
    """The build's DiT constructs the reference's parameters: same keys, shapes and (seeded) values."""
    from diffusion_models_collection_amd.models import DiT
    for name, cfg in DIT.items():
        g = load_golden(name)
        torch.manual_seed(1234)
        sd = perturb_dit(DiT(**cfg), 0.05).state_dict()
        ref = split_params(g, "param/")
        assert list(sd) == list(ref), name
        for k in sd:
            assert torch.equal(sd[k], ref[k]), (name, k)


def test_oracle_dit_s2():
    """BASELINE config #4 shape (DiT-S/2, 32x32, 10 classes), B=2: output, grad_x and gradient summaries."""
    from oracle.dit_oracle import make_oracle as make_dit
    m, g = dit_s2_state_dict()
    orc, sd = make_dit(m.state_dict(), DIT_S2, requires_grad=True)
    x = g["x"].clone().requires_grad_(True)
    out = orc.forward(x, g["t"], g["y"])
    torch.testing.assert_close(out, g["out"], rtol=1e-4, atol=1e-4)
    (out * g["cot"]).sum().backward()
    torch.testing.assert_close(x.grad, g["grad_x"], rtol=1e-3, atol=1e-4)
    for k, p in sd.items():
        check_grad_summary(k, p.grad, g, 1e-3)


def test_oracle_trainer_1k_snapshots():
    """The 1000-step fixture (tests/golden/trainer_1k.npz, the reference's own DiffusionTrainer run): at every stored
    theta_k the oracle's step-k loss equals the reference's within 1e-6 and its gradient matches the stored
    summaries within 1e-4 of each tensor's absmax; the inputs are regenerated from the fixture's seeds (numpy PCG64,
    host-independent); and the reference's two runs (8 vs 1 host threads) agree to 1e-5 per step."""
    import numpy as np
    from k1_draws import k1_inputs
    g = load_golden("trainer_1k")
    xs, ts, ns = k1_inputs(g)
    assert len(xs) == 1000 and tuple(xs[0].shape) == (4, 3, 16, 16)
    tab = DO.schedule()
    for k in (int(s) for s in g["snap_steps"]):
        orc, sd = make_oracle(split_params(g, f"theta/{k}/"), TINY["unet_tiny_uncond"], requires_grad=True)
        loss = DO.loss("l2", ns[k], orc.forward(DO.q_sample(tab, xs[k], ts[k], ns[k]), ts[k], None, training=True))
        loss.backward()
        assert abs(loss.item() - float(g["losses"][k])) < 1e-6, (k, loss.item(), float(g["losses"][k]))
        pre = f"g{k}/"
        summ = {"g" + key[len(pre):]: v for key, v in g.items() if key.startswith(pre)}
        for name, p in sd.items():
            if p.grad is not None:
                check_grad_summary(name, p.grad, summ, 1e-4)
    assert np.abs(g["losses"].numpy() - g["losses_alt"].numpy()).max() < 1e-5
