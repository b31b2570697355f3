"""GPU parity of the DiT (models/dit.py of the reference; SURVEY §8f rank 2, BASELINE config #4) against the
reference's golden fixtures and the CPU oracle.

Tolerances:
  fp32: output within 2e-5 of max |ref| (tiny) / 1e-4 (DiT-S/2), every gradient within 2e-4 of its max |ref|
        (summation order only); DiT-S/2 gradient summaries within 2e-3 of the tensor's absmax.
  bf16: GEMM operands in bf16, residual stream / LayerNorm statistics / modulation in fp32: output within 3e-2 of
        max |ref| with cosine > 0.999; gradient cosine > 0.99.
"""
import pytest
import torch

from conftest import load_golden
from test_gpu_model import cos, rel
from test_oracle import DIT, DIT_S2, check_grad_summary, dit_s2_state_dict, split_params

pytestmark = pytest.mark.gpu
DEV = "cuda"


def build(name, dtype="fp32"):
    from diffusion_models_collection_amd.models import DiT
    g = load_golden(name)
    m = DiT(**DIT[name], compute_dtype=dtype)
    m.load_state_dict(split_params(g, "param/"))
    return m.to(DEV), g


@pytest.mark.parametrize("name", list(DIT))
def test_dit_tiny_fp32_matches_reference(name):
    m, g = build(name)
    m.train()
    x = g["x"].to(DEV).requires_grad_(True)
    y = g["y"].to(DEV) if "y" in g else None
    out = m(x, g["t"].to(DEV), y)
    assert rel(out, g["out"]) < 2e-5, rel(out, g["out"])
    (out * g["cot"].to(DEV)).sum().backward()
    assert rel(x.grad, g["grad_x"]) < 2e-4, rel(x.grad, g["grad_x"])
    for k, p in m.named_parameters():
        ref = g["grad/" + k]
        assert rel(p.grad, ref) < 2e-4, (k, rel(p.grad, ref))
    if "out_ynone" in g:
        m.eval()
        with torch.no_grad():
            o2 = m(g["x"].to(DEV), g["t"].to(DEV), None)
        assert rel(o2, g["out_ynone"]) < 2e-5


@pytest.mark.parametrize("name", list(DIT))
def test_dit_tiny_bf16_close_to_reference(name):
    m, g = build(name, "bf16")
    x = g["x"].to(DEV).requires_grad_(True)
    y = g["y"].to(DEV) if "y" in g else None
    out = m(x, g["t"].to(DEV), y)
    assert rel(out, g["out"]) < 3e-2 and cos(out, g["out"]) > 0.999, (rel(out, g["out"]), cos(out, g["out"]))
    (out * g["cot"].to(DEV)).sum().backward()
    worst = min((cos(p.grad, g["grad/" + k]), k) for k, p in m.named_parameters())
    assert worst[0] > 0.99, worst


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_dit_s2_matches_reference(dtype):
    """BASELINE config #4 network (DiT-S/2, 32x32, 10 classes, 256 tokens, head dim 64), B=2, forward + backward
    against the reference's fixture."""
    m, g = dit_s2_state_dict()
    m.set_compute_dtype(dtype)
    m = m.to(DEV).train()
    x = g["x"].to(DEV).requires_grad_(True)
    out = m(x, g["t"].to(DEV), g["y"].to(DEV))
    (out * g["cot"].to(DEV)).sum().backward()
    eo, eg = rel(out, g["out"]), rel(x.grad, g["grad_x"])
    print(f"dit_s2 {dtype}: out rel {eo:.2e} cos {cos(out, g['out']):.6f}; grad_x rel {eg:.2e}")
    if dtype == "fp32":
        assert eo < 1e-4 and eg < 1e-3, (eo, eg)
        for k, p in m.named_parameters():
            check_grad_summary(k, p.grad, g, 2e-3)
    else:
        assert eo < 5e-2 and cos(out, g["out"]) > 0.999, eo
        assert cos(x.grad, g["grad_x"]) > 0.99


def test_dit_batch_independence_and_graph():
    """B=16 rows equal the B=2 rows (fp32), and DDIM-10 CFG sampling with the graphed step equals the eager loop
    bitwise and the oracle's loop within 1e-3."""
    from diffusion_models_collection_amd.diffusion import DDIM
    from oracle import diffusion_oracle as DO
    from oracle.dit_oracle import make_oracle
    m, g = build("dit_tiny_cond")
    m.eval()
    torch.manual_seed(0)
    x = torch.randn(16, 3, 16, 16)
    t = torch.randint(0, 1000, (16,))
    y = torch.randint(0, 11, (16,))
    with torch.no_grad():
        a = m(x.to(DEV), t.to(DEV), y.to(DEV))
        b = m(x[:2].to(DEV), t[:2].to(DEV), y[:2].to(DEV))
    assert rel(b, a[:2]) < 1e-5
    ddim = DDIM(1000, 10, device=DEV)
    xT = torch.randn(4, 3, 16, 16)
    yy = torch.tensor([1, 2, 3, 4])
    outs = []
    import os
    for gr in ("0", "1"):
        os.environ["DMC_GRAPH"] = gr
        try:
            with torch.no_grad():
                outs.append(ddim.sample_with_cfg(m, (4, 3, 16, 16), yy.to(DEV), cfg_scale=3.0, x_T=xT.to(DEV)).cpu())
        finally:
            os.environ.pop("DMC_GRAPH", None)
    assert torch.equal(outs[0], outs[1])
    orc, _ = make_oracle(m.state_dict(), DIT["dit_tiny_cond"])
    tab = DO.schedule()
    ref = DO.ddim_sample(lambda xx, tt, y_: orc.forward(xx, tt, y_), tab["alphas_cumprod"],
                         DO.ddim_timesteps(1000, 10), xT, y=yy, cfg_scale=3.0)
    assert rel(outs[0], ref) < 1e-3, rel(outs[0], ref)


def test_dit_train_step_graphed_matches_eager(monkeypatch):
    """DiffusionTrainer on a DiT (dropout 0, bf16, EMA, conditional with label dropout): the fused flat AdamW and
    the HIP-graph step run for the DiT executor too, bitwise equal to the eager step over 5 steps."""
    from diffusion_models_collection_amd.models import DiT
    from diffusion_models_collection_amd.diffusion import DDPM
    from diffusion_models_collection_amd.utils.trainer import DiffusionTrainer
    mp = dict(DIT["dit_tiny_cond"])
    mp.pop("num_classes")

    def run(graph):
        monkeypatch.setenv("DMC_GRAPH", "1" if graph else "0")
        torch.manual_seed(0)
        torch.cuda.manual_seed(0)
        m = DiT(**mp, num_classes=10, compute_dtype="bf16").to(DEV)
        opt = torch.optim.AdamW(m.parameters(), lr=1e-3, weight_decay=1e-4)
        cfg = {"epochs": 1, "save_dir": "/tmp/dmc_dit_ckpt", "sample_dir": "/tmp/dmc_dit_smp", "loss_type": "l2",
               "use_ema": True, "ema_decay": 0.99, "conditional": True, "num_classes": 10, "cfg_dropout_prob": 0.2,
               "model_type": "dit", "model_params": dict(mp)}
        tr = DiffusionTrainer(m, DDPM(device=DEV), None, opt, None, device=DEV, config=cfg)
        assert tr._flat is not None and (tr._graph is not None) == graph
        m.train()
        gen = torch.Generator().manual_seed(5)
        losses = []
        for i in range(5):
            x = (torch.rand(8, 3, 16, 16, generator=gen) * 2 - 1).to(DEV)
            losses.append(tr.train_step((x, torch.randint(0, 10, (8,), generator=gen).to(DEV)), i).detach().float()
                          .cpu().reshape(()))
        torch.cuda.synchronize()
        return (torch.stack(losses), {k: v.detach().cpu().clone() for k, v in m.state_dict().items()},
                {k: v.detach().cpu().clone() for k, v in tr.ema_model.state_dict().items()}, tr)

    le, se, ee, _ = run(False)
    lg, sg, eg, trg = run(True)
    assert trg._graph.graph is not None and not trg._graph.failed
    assert torch.isfinite(le).all()
    assert torch.equal(le, lg), (le, lg)
    for k in se:
        assert torch.equal(se[k], sg[k]), k
        assert torch.equal(ee[k], eg[k]), k


def test_dit_train_step_grads_match_oracle():
    """One p_losses step of the DiT-S/2 network (fp32, dropout 0): loss and every parameter gradient vs the
    oracle, B=2."""
    from diffusion_models_collection_amd.diffusion import DDPM
    from oracle import diffusion_oracle as DO
    from oracle.dit_oracle import make_oracle
    m, _ = dit_s2_state_dict()
    m = m.to(DEV).train()
    orc, sd = make_oracle(m.state_dict(), DIT_S2, requires_grad=True)
    x0 = torch.rand(2, 3, 32, 32) * 2 - 1
    t = torch.tensor([3, 801])
    y = torch.tensor([0, 7])
    noise = torch.randn_like(x0)
    tab = DO.schedule()
    lref = DO.loss("l2", noise, orc.forward(DO.q_sample(tab, x0, t, noise), t, y))
    lref.backward()
    loss = DDPM(device=DEV).p_losses(m, x0.to(DEV), t.to(DEV), y.to(DEV), noise=noise.to(DEV))
    loss.backward()
    assert abs(loss.item() - lref.item()) < 1e-5 * max(1.0, abs(lref.item()))
    for k, p in m.named_parameters():
        assert rel(p.grad, sd[k].grad) < 5e-4, (k, rel(p.grad, sd[k].grad))


def test_dit_training_with_dropout_graphed_matches_eager(monkeypatch):
    """The reference DiT config trains with dropout 0.1 (configs/cifar10_dit.py): attention-probability dropout in
    the flash kernels plus both MLP dropouts. Over 4 DiffusionTrainer steps (bf16, conditional, EMA) the losses are
    finite and the HIP-graph step (dropout seed read from device memory per replay) equals the eager step bitwise;
    eval mode switches every dropout off (deterministic output)."""
    from diffusion_models_collection_amd.models import DiT
    from diffusion_models_collection_amd.diffusion import DDPM
    from diffusion_models_collection_amd.utils.trainer import DiffusionTrainer
    mp = dict(DIT["dit_tiny_cond"], dropout=0.1)
    mp.pop("num_classes")

    def run(graph):
        monkeypatch.setenv("DMC_GRAPH", "1" if graph else "0")
        torch.manual_seed(0)
        torch.cuda.manual_seed(0)
        m = DiT(**mp, num_classes=10, compute_dtype="bf16").to(DEV)
        opt = torch.optim.AdamW(m.parameters(), lr=1e-3, weight_decay=1e-4)
        cfg = {"epochs": 1, "save_dir": "/tmp/dmc_ditd_ckpt", "sample_dir": "/tmp/dmc_ditd_smp", "loss_type": "l2",
               "use_ema": True, "ema_decay": 0.99, "conditional": True, "num_classes": 10, "cfg_dropout_prob": 0.2,
               "model_type": "dit", "model_params": dict(mp)}
        tr = DiffusionTrainer(m, DDPM(device=DEV), None, opt, None, device=DEV, config=cfg)
        m.train()
        gen = torch.Generator().manual_seed(5)
        losses = []
        for i in range(4):
            x = (torch.rand(8, 3, 16, 16, generator=gen) * 2 - 1).to(DEV)
            losses.append(tr.train_step((x, torch.randint(0, 10, (8,), generator=gen).to(DEV)), i).detach().float()
                          .cpu().reshape(()))
        torch.cuda.synchronize()
        return torch.stack(losses), {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}, m, tr

    le, se, m, _ = run(False)
    lg, sg, _, trg = run(True)
    assert torch.isfinite(le).all()
    assert trg._graph is not None and trg._graph.graph is not None and not trg._graph.failed
    assert torch.equal(le, lg), (le, lg)
    for k in se:
        assert torch.equal(se[k], sg[k]), k
    m.eval()
    x = torch.randn(2, 3, 16, 16, device=DEV)
    t = torch.tensor([1, 2], device=DEV)
    with torch.no_grad():
        assert torch.equal(m(x, t, None), m(x, t, None))


def test_dit_dropout_masks_follow_the_torch_seed():
    """With dropout active the training-mode forward differs from eval mode, and the two MLP masks and the
    attention mask change with the torch seed (torch.manual_seed drives the per-step mask seed)."""
    from diffusion_models_collection_amd.models import DiT
    from test_oracle import perturb_dit
    torch.manual_seed(1)
    m = perturb_dit(DiT(**{**DIT["dit_tiny_cond"], "dropout": 0.3}), 0.05).to(DEV)   # off the zero adaLN init
    x = torch.randn(2, 3, 16, 16, device=DEV)
    t = torch.tensor([5, 600], device=DEV)
    with torch.no_grad():
        m.eval()
        e = m(x, t, None)
        m.train()
        torch.manual_seed(7)
        a = m(x, t, None)
        torch.manual_seed(7)
        b = m(x, t, None)
        torch.manual_seed(8)
        c = m(x, t, None)
    assert torch.equal(a, b) and not torch.equal(a, c) and not torch.equal(a, e)
