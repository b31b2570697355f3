"""Data parallel with the REAL UNet executor: 2 ranks sharing one MI355X over gloo (RCCL needs one GPU per rank;
the driver's N>1 bench runs RCCL). Covers SURVEY §8 a17 (utils/trainer.py:57-61, :255):

  * the init broadcast (utils/trainer.py:348-351 here, DDP's constructor broadcast in the reference): rank 1
    starts from different weights and trains from rank 0's;
  * GradSync over the executor's grad-ready watermarks: the averaged gradient of two B=2 shards equals the
    single-process gradient of the B=4 batch (fp32, 1e-5 of the largest gradient);
  * the segmented HIP-graph step of the distributed trainer (graphs cut at the all-reduce points, collectives
    issued eagerly between replays) computes bitwise what the eager distributed step computes.

The ranks are spawned processes (torch.multiprocessing, start method spawn): each initialises its own HIP
context; results come back through files.
"""
import os
import socket
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
STEPS = 4


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _data(step):
    g = torch.Generator().manual_seed(77 + step)
    x = torch.rand(4, 3, 16, 16, generator=g) * 2 - 1
    t = torch.randint(0, 1000, (4,), generator=g)
    n = torch.randn(4, 3, 16, 16, generator=g)
    return x, t, n


def _config(tmp, cfg, kind="unet"):
    return {"epochs": 1, "save_dir": os.path.join(tmp, "c"), "sample_dir": os.path.join(tmp, "s"), "loss_type": "l2",
            "use_ema": True, "ema_decay": 0.9, "model_type": "dit" if kind.startswith("dit") else "unet",
            "ddp_bucket_mb": 0.1, "model_params": {k: v for k, v in cfg.items() if k != "num_classes"}}


def _model(kind):
    """(class, constructor kwargs) of the tiny backbone a case trains: the UNet, or the DiT (the DiT
    executor's publish() watermarks and block-prefix buckets), unconditional, with or without dropout."""
    from test_oracle import DIT, TINY
    if kind == "unet":
        from diffusion_models_collection_amd.models import UNet
        return UNet, dict(TINY["unet_tiny_uncond"])
    from diffusion_models_collection_amd.models import DiT
    return DiT, dict(DIT["dit_tiny_cond"], num_classes=None, dropout=0.1 if kind == "dit_dropout" else 0.0)


def _worker(rank, world, port, outdir, graph, kind="unet"):
    sys.path.insert(0, os.path.dirname(HERE))
    sys.path.insert(0, HERE)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["DMC_GRAPH"] = "1" if graph else "0"
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from diffusion_models_collection_amd.diffusion import DDPM
    from diffusion_models_collection_amd.utils.trainer import DiffusionTrainer
    cls, cfg = _model(kind)
    torch.manual_seed(100 + rank)                      # different weights per rank: the broadcast must fix it
    m = cls(**cfg)
    if kind.startswith("dit"):
        from test_oracle import perturb_dit
        perturb_dit(m, 0.05, seed=11 + rank)           # off the zero adaLN init so every path carries gradient
    m = m.cuda()
    before = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3, weight_decay=1e-4)
    tr = DiffusionTrainer(m, DDPM(device="cuda"), None, opt, None, device="cuda", config=_config(outdir, cfg, kind),
                          rank=rank, world_size=world)
    m.train()
    init = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    ex = m.executor
    losses, flats = [], []
    orig_randint, orig_randn_like = torch.randint, torch.randn_like
    for step in range(STEPS):
        x, t, n = _data(step)
        sl = slice(2 * rank, 2 * rank + 2)
        # the step's t and noise draws return this rank's shard (patched only around the step)
        # the trainer's timestep draw (size (B,)); the dropout-seed draw of the executors (size (1,)) stays torch's
        torch.randint = lambda lo, hi, size, *a, **k: (t[sl].cuda() if tuple(size) == (2,)
                                                      else orig_randint(lo, hi, size, *a, **k))
        torch.randn_like = lambda a, *k, **kw: n[sl].cuda()
        try:
            loss = tr.train_step(x[sl].cuda(), step)
        finally:
            torch.randint, torch.randn_like = orig_randint, orig_randn_like
        torch.cuda.synchronize()
        losses.append(float(loss))
        flats.append(ex.flat.detach().cpu().clone())
    res = {"before": before, "init": init, "losses": torch.tensor(losses), "flats": torch.stack(flats),
           "final": {k: v.detach().cpu().clone() for k, v in m.state_dict().items()},
           "graphed": tr._graph is not None and tr._graph.graph is not None and tr._graph.segs is not None,
           "nsegs": len(tr._graph.segs) if tr._graph is not None and tr._graph.segs else 0}
    if tr.ema_model is not None:
        res["ema"] = {k: v.detach().cpu().clone() for k, v in tr.ema_model.state_dict().items()}
    torch.save(res, os.path.join(outdir, f"{kind}_rank{rank}_{'graph' if graph else 'eager'}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _run(tmp_path, graph, kind):
    import torch.multiprocessing as mp
    mp.start_processes(_worker, args=(2, _free_port(), str(tmp_path), graph, kind), nprocs=2, start_method="spawn")
    tag = "graph" if graph else "eager"
    return [torch.load(tmp_path / f"{kind}_rank{r}_{tag}.pt", weights_only=True) for r in range(2)]


@pytest.mark.parametrize("kind", ["unet", "dit", "dit_dropout"])
def test_ddp_two_ranks_real_executor(tmp_path, kind):
    from diffusion_models_collection_amd.diffusion import DDPM
    eager = _run(tmp_path, False, kind)
    r0, r1 = eager
    # init broadcast: rank 1 started elsewhere and now holds rank 0's weights
    assert any(not torch.equal(r0["before"][k], r1["before"][k]) for k in r0["before"])
    for k in r0["init"]:
        assert torch.equal(r0["init"][k], r1["init"][k]), k
        assert torch.equal(r0["init"][k], r0["before"][k]), k
    # every rank sees the same averaged gradients and ends with the same parameters
    assert torch.equal(r0["flats"], r1["flats"])
    for k in r0["final"]:
        assert torch.equal(r0["final"][k], r1["final"][k]), k
    # averaged shard gradients == the single-process gradient of the whole batch (step 0, same weights; without
    # dropout: its masks are keyed by the element index within each rank's shard)
    if kind != "dit_dropout":
        cls, cfg = _model(kind)
        m = cls(**cfg)
        m.load_state_dict(r0["init"])
        m = m.cuda().train()
        x, t, n = _data(0)
        loss = DDPM(device="cuda").p_losses(m, x.cuda(), t.cuda(), noise=n.cuda())
        loss.backward()
        ref = m.executor.flat.detach().cpu()
        err = ((r0["flats"][0] - ref).abs().max() / ref.abs().max()).item()
        assert err < 1e-5, err
        assert abs((r0["losses"][0] + r1["losses"][0]).item() / 2 - loss.item()) < 1e-5

    # the segmented-graph distributed step: bitwise the eager distributed step
    graph = _run(tmp_path, True, kind)
    for r in range(2):
        assert graph[r]["graphed"] and graph[r]["nsegs"] >= (4 if kind == "unet" else 2), (graph[r]["graphed"],
                                                                                          graph[r]["nsegs"])
        assert torch.equal(graph[r]["losses"], eager[r]["losses"]), (graph[r]["losses"], eager[r]["losses"])
        assert torch.equal(graph[r]["flats"], eager[r]["flats"])
        for k in eager[r]["final"]:
            assert torch.equal(graph[r]["final"][k], eager[r]["final"][k]), k
    for k in eager[0]["ema"]:
        assert torch.equal(graph[0]["ema"][k], eager[0]["ema"][k]), k
