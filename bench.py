"""Benchmark: CIFAR-10 UNet DDPM training img/s (BASELINE.json metric), plus DDIM-50 sampling img/s.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

A "step" is one full DiffusionTrainer.train_step of the reference loop (utils/trainer.py:222-265) on a
synthetic 128 x 3 x 32 x 32 batch already resident in HBM: t ~ randint, q_sample, UNet forward, MSE,
backward, fused clip_grad_norm(1.0), AdamW step, zero_grad, fused EMA (rank 0, decay 0.9999), with
dropout 0.1, on the configs/cifar10_unet.py network (37.06 M params, random init), bf16 compute.
Data parallel: one process per GPU, gradients averaged by RCCL all-reduce overlapped with backward; each
rank trains its own 128-image shard (weak scaling). value = images of all ranks / max-over-ranks time.

The JSON line also carries:
  roofline      the dominant kernel (implicit-GEMM 3x3 conv, bf16 MFMA): achieved = algorithmic FLOPs per
                launch / average launch time, vs the 2.5 PFLOP/s dense bf16 MFMA peak (MI355X_MICROARCH.md);
                the headline uses the rocprofv3 kernel-trace average committed under profiles/ for this tree,
                the figure timed live with HIP events on the launch stream sits beside it ("live")
  cpu_baseline  the CPU oracle (oracle/unet_oracle.py, fp32, a port of the reference path) running the
                same train step on the host cores, rank 0 only, bounded sample (B=32, 3 timed steps)
  ddim50        DDIM-50 sampling img/s (eta 0, B=128 per GPU, replicas), with its own cpu_baseline (the
                oracle's DDIM at B=16)
  ddim50_cfg    DDIM-50 + classifier-free guidance (scale 3.0, dynamic threshold 0.995) img/s, conditional
                UNet (10 classes), B=128 per GPU as one 256-row forward per step
  celeba64      BASELINE config #5 on one GPU: the same network at 64x64, train img/s and DDIM-100 img/s
  fp32          the headline train step in the reference's own arithmetic (fp32 parity mode)
  data_loader   the device-resident data path (datasets/loader.py): dmc_load_batch per batch, the train step
                fed by it, and the oracle's per-sample transform on one host thread as its CPU baseline
  dit_s2_ddim50_cfg  BASELINE config #4: DiT-S/2 conditional DDIM-50 + CFG 3.0 sampling img/s (replicas) with
                its MFMA roofline, and the DiT train step img/s (--no-dit skips it)
(celeba64 / fp32 only at N=1; --no-extra skips them.) `--image-size 64 --sample-steps 100` makes config #5 the
headline line instead.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CIFAR = dict(image_size=(32, 32), in_channels=3, model_channels=128, out_channels=3, num_res_blocks=2,
             attention_resolutions=(16, 8), dropout=0.1, channel_mult=(1, 2, 2, 2), use_attention=True)
MFMA_BF16_PEAK_TFLOPS = 2500.0   # dense, MI355X_MICROARCH.md
TRAIN_GFLOP_PER_IMG = 37.890     # fwd + bwd, = 3 x 12.632 forward
PMC_FILE = "r6_pmc_roofline_conv.json"          # rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE of the roofline conv
ROOFLINE_CSV = "r6_roofline_kernel_stats.csv"   # rocprofv3 --kernel-trace --stats of `bench.py --roofline-only`
DIT_PMC_FILE = "r6_pmc_dit_loop.json"           # rocprofv3 --pmc over `bench.py --dit-only --no-train`


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def conv_roofline(dtype, B=128):
    """Time the dominant kernel (the ResBlock 3x3 conv 128->128 @32x32, B=128, bias + time-embedding epilogue that
    also emits the next GroupNorm's partials, as conv1 of a ResBlock does in the training step (models/_unet_exec.py
    _res_fwd, stats=h1); its GN+SiLU input is materialised by the GN-apply pass, as in training; the halo kernel the library picks by
    default: conv3x3_halo2_kernel, two 128-pixel blocks per CU) with HIP events on the stream it is
    launched on. `achieved` / `avg_launch_ms`: the average of 50 launches issued back to back between two events
    (agrees with the rocprofv3 kernel-trace average, profiles/r3_roofline_kernel_stats.csv);
    `per_launch_events_ms`: an event pair around every launch (includes the events' own overhead)."""
    from diffusion_models_collection_amd import _lib as L, kernels as K
    H = W = 32
    C = 128
    dev = "cuda"
    x = torch.randn(B, H, W, C, device=dev).to(dtype)
    w = torch.randn(C, C, 3, 3, device=dev) * 0.03
    Kc = L.kc_for(C, dtype)
    wp = K.pack_weight(L.PACK_FWD, dtype, w, Kc)
    bias = torch.randn(C, device=dev)
    addv = torch.randn(B, C, device=dev)
    y = torch.empty(B, H, W, C, device=dev, dtype=dtype)
    d = K.make_desc(dtype, B, H, W, C, 0, C, 0, Kc, H, W, C, K.TAPS3)
    gpart = torch.empty(B * H * W // 64 * (C // 8) * 2, dtype=torch.float32, device=dev) \
        if dtype == torch.bfloat16 else None
    K.set_epilogue(d, bias=bias, addvec=addv, ld_add=C, ldy1=C, gn_part=gpart)
    for _ in range(5):
        K.conv(d, x, None, wp, y)
    s = torch.cuda.current_stream()
    n = 50
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * n)]
    for i in range(n):
        ev[2 * i].record(s)
        K.conv(d, x, None, wp, y)
        ev[2 * i + 1].record(s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(n):
        K.conv(d, x, None, wp, y)
    e1.record(s)
    e1.synchronize()
    avg_ms = sum(ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(n)) / n
    b2b_ms = e0.elapsed_time(e1) / n
    flops = 2.0 * B * H * W * C * C * 9
    # the live launch duration is taken from the 50 back-to-back launches between two events (an event pair
    # around every launch adds its own ~4 us); the headline below is the committed rocprofv3 figure
    achieved = flops / (b2b_ms * 1e-3) / 1e12
    kname = "conv3x3_halo2_kernel"
    live = {"achieved": round(achieved, 2), "frac": round(achieved / MFMA_BF16_PEAK_TFLOPS, 4),
            "avg_launch_ms": round(b2b_ms, 4), "per_launch_events_ms": round(avg_ms, 4)}
    out = {"kernel": f"{kname} bf16 implicit GEMM (ResBlock 3x3 128->128 @32x32, B=128, "
                     "bias+temb epilogue + GroupNorm partials)" if dtype == torch.bfloat16 else "conv_fwd_kernel<f32,128,128>",
           "bound": "mfma", "achieved": live["achieved"], "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
           "frac": live["frac"], "traffic": pmc_traffic(), "flops_per_launch": flops,
           "avg_launch_ms": live["avg_launch_ms"], "per_launch_events_ms": live["per_launch_events_ms"],
           "algorithmic_bytes_per_launch": 2 * (2 * B * H * W * C) + 2 * C * 9 * C + B * H * W // 64 * (C // 8) * 8,
           "source": "live"}
    rc = rocprof_committed(kname, flops) if dtype == torch.bfloat16 else None
    if rc and rc.get("frac"):
        # the headline is the figure a reader recomputes from profiles/ (the rocprofv3 kernel-trace average of this
        # same command, committed for this tree); this run's own HIP-event figure sits beside it. Back-to-back
        # launches can overlap one launch's tail with the next one's start, so the live figure reads a little high.
        out.update(achieved=rc["achieved"], frac=rc["frac"], avg_launch_ms=round(rc["avg_us"] / 1e3, 4),
                   source=rc["file"])
        out["live"] = dict(live, vs_committed=round(live["frac"] / rc["frac"], 4))
    out["rocprof_committed"] = rc
    return out


def rocprof_committed(kernel="conv3x3_halo2_kernel", flops=None):
    """The roofline conv's average duration in the rocprofv3 kernel-stats CSV committed under profiles/ for this
    tree (the same `bench.py --roofline-only` command under the profiler), and the frac it gives: the figure a
    reader can recompute from profiles/ (the live `achieved` above is this run's own box)."""
    import csv
    f = os.path.join(ROOT, "profiles", ROOFLINE_CSV)
    if not os.path.exists(f):
        return None
    for r in csv.DictReader(open(f)):
        if kernel in r["Name"]:
            us = float(r["AverageNs"]) / 1e3
            out = {"file": f"profiles/{ROOFLINE_CSV}", "calls": int(r["Calls"]), "avg_us": round(us, 3)}
            if flops:
                tf = flops / (us * 1e-6) / 1e12
                out.update(achieved=round(tf, 2), frac=round(tf / MFMA_BF16_PEAK_TFLOPS, 4))
            return out
    return None


def loop_roofline(flops, seconds, scope, traffic=None):
    """Whole-loop MFMA roofline: algorithmic FLOPs of the loop (model forward FLOPs x rows x steps) / wall."""
    tf = flops / seconds / 1e12
    return {"bound": "mfma", "achieved": round(tf, 1), "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(tf / MFMA_BF16_PEAK_TFLOPS, 4), "traffic": traffic, "scope": scope}


def dit_pmc_traffic():
    f = os.path.join(ROOT, "profiles", DIT_PMC_FILE)
    if not os.path.exists(f):
        return None
    with open(f) as fh:
        return json.load(fh).get("hbm_bytes_per_loop")


def pmc_traffic():
    """HBM bytes per launch of the roofline conv from the committed rocprofv3 --pmc passes
    (profiles/PMC_FILE, written by scripts/pmc_to_json.py: FETCH_SIZE doubled per the gfx950 correction of
    MI355X_MICROARCH.md + WRITE_SIZE, averaged over the dispatches of the kernel), or None if absent."""
    f = os.path.join(ROOT, "profiles", PMC_FILE)
    if not os.path.exists(f):
        return None
    with open(f) as fh:
        return json.load(fh).get("hbm_bytes_per_launch")


def cpu_cores():
    """Cores this process may actually use: its CPU affinity, capped by a cgroup v2 CPU quota if one is set
    (a GPU box shows the whole machine in os.cpu_count() but gives a job a share of it)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    return n


def cpu_model():
    """The host CPU's model string (/proc/cpuinfo), reported beside the core count."""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(B=32, warm=3, steps=5):
    """The CPU oracle (a port of the reference path, fp32) doing the same train step on the host cores, with
    BASELINE.md §3's protocol: B=32, 3 warm-up + 5 timed steps."""
    from oracle.unet_oracle import make_oracle
    from oracle import diffusion_oracle as DO
    from diffusion_models_collection_amd.models import UNet
    threads = cpu_cores()
    torch.set_num_threads(threads)
    torch.manual_seed(42)
    m = UNet(**CIFAR)
    orc, sd = make_oracle(m.state_dict(), dict(CIFAR, num_classes=None), requires_grad=True)
    params = list(sd.values())
    opt = torch.optim.AdamW(params, lr=2e-4, weight_decay=1e-4)
    ema = {k: v.detach().clone() for k, v in sd.items()}
    tab = DO.schedule()
    x0 = torch.rand(B, 3, 32, 32) * 2 - 1

    def step():
        t = torch.randint(0, 1000, (B,))
        noise = torch.randn_like(x0)
        loss = DO.loss("l2", noise, orc.forward(DO.q_sample(tab, x0, t, noise), t, None, training=True))
        loss.backward()
        torch.nn.utils.clip_grad_norm_(params, 1.0)
        opt.step()
        opt.zero_grad()
        DO.ema_update(ema, {k: v.detach() for k, v in sd.items()}, 0.9999)

    for _ in range(warm):
        step()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    dt = time.perf_counter() - t0
    return {"value": round(B * steps / dt, 3), "unit": "img/s", "cores": threads, "os_cpu_count": os.cpu_count(),
            "cpu_model": cpu_model(), "kind": "port",
            "sample": f"BASELINE.md §3 protocol: oracle fp32 train step (q_sample, UNet fwd+bwd, clip, AdamW, EMA), "
                      f"B={B}, {steps} timed steps after {warm} warm-up steps, torch CPU with {threads} threads "
                      f"(the cores available to the process: affinity and cgroup quota)"}


def cpu_ddim_baseline(B=16, S=50):
    """DDIM-50 sampling on the CPU oracle with BASELINE.md §3's protocol: B=16, one warm-up forward, then one
    whole S-step loop (UNet forward + DDIM update per step, diffusion/ddim.py:210-249) timed."""
    from oracle.unet_oracle import make_oracle
    from oracle import diffusion_oracle as DO
    from diffusion_models_collection_amd.models import UNet
    threads = cpu_cores()
    torch.set_num_threads(threads)
    torch.manual_seed(42)
    orc, _ = make_oracle(UNet(**CIFAR).state_dict(), dict(CIFAR, num_classes=None))
    ac = DO.schedule()["alphas_cumprod"]
    ts = DO.ddim_timesteps(1000, S)
    img = torch.randn(B, 3, 32, 32)
    with torch.no_grad():
        orc.forward(img, torch.full((B,), int(ts[0])), None)          # warm-up forward
        t0 = time.perf_counter()
        img = DO.ddim_sample(lambda x, t, y: orc.forward(x, t, y), ac, ts, img)
        dt = time.perf_counter() - t0
    assert torch.isfinite(img).all()
    return {"value": round(B / dt, 4), "unit": "img/s", "cores": threads, "cpu_model": cpu_model(), "kind": "port",
            "sample": f"BASELINE.md §3 protocol: oracle fp32 DDIM-{S}, B={B}, one warm-up forward, then the whole "
                      f"{S}-step loop timed ({dt:.2f} s)"}


def train_rate(trainer, pool, steps, warmup, world):
    """Time `steps` train steps after `warmup`, barrier + synchronize on both sides, max over ranks. A graphed trainer
    warms up at least GraphedTrainStep.WARM + 1 steps, so its capture (after WARM eager steps) and first replay are
    never inside the timed region (trainer._bench_warmup: the warm-up steps actually run)."""
    g = getattr(trainer, "_graph", None)
    if g is not None:
        warmup = max(warmup, g.WARM + 1)
    trainer._bench_warmup = warmup
    for i in range(warmup):
        trainer.train_step(pool[i % len(pool)], 0)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    w0 = g.ring_wait_s if g is not None else 0.0
    r0 = g.replays if g is not None else 0
    t0 = time.perf_counter()
    for i in range(steps):
        trainer.train_step(pool[i % len(pool)], 0)
    host_el = time.perf_counter() - t0      # until the last train_step returned (the GPU may still be running)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    # host enqueue = that time minus the waits on the graphed step's pinned-argument ring (which blocks the host
    # until step k-4 has run, i.e. paces the host to the GPU)
    ring = (g.ring_wait_s - w0) if g is not None else 0.0
    trainer._bench_graphed = g is not None and g.replays - r0 == steps   # every timed step was a graph replay
    return max_over_ranks(el, world), (host_el - ring, ring)


def exposed_comm(trainer, pool, steps=5):
    """Data-parallel runs: after the timed region, `steps` more steps with GraphedTrainStep.measure_comm on (two
    HIP events on the compute stream around its waits for the RCCL buckets, i.e. after the backward's last
    bucketed segment): the mean ms per step the backward did not hide, max over ranks (None if not graphed)."""
    g = getattr(trainer, "_graph", None)
    if g is None or g.segs is None:
        return None
    g.measure_comm = True
    try:
        for i in range(steps):
            trainer.train_step(pool[i % len(pool)], 0)
        v = g.comm_ms()
    finally:
        g.measure_comm = False
    return v


def max_over_ranks(v, world):
    if world > 1:
        dist.barrier()
        tt = torch.tensor([v], device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        v = tt.item()
    return v


def make_trainer(mp, dtype, dev, rank, world, num_classes=None):
    from diffusion_models_collection_amd.models import UNet
    from diffusion_models_collection_amd.diffusion import DDPM
    from diffusion_models_collection_amd.utils.trainer import DiffusionTrainer
    torch.manual_seed(42 + rank)
    model = UNet(**mp, num_classes=num_classes, compute_dtype=dtype).to(dev)
    ddpm = DDPM(1000, 1e-4, 0.02, "linear", device=dev)
    opt = torch.optim.AdamW(model.parameters(), lr=2e-4, weight_decay=1e-4)
    cfg = {"epochs": 1, "save_dir": "/tmp/dmc_bench_ckpt", "sample_dir": "/tmp/dmc_bench_smp", "loss_type": "l2",
           "use_ema": True, "ema_decay": 0.9999, "model_type": "unet", "model_params": dict(mp)}
    return model, DiffusionTrainer(model, ddpm, None, opt, None, device=dev, config=cfg, rank=rank, world_size=world)


def sample_rate(fn, world):
    """Seconds of one sampling call after a warm-up call (replicas: each rank samples its own batch)."""
    with torch.no_grad():
        fn()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    return max_over_ranks(el, world)


def data_line(trainer, dev, B, steps):
    """The device-resident data path (datasets/loader.py): a synthetic CIFAR-shaped uint8 bank
    (50,000 x 32 x 32 x 3) in HBM, the train transform (flip 0.5, Normalize 0.5/0.5). `kernel`: one epoch of
    dmc_load_batch launches timed with HIP events; `train_with_loader_img_s`: the headline train step fed by the
    loader instead of the resident synthetic pool (loader cost inside the timed region); `cpu_baseline`: the
    oracle's per-sample transform (the reference's DataLoader worker path) on one host thread."""
    import numpy as np
    from diffusion_models_collection_amd.datasets import DiffusionDataset, from_arrays
    from diffusion_models_collection_amd.datasets.loader import DeviceLoader
    rng = np.random.default_rng(0)
    imgs = rng.integers(0, 256, (50000, 32, 32, 3), dtype=np.uint8)
    tr = DiffusionDataset.get_default_transform(32, "cifar10", train=True)
    ld = DeviceLoader(from_arrays(imgs, transform=tr), B, shuffle=True, drop_last=True, device=dev)
    it = iter(ld)
    next(it)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    n = 0
    for _ in it:
        n += 1
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / max(n, 1)
    nbytes = B * 3072 * (1 + 4)         # algorithmic: uint8 images in, fp32 NCHW out
    # the train step fed by the loader (same timing rules as the headline)
    it = iter(ld)
    for _ in range(3):
        trainer.train_step(next(it), 0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        trainer.train_step(next(it), 0)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    from oracle import data_oracle as O
    k = 2048
    t1 = time.perf_counter()
    for i in range(k):
        O.to_tensor_normalize(imgs[i], tr.mean, tr.std, flip=bool(i & 1))
    cpu = k / (time.perf_counter() - t1)
    return {"batch": B, "batches_timed": n, "kernel_us_per_batch": round(ms * 1e3, 2),
            "kernel_img_s": round(B / (ms * 1e-3), 1), "kernel_gb_s": round(nbytes / (ms * 1e-3) / 1e9, 1),
            "train_with_loader_img_s": round(B * steps / el, 2), "steps": steps,
            "cpu_baseline": {"value": round(cpu, 1), "unit": "img/s", "cores": 1, "kind": "port",
                             "sample": f"oracle per-sample flip+ToTensor+Normalize, {k} CIFAR images, one thread "
                                       "(one reference DataLoader worker's transform work; the reference runs 4)"}}


def rccl_one_rank_line(args, base_ms):
    """The data-parallel step (GradSync + the graphed step: the RCCL all-reduce of each 25 MB bucket captured into the
    one step graph -- round 6 -- or, if that capture fails, graphs cut at the all-reduce points with the collectives
    issued between the replays) on a world_size-1 'nccl' (RCCL)
    process group, timed like the headline beside it: what the distributed plumbing costs per step on one GPU
    (segment launches + collective calls + the stream waits), with no inter-GPU traffic. Run as a child process
    (`bench.py --dist-one-rank`): a failure inside RCCL or its watchdog thread aborts that process, never the
    headline run."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--dist-one-rank", "--dist-force-avg", "--no-sample", "--no-extra",
           "--no-dit", "--no-cpu", "--no-roofline", "--steps", str(args.steps), "--warmup", str(args.warmup),
           "--dtype", args.dtype, "--batch", str(args.batch), "--image-size", str(args.image_size)]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    if r.returncode != 0:
        return {"error": f"exit {r.returncode}: " + (r.stderr or "")[-400:]}
    d = json.loads(r.stdout.strip().splitlines()[-1])
    ms = d["ms_per_step"]
    return {"train_img_s": d["value"], "ms_per_step": ms, "overhead_ms_per_step": round(ms - base_ms, 3),
            "graph_segments": d.get("graph_segments"), "steps": args.steps, "batch": d["config"]["per_gpu_batch"],
            "graphed": d.get("graphed"), "reduce_op": d.get("reduce_op"),
            "comm_in_graph": d.get("comm_in_graph"), "comm_capture_fallback": d.get("comm_capture_fallback"),
            "exposed_comm_ms_per_step": d.get("exposed_comm_ms_per_step"),
            "note": "world_size-1 RCCL group (child process), ReduceOp.AVG forced (the op every multi-rank run takes, "
                    "with RCCL's averaging kernel): GradSync buckets with the all-reduces captured into the one step "
                    "graph (comm_in_graph; else the segmented graph chain) vs the single-graph headline"}


DIT_S2 = dict(img_size=(32, 32), patch_size=2, in_channels=3, hidden_size=384, depth=12, num_heads=6, mlp_ratio=4.0)


def dit_lines(args, dev, rank, world, B):
    """BASELINE config #4: DiT-S/2 (conditional, 10 classes) DDIM-50 + CFG 3.0 sampling img/s, replicas (each rank
    samples its own B images; the cond and null-label rows run as ONE 2B forward per step). The roofline is the
    whole sampling loop's MFMA work: DiT forward FLOPs (linears, patch conv, attention matmuls) x 2B rows x 50
    steps / measured seconds, vs the dense bf16 peak. Also the DiT train step img/s with the reference config's
    dropout 0.1."""
    from diffusion_models_collection_amd.models import DiT
    from diffusion_models_collection_amd.models._dit_exec import dit_flops_per_image
    from diffusion_models_collection_amd.diffusion import DDIM, DDPM
    from diffusion_models_collection_amd.utils.trainer import DiffusionTrainer
    torch.manual_seed(44 + rank)
    m = DiT(**DIT_S2, num_classes=10, dropout=0.0, compute_dtype=args.dtype).to(dev).eval()
    ddim = DDIM(1000, 50, device=dev)
    yl = torch.arange(B, device=dev) % 10 + 1
    el = sample_rate(lambda: ddim.sample_with_cfg(m, (B, 3, 32, 32), yl, cfg_scale=3.0), world)
    gf = dit_flops_per_image(m) / 1e9
    tfs = 2 * B * 50 * gf / el / 1e3
    res = {"value": round(world * B / el, 2), "unit": "img/s", "batch_per_gpu": B, "steps": 50, "cfg_scale": 3.0,
           "p_threshold": 0.995, "forward_batch": 2 * B, "seconds": round(el, 3), "scaling": "replicas",
           "model": "DiT-S/2 (hidden 384, depth 12, 6 heads, patch 2, 256 tokens), 10 classes",
           "gflop_per_forward_img": round(gf, 3),
           "roofline": {"bound": "mfma", "achieved": round(tfs, 1), "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": round(tfs / MFMA_BF16_PEAK_TFLOPS, 4), "traffic": dit_pmc_traffic(),
                        "traffic_unit": "HBM bytes per 50-step loop (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE over all "
                                        f"dispatches, profiles/{DIT_PMC_FILE})",
                        "scope": "whole DDIM-50 CFG loop per GPU"}}
    if not args.no_train:
        mt = DiT(**DIT_S2, num_classes=10, dropout=0.1, compute_dtype=args.dtype).to(dev)
        opt = torch.optim.AdamW(mt.parameters(), lr=1e-4, weight_decay=1e-4)
        cfg = {"epochs": 1, "save_dir": "/tmp/dmc_bench_ckpt", "sample_dir": "/tmp/dmc_bench_smp", "loss_type": "l2",
               "use_ema": True, "ema_decay": 0.9999, "model_type": "dit", "conditional": True, "num_classes": 10,
               "cfg_dropout_prob": 0.2, "model_params": dict(DIT_S2, dropout=0.1)}
        tr = DiffusionTrainer(mt, DDPM(device=dev), None, opt, None, device=dev, config=cfg, rank=rank,
                              world_size=world)
        gen = torch.Generator(device=dev).manual_seed(77 + rank)
        pool = [(torch.rand(B, 3, 32, 32, device=dev, generator=gen) * 2 - 1,
                 torch.randint(0, 10, (B,), device=dev, generator=gen)) for _ in range(2)]
        mt.train()
        et, _ = train_rate(tr, pool, 10, 3, world)
        res["train_img_s"] = round(world * B * 10 / et, 2)
        res["train_ms_per_step"] = round(et / 10 * 1e3, 3)
        res["train_tflops_per_gpu"] = round(B * 10 / et * 3 * gf / 1e3, 2)
        res["train_note"] = ("configs/cifar10_dit.py dropout 0.1 (attention-probability + MLP dropouts), conditional, "
                             "CFG label dropout 0.2, EMA (fwd+bwd = 3x forward FLOPs)")
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-sample", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-cfg", action="store_true", help="skip the conditional CFG sampling line")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (RCCL over xGMI) for real runs; gloo only to rehearse N>1 on one GPU")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--sample-steps", type=int, default=50)
    ap.add_argument("--no-train", action="store_true", help="sampling only (profiling)")
    ap.add_argument("--roofline-only", action="store_true", help="time only the roofline conv (PMC passes)")
    ap.add_argument("--image-size", type=int, default=32, help="32 (CIFAR-10, headline) or 64 (CelebA, config #5)")
    ap.add_argument("--no-extra", dest="extra", action="store_false",
                    help="skip the 64x64 (config #5) and fp32 side lines")
    ap.add_argument("--no-dit", dest="dit", action="store_false", help="skip the DiT-S/2 (config #4) line")
    ap.add_argument("--dit-only", action="store_true", help="only the DiT-S/2 line (profiling)")
    ap.add_argument("--dist-one-rank", action="store_true",
                    help="profiling: the headline step through GradSync + the segmented graph on a 1-rank RCCL group")
    ap.add_argument("--dist-force-avg", action="store_true",
                    help="with --dist-one-rank: all-reduce with ReduceOp.AVG (the multi-rank op) instead of SUM")
    args = ap.parse_args()
    if args.dit_only:
        torch.cuda.set_device(0)
        print(json.dumps(dit_lines(args, torch.device("cuda", 0), 0, 1, args.batch)), flush=True)
        return
    if args.roofline_only:
        print(json.dumps(conv_roofline(torch.bfloat16 if args.dtype == "bf16" else torch.float32)), flush=True)
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; --dist-backend gloo with more ranks than GPUs is a rehearsal of the multi-rank code
    # path on a 1-GPU box (ranks share the card, gloo stages the all-reduces through the host)
    ndev = torch.cuda.device_count()
    gpu = local_rank % ndev if args.dist_backend == "gloo" else local_rank
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)

    from diffusion_models_collection_amd.models import UNet
    from diffusion_models_collection_amd.models.unet import unet_flops_per_image
    from diffusion_models_collection_amd.diffusion import DDIM

    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    S = args.image_size
    mp = dict(CIFAR, image_size=(S, S))
    model, trainer = make_trainer(mp, args.dtype, dev, rank, world)
    if args.dist_one_rank and world == 1:
        import socket
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
        trainer.enable_grad_sync(force_avg=args.dist_force_avg)
    B = args.batch
    gen = torch.Generator(device=dev).manual_seed(1234 + rank)
    pool = [torch.rand(B, 3, S, S, device=dev, generator=gen) * 2 - 1 for _ in range(4)]

    model.train()
    if args.no_train:
        args.warmup, args.steps = 0, 1
        el, (host_el, ring_el) = 1.0, (0.0, 0.0)
    else:
        el, (host_el, ring_el) = train_rate(trainer, pool, args.steps, args.warmup, world)
    ms = el / args.steps * 1e3
    value = world * B * args.steps / el
    log(f"[bench] rank {rank}: {ms:.2f} ms/step, {value:.1f} img/s aggregate")
    gflop = TRAIN_GFLOP_PER_IMG * (S / 32) ** 2

    name = "CIFAR-10" if S == 32 else f"CelebA {S}x{S}"
    out = {"metric": f"{name} UNet DDPM train imgs/sec (aggregate over GPUs)", "value": round(value, 2),
           "unit": "img/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
           "data": f"synthetic (U(-1,1) {S}x{S}x3 batches resident in HBM, random-init weights)",
           "config": {"workload": f"configs/cifar10_unet.py UNet DDPM train step at {S}x{S} (q_sample, fwd, MSE, "
                                  "bwd, clip, AdamW, EMA), dropout 0.1", "model": "UNet 37.06M (128ch, mult 1,2,2,2, "
                                  "attn 16/8)", "global_batch": world * B, "per_gpu_batch": B, "seq_len": None,
                      "parallelism": f"dp{world}"},
           "per_gpu_imgs_per_sec": round(value / world, 2),
           "host_enqueue_ms_per_step": round(host_el / max(args.steps, 1) * 1e3, 3),
           "host_ring_wait_ms_per_step": round(ring_el / max(args.steps, 1) * 1e3, 3),
           "train_tflops_per_gpu": round(value / world * gflop / 1e3, 2)}
    graphed = bool(getattr(trainer, "_bench_graphed", False))
    out["graphed"] = graphed if not args.no_train else None
    if not args.no_train and trainer._bench_warmup != args.warmup:
        out["warmup_run"] = trainer._bench_warmup     # raised so that the graph capture is not timed
    if args.no_train:
        out["value"] = None
    elif not graphed and os.environ.get("DMC_GRAPH", "1") != "0":
        # the headline is the graph-replayed step: a timed step that ran eagerly means the capture was refused
        raise SystemExit("bench: a timed training step was not a HIP graph replay (graph capture did not happen)")
    if trainer.grad_sync is not None:
        out["world_size"] = dist.get_world_size()
        out["reduce_op"] = str(trainer.grad_sync.op).split(".")[-1]
        if trainer._graph is not None and trainer._graph.segs:
            out["graph_segments"] = len(trainer._graph.segs)
        elif trainer._graph is not None and trainer._graph.comm_in_graph:
            out["graph_segments"] = 1          # the all-reduces are captured inside the one step graph
        if trainer._graph is not None:
            out["comm_in_graph"] = bool(trainer._graph.comm_in_graph)
            if trainer._graph.capture_fallback:
                out["comm_capture_fallback"] = trainer._graph.capture_fallback
        if not args.no_train:
            # the part of the gradient all-reduce the backward did not hide (measured after the timed region)
            v = exposed_comm(trainer, pool)
            out["exposed_comm_ms_per_step"] = None if v is None else round(max_over_ranks(v, world), 4)
    if args.extra and S == 32 and not args.no_train and world == 1:
        out["data_loader"] = data_line(trainer, dev, B, args.steps)
        try:
            out["dp1_rccl"] = rccl_one_rank_line(args, ms)
        except Exception as e:  # noqa: BLE001 -- a side line must never hide the headline
            out["dp1_rccl"] = {"error": repr(e)}

    if not args.no_sample:
        model.eval()
        ddim = DDIM(1000, args.sample_steps, device=dev)
        sel = sample_rate(lambda: ddim.sample(model, (B, 3, S, S)), world)
        fwd_gf = unet_flops_per_image(model) / 1e9
        out[f"ddim{args.sample_steps}"] = {
            "value": round(world * B / sel, 2), "unit": "img/s", "batch_per_gpu": B, "steps": args.sample_steps,
            "seconds": round(sel, 3), "scaling": "replicas", "gflop_per_forward_img": round(fwd_gf, 3),
            "roofline": loop_roofline(B * args.sample_steps * fwd_gf * 1e9, sel,
                                      f"whole DDIM-{args.sample_steps} loop per GPU: UNet forward FLOPs x B x steps")}
        if not args.no_cfg:
            # conditional UNet (10 classes), DDIM + classifier-free guidance 3.0 + dynamic thresholding
            # (diffusion/ddim.py:251-346): cond and null-label rows as ONE 2B forward per step
            torch.manual_seed(43 + rank)
            cmodel = UNet(**mp, num_classes=10, compute_dtype=args.dtype).to(dev).eval()
            yl = torch.arange(B, device=dev) % 10
            cel = sample_rate(lambda: ddim.sample_with_cfg(cmodel, (B, 3, S, S), yl, cfg_scale=3.0), world)
            out[f"ddim{args.sample_steps}_cfg"] = {
                "value": round(world * B / cel, 2), "unit": "img/s", "batch_per_gpu": B, "steps": args.sample_steps,
                "cfg_scale": 3.0, "p_threshold": 0.995, "forward_batch": 2 * B, "seconds": round(cel, 3),
                "scaling": "replicas",
                "roofline": loop_roofline(2 * B * args.sample_steps * fwd_gf * 1e9, cel,
                                          f"whole DDIM-{args.sample_steps} CFG loop per GPU: forward FLOPs x 2B x "
                                          "steps")}
            del cmodel
    if args.dit and S == 32:
        model = trainer = None          # free the UNet's HBM before the DiT runs
        out["dit_s2_ddim50_cfg"] = dit_lines(args, dev, rank, world, B)
    if args.extra and S == 32 and not args.no_train and world == 1:
        # BASELINE config #5 beside the headline: the same network at 64x64 (CelebA), train + DDIM-100
        del model, trainer
        mp64 = dict(CIFAR, image_size=(64, 64))
        m64, tr64 = make_trainer(mp64, args.dtype, dev, rank, world)
        pool64 = [torch.rand(B, 3, 64, 64, device=dev, generator=gen) * 2 - 1 for _ in range(2)]
        m64.train()
        e64, _ = train_rate(tr64, pool64, 5, 3, world)
        graphed64 = tr64._bench_graphed
        m64.eval()
        d100 = DDIM(1000, 100, device=dev)
        s64 = sample_rate(lambda: d100.sample(m64, (B, 3, 64, 64)), world)
        gf64 = unet_flops_per_image(m64) / 1e9
        out["celeba64"] = {"train_img_s": round(world * B * 5 / e64, 2), "train_ms_per_step": round(e64 / 5 * 1e3, 3),
                           "ddim100_img_s": round(world * B / s64, 2), "ddim100_seconds": round(s64, 3),
                           "batch_per_gpu": B, "dtype": args.dtype, "steps_timed": 5, "graphed": graphed64,
                           "gflop_per_forward_img": round(gf64, 3),
                           "train_tflops_per_gpu": round(B * 5 / e64 * 3 * gf64 / 1e3, 2),
                           "roofline": loop_roofline(B * 5 * 3 * gf64 * 1e9, e64, "64x64 train step (fwd + bwd = 3x "
                                                     "forward FLOPs) per GPU"),
                           "ddim100_roofline": loop_roofline(B * 100 * gf64 * 1e9, s64, "whole DDIM-100 loop per GPU")}
        del m64, tr64
        if args.dtype == "bf16":
            # the reference's own arithmetic (fp32) on the same step, for comparison with the bf16 headline
            mf, trf = make_trainer(CIFAR, "fp32", dev, rank, world)
            mf.train()
            ef, _ = train_rate(trf, pool, 5, 3, world)
            out["fp32"] = {"train_img_s": round(world * B * 5 / ef, 2), "train_ms_per_step": round(ef / 5 * 1e3, 3),
                           "steps_timed": 5, "warmup": trf._bench_warmup, "graphed": trf._bench_graphed,
                           "note": "exact-fp32 MFMA (v_mfma_f32_16x16x4f32) parity mode"}
            del mf, trf
    if rank == 0 and not args.no_roofline:
        out["roofline"] = conv_roofline(dtype)
    if rank == 0 and world == 1 and not args.no_cpu:
        try:
            out["cpu_baseline"] = cpu_baseline()
            if f"ddim{args.sample_steps}" in out and S == 32:
                out[f"ddim{args.sample_steps}"]["cpu_baseline"] = cpu_ddim_baseline(S=args.sample_steps)
        except Exception as e:  # the CPU leg must never hide the GPU result
            out["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
