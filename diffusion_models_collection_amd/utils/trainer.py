"""DiffusionTrainer with the reference API (utils/trainer.py of sunyzhi55/Diffusion_Models_Collection).

Same constructor (:37-49), config keys (:70-91), and methods train / train_epoch / sample_images /
save_checkpoint / load_checkpoint / cleanup, same checkpoint dict format (:336-348) and the same step
order (:221-273): t ~ randint -> p_losses -> backward -> clip_grad_norm(1.0) -> optimizer.step ->
zero_grad -> EMA.

What changes (MI355X-first):
  * data parallel: instead of wrapping the UNet in torch DDP, parameters are broadcast from rank 0 once
    and gradients are averaged with RCCL all-reduces over xGMI (torch.distributed backend "nccl" IS RCCL
    on ROCm) issued in ~25 MB buckets from inside the HIP backward as soon as each bucket's gradients are
    final, on RCCL's own stream, overlapping the rest of the backward (GradSync below). Other models
    fall back to torch DDP exactly like the reference.
  * clip_grad_norm_ and the EMA update are single fused multi-tensor kernels (dmc_clip_grad_norm,
    dmc_ema_update) instead of ~700 tiny launches; no host sync.
  * the loss is accumulated on device; the host reads it every `log_every` steps and at epoch end
    (the reference syncs twice per step via loss.item()).
"""
import math
import os
import time
import warnings
import weakref
from pathlib import Path

import torch
import torch.distributed as dist
from torch.nn.parallel import DistributedDataParallel as DDP
from tqdm import tqdm

from .. import kernels as K
from .helpers import resolve_image_size


def _is_dmc_model(m):
    """A backbone run by one of this package's executors (UNet, DiT): flat gradients, fused optimizer, graphs."""
    return type(m).__name__ in ("UNet", "DiT") and hasattr(m, "executor") and type(m).__module__.startswith(
        "diffusion_models_collection_amd")


class GradSync:
    """Bucketed, backward-overlapped gradient averaging over the UNet executor's flat gradient buffer.

    The executor lays gradients out in the order the backward finishes them and calls `hook(flat, hi,
    final)` after each layer with the length `hi` of the finished prefix. Every time >= bucket_bytes of new
    finished gradients exist, an async all-reduce of that slice is issued -- ReduceOp.AVG on RCCL (ncclAvg,
    the op every multi-rank run takes), SUM then a division on gloo; RCCL waits on the compute stream for the
    slice, then runs concurrently with the remaining backward kernels. At the end the compute stream waits for
    all of them (no host synchronisation).

    On a one-rank group the average is the identity and SUM is used (RCCL launches nothing for it, whereas a
    one-rank AVG runs its premultiplied-average kernel, ~130 us per 25 MB bucket on MI355X); force_avg=True
    keeps ReduceOp.AVG there too, so a single GPU exercises (and times) exactly the multi-rank code path.
    """

    def __init__(self, executor, process_group=None, bucket_bytes=25 * 1024 * 1024, force_avg=False):
        self._ex = weakref.ref(executor)    # the executor holds self.hook: no cycle back to it
        self.gtotal = executor.gtotal
        self.pg = process_group
        self.bucket = bucket_bytes // 4
        self.works = []
        self.done = 0
        # RCCL/NCCL averages natively (ncclAvg); gloo (CPU tests) has no AVG: sum, then scale
        self.native_avg = dist.get_backend(process_group) == "nccl"
        self.world = dist.get_world_size(process_group)
        self.op = dist.ReduceOp.AVG if self.native_avg and (self.world > 1 or force_avg) else dist.ReduceOp.SUM
        self.post_div = not self.native_avg and self.world > 1
        executor.grad_hook = self.hook

    TAIL = 256 * 1024      # elements: once at most this much is unfinished, flush what is finished

    def cut(self, hi, done, total, final):
        """Whether the finished prefix [done, hi) is issued now: a full bucket, the end of the backward, or all but
        a small tail finished (so the bucket left for after the backward is only that tail -- the UNet's input
        conv, whose gradient comes last)."""
        return hi > done and (hi - done >= self.bucket or final or total - hi <= self.TAIL)

    def wants(self, hi, final):
        """Whether hook(flat, hi, final) will issue an all-reduce (the executor then joins its side stream)."""
        return final or self.cut(hi, self.done, self.gtotal, final)

    def hook(self, flat, hi, final):
        if self.cut(hi, self.done, flat.numel(), final):
            seg = flat[self.done:hi]
            self.works.append((seg, dist.all_reduce(seg, op=self.op, group=self.pg, async_op=True)))
            self.done = hi
        if final:
            for seg, w in self.works:
                w.wait()          # makes the current stream wait for RCCL; no host sync
                if self.post_div:
                    seg.div_(self.world)
            self.works = []
            self.done = 0


class FlatAdamW:
    """clip_grad_norm_ + torch.optim.AdamW.step + EMA as one streaming kernel over flat fp32 buffers.

    The UNet's parameters are re-seated as views of one flat buffer laid out like the executor's flat
    gradient buffer (reverse module order), and so are the optimizer's exp_avg / exp_avg_sq (kept in
    `optimizer.state` in torch's own format, so optimizer.state_dict() and checkpoints are unchanged) and
    the EMA model's parameters. The step is then dmc_grad_norm_flat (norm + clip coefficient, on device)
    followed by dmc_adamw_flat (clip scaling, AdamW, EMA in one pass: ~36 B/parameter of HBM traffic
    instead of the ~700 launches of the reference's clip + foreach AdamW + per-tensor EMA).
    Used only when the optimizer is a plain torch.optim.AdamW over exactly the model's parameters;
    anything else takes the reference path (clip, optimizer.step(), EMA).
    """

    def __init__(self, model, optimizer, ema_model=None):
        self.model, self.opt, self.ema = model, optimizer, ema_model
        self.ex = model.executor
        self.params = list(model.parameters())
        self._bound = False

    @staticmethod
    def supported(model, optimizer):
        if type(optimizer) is not torch.optim.AdamW or len(optimizer.param_groups) != 1:
            return False
        g = optimizer.param_groups[0]
        if g.get("amsgrad") or g.get("maximize") or g.get("capturable") or g.get("differentiable"):
            return False
        mp = list(model.parameters())
        if {id(p) for p in g["params"]} != {id(p) for p in mp} or len(g["params"]) != len(mp):
            return False
        return all(p.dtype == torch.float32 and p.is_cuda and p.requires_grad for p in mp)

    def _bind(self):
        ex, dev = self.ex, self.params[0].device
        n = ex.gtotal
        self.flat_p = torch.empty(n, dtype=torch.float32, device=dev)
        self.flat_m = torch.zeros(n, dtype=torch.float32, device=dev)
        self.flat_v = torch.zeros(n, dtype=torch.float32, device=dev)
        self.slots = []
        st = self.opt.state
        steps = set()
        for i, p in enumerate(self.params):
            o = ex.goff[i]
            view = self.flat_p[o:o + p.numel()].view(p.shape)
            view.copy_(p.detach())
            p.data = view
            s = st.get(p)
            if s and "exp_avg" in s:
                self.flat_m[o:o + p.numel()].copy_(s["exp_avg"].reshape(-1))
                self.flat_v[o:o + p.numel()].copy_(s["exp_avg_sq"].reshape(-1))
                steps.add(float(s["step"]))
            self.slots.append((p, o))
        if len(steps) > 1:
            raise RuntimeError(f"FlatAdamW: parameters have different step counts {sorted(steps)}")
        self.t = int(steps.pop()) if steps else 0
        # one step tensor per parameter, as torch keeps them (a single shared tensor would be incremented once
        # per parameter by a plain torch AdamW that loads the checkpoint): 0-dim views of distinct elements of
        # one buffer, so a step updates all of them with one fill
        self.steps_base = torch.full((len(self.slots),), float(self.t), dtype=torch.float32)
        for i, (p, o) in enumerate(self.slots):
            st[p] = {"step": self.steps_base[i],
                     "exp_avg": self.flat_m[o:o + p.numel()].view(p.shape),
                     "exp_avg_sq": self.flat_v[o:o + p.numel()].view(p.shape)}
        self.state_obj = st
        self.flat_e = None
        if self.ema is not None:
            ep = dict(self.ema.named_parameters())
            names = [k for k, _ in self.model.named_parameters()]
            if set(ep) != set(names) or any(b.is_floating_point() for b in self.ema.buffers()):
                raise RuntimeError("FlatAdamW: EMA model layout differs from the model")
            self.flat_e = torch.empty(n, dtype=torch.float32, device=dev)
            for (p, o), k in zip(self.slots, names):
                e = ep[k]
                view = self.flat_e[o:o + p.numel()].view(p.shape)
                view.copy_(e.detach())
                e.data = view
            self.ema_params = [ep[k] for k in names]
        self.expect = [(p, self.flat_p.data_ptr() + 4 * o) for p, o in self.slots]
        if self.flat_e is not None:
            self.expect += [(e, self.flat_e.data_ptr() + 4 * o) for e, (_, o) in zip(self.ema_params, self.slots)]
        self._bound = True

    def _valid(self):
        """The flat binding still holds: nobody re-seated a parameter (model.to(...)), replaced the optimizer
        state (load_state_dict) or left gradients outside the executor's flat buffer (accumulation)."""
        if self.opt.state is not self.state_obj or any(p.data_ptr() != a for p, a in self.expect):
            return False
        st = self.opt.state
        return all(st.get(p, {}).get("exp_avg") is not None and
                   st[p]["exp_avg"].data_ptr() == self.flat_m.data_ptr() + 4 * o for p, o in self.slots[:1])

    def _sync_steps(self):
        self.steps_base.fill_(float(self.t))

    def grads_flat(self):
        flat = getattr(self.ex, "flat", None)
        if flat is None:
            return None
        base = flat.data_ptr()
        for p, o in self.slots:
            if p.grad is None or p.grad.data_ptr() != base + 4 * o:
                return None
        return flat

    def step(self, max_norm=1.0, ema_decay=None):
        """Returns the gradient norm (device scalar), or None when the flat path does not apply."""
        if not self._bound or not self._valid():
            self._bind()
        g = self.grads_flat()
        if g is None:
            # the caller falls back to torch's optimizer.step(): give every parameter its own step counter
            # (torch increments each one) and re-bind from the optimizer state next time
            self._sync_steps()
            self._bound = False
            return None
        total, coef = K.grad_norm_flat(g, max_norm if max_norm is not None else -1.0)
        sc = self.scalars(ema_decay)
        K.adamw_flat(self.flat_p, g, self.flat_m, self.flat_v, self.flat_e if self.uses_ema(ema_decay) else None,
                     coef, *sc)
        self.bump(ema_decay)
        return total

    def uses_ema(self, ema_decay):
        return self.flat_e is not None and ema_decay is not None

    def scalars(self, ema_decay):
        """Advance the step count; the nine dmc_adamw_flat scalars of this step, in double like torch:
        (1-lr*wd, 1-beta1, beta2, 1-beta2, eps, -lr/(1-beta1^t), sqrt(1-beta2^t), ema decay, 1-ema decay)."""
        grp = self.opt.param_groups[0]
        lr, (b1, b2), eps, wd = float(grp["lr"]), grp["betas"], grp["eps"], grp["weight_decay"]
        self.t += 1
        self.steps_base.fill_(float(self.t))
        bc1 = 1 - b1 ** self.t
        bc2 = 1 - b2 ** self.t
        use_ema = self.uses_ema(ema_decay)
        return (1 - lr * wd, 1 - b1, b2, 1 - b2, eps, (lr / bc1) * -1, bc2 ** 0.5,
                ema_decay if use_ema else 1.0, (1 - ema_decay) if use_ema else 0.0)

    def bump(self, ema_decay):
        """The parameters (and EMA) changed: the executors repack their weights on the next forward."""
        self.ex.wgen += 1
        if self.uses_ema(ema_decay):
            self.ema.executor.wgen += 1


class GraphCaptureError(RuntimeError):
    """The training step's HIP graph capture failed (GraphedTrainStep.step)."""


class GraphedTrainStep:
    """The training step captured once as a HIP graph and replayed (single process, fused optimizer path).

    An eager step is ~950 kernel launches whose Python/ctypes enqueue costs about as much host time as the
    GPU needs to run them (bench.py host_enqueue_ms_per_step); a replay is one graph launch. Everything
    that differs per step stays outside the graph, with the eager step's RNG calls in the eager order: the
    batch and labels are copied into static buffers, t (torch.randint) and the noise (torch.randn_like) are
    drawn eagerly into static buffers, and the dropout seed (torch's CPU generator, as the eager forward
    draws it) and the nine AdamW/EMA scalars go to device memory with one pinned H2D copy per step; the
    captured kernels read them there (drop_seed_base, dmc_adamw_flat_dev). Replays are therefore bitwise
    identical to eager steps (tests/test_gpu_model.py). Captured after WARM eager steps, once per batch
    shape; a step with another shape runs eagerly. A capture failure raises GraphCaptureError: the failed
    capture may have left the stream's error state poisoned, so the step is never retried eagerly on it (set
    DMC_GRAPH=0 to train without graphs).

    `replays` counts graph replays (bench.py records whether every timed step was one). With `measure_comm` set, a
    data-parallel replay records two events on the compute stream: once the last segment that hands a bucket to
    RCCL is enqueued, and after the compute stream's waits for every bucket -- their distance is the
    communication the backward did not hide (comm_ms()).
    """
    WARM = 2
    RING = 4

    def __init__(self, trainer):
        self._tr = weakref.ref(trainer)     # the trainer holds this step (trainer._graph): no cycle back to it
        self.calls = 0
        self.replays = 0
        self.ring_wait_s = 0.0       # host seconds spent waiting for a pinned ring slot (paces the host to the GPU)
        self.graph = None
        self.failed = False
        self.key = None
        self.measure_comm = False
        self.comm_events = []
        self.comm_in_graph = False     # data parallel: the RCCL all-reduces are inside the one step graph
        self.capture_fallback = None   # why that capture was not possible (the segmented chain runs instead)

    @property
    def tr(self):
        return self._tr()

    @staticmethod
    def supported(trainer):
        import os
        return (os.environ.get("DMC_GRAPH", "1") != "0"
                and (not trainer.is_distributed or trainer.grad_sync is not None)
                and trainer._flat is not None and trainer.gradient_accumulation_steps == 1
                and _is_dmc_model(trainer._raw_model))

    def _key(self, images, y):
        return (tuple(images.shape), images.device, None if y is None else tuple(y.shape))

    def _capture(self, images, y):
        tr = self.tr
        f = tr._flat
        dev = images.device
        ex = tr._raw_model.executor
        self.segs = None
        self.x_s = torch.empty_like(images)
        self.n_s = torch.empty_like(images)
        self.t_s = torch.empty(images.shape[0], dtype=torch.long, device=dev)
        self.y_s = None if y is None else torch.empty_like(y)
        self.h_dev = torch.zeros(16, dtype=torch.float32, device=dev)   # [0..8] AdamW scalars, [9] seed
        self.ring = [torch.zeros(16, dtype=torch.float32).pin_memory() for _ in range(self.RING)]
        self.ring_ev = [None] * self.RING
        self.slot = 0
        self.use_ema = f.uses_ema(tr.ema_decay if tr.use_ema else None)
        drop_on = tr._raw_model.training and tr._raw_model.dropout > 0
        self.drop_on = drop_on
        ex.wgen += 1                      # the captured forward must contain the weight-pack launch
        ex.seed_ptr = self.h_dev.data_ptr() + 9 * 4
        try:
            gs = tr.grad_sync
            self.comm_in_graph = False
            if gs is not None and gs.native_avg and os.environ.get("DMC_DDP_CAPTURE", "0") == "1":
                # opt-in: RCCL collectives captured into the one step graph (no graph boundaries, no host-side
                # collective calls per step); any failure falls back to the segmented chain below. Measured slower
                # on one MI355X (one-rank AVG: 12.27 vs 11.94 ms per step, 11.43 for the plain graph): the replayed
                # graph runs the collective branch in line with the compute instead of beside it, which with real
                # inter-GPU traffic would expose all of it
                try:
                    self._capture_direct(ex, f, comm_in_graph=True)
                    self.comm_in_graph = True
                except Exception as e:   # noqa: BLE001
                    warnings.warn(f"capturing the RCCL all-reduces into the step graph failed ({e!r}); "
                                  "using the segmented graph chain")
                    self.capture_fallback = repr(e)
                    gs.works, gs.done = [], 0
                    torch.cuda.synchronize()
            if not self.comm_in_graph:
                self._capture_direct(ex, f)
        finally:
            ex.seed_ptr = None
        tr.optimizer.zero_grad()

    def _capture_direct(self, ex, f, comm_in_graph=False):
        """The step captured straight from the executor, without autograd: one graph -- with the RCCL all-reduces
        captured inside it when comm_in_graph (GradSync.hook runs during the capture: the collectives go on RCCL's
        stream behind event edges from the compute stream, and the optimizer segment waits for them; round 6) --
        or (gloo, DMC_DDP_CAPTURE=0, or a failed comm capture) a chain of graphs cut at the all-reduce points.

        No autograd node takes part in a capture. Round 6 found why that matters: a caller that still holds the
        previous step's loss (the reference loop keeps `loss` alive across iterations, utils/trainer.py:249-268)
        keeps that step's AccumulateGrad nodes alive, whose stream is the default stream; autograd then syncs the
        capturing stream with the default stream inside the capture, and hipStreamEndCapture crashed the process
        (tests/test_gpu_model.py::test_graphed_capture_with_previous_loss_alive).

        The step runs without autograd (q_sample -> executor forward -> loss -> executor backward, all on this
        thread) so that the bucket hook of the backward can end the current capture and begin the next one at
        every point where GradSync would issue an all-reduce. The collectives themselves are never captured:
        a replay launches segment i, then issues bucket i's all-reduce eagerly on RCCL's stream (it waits for
        segment i on the device and overlaps segment i+1), and before the last segment (grad norm, clip,
        AdamW, EMA) the compute stream waits for every bucket. Host cost per step: ~8 graph launches and ~7
        collective calls instead of ~950 kernel launches. All segments share one memory pool and replay in
        capture order."""
        tr = self.tr
        gs = tr.grad_sync
        dev = self.x_s.device
        pool = torch.cuda.graph_pool_handle()
        stream = torch.cuda.Stream(device=dev)
        stream.wait_stream(torch.cuda.current_stream())
        segs = []                                        # [(graph, (lo, hi) or None)]
        state = {"g": None, "done": 0}

        def begin():
            state["g"] = torch.cuda.CUDAGraph()
            # thread-local capture: the process group's watchdog thread polls the earlier all-reduce events
            # (hipEventQuery) while this thread captures; under the default global mode that query is illegal and
            # aborts the process (seen on MI355X with a one-rank RCCL group)
            state["g"].capture_begin(pool=pool, capture_error_mode="thread_local")

        def end(bucket):
            state["g"].capture_end()
            segs.append((state["g"], bucket))

        def hook(flat, hi, final):
            if comm_in_graph:
                gs.hook(flat, hi, final)   # async all-reduces (and the final waits) captured into this graph
                return
            if gs.cut(hi, state["done"], flat.numel(), final):
                end((state["done"], hi))
                state["done"] = hi
                begin()

        # the executor joins its weight-gradient side stream only where a segment ends (True here
        # serialised the side stream after every record of every captured segment)
        hook.wants = gs.wants if comm_in_graph else (lambda hi, final: final or gs.cut(hi, state["done"], ex.gtotal,
                                                                                        final))
        self.one = torch.ones((), dtype=torch.float32, device=dev)
        old_hook = ex.grad_hook
        ex.grad_hook = hook if gs is not None else None
        try:
            with torch.cuda.stream(stream):
                begin()
                xt = tr.diffusion.q_sample(self.x_s, self.t_s, self.n_s)
                pred, tape = ex.forward(xt, self.t_s, self.y_s, keep=True)
                lt = tr.loss_type
                if lt not in ("l1", "l2", "huber"):
                    raise ValueError(f"Unknown loss type: {lt}")
                pred = pred.contiguous()
                loss = K.loss_fwd(lt, pred, self.n_s)
                dpred = K.loss_bwd(lt, pred, self.n_s, self.one)
                ex.backward(tape, dpred, False)
                del tape
                _, coef = K.grad_norm_flat(ex.flat, 1.0)
                K.adamw_flat_dev(f.flat_p, ex.flat, f.flat_m, f.flat_v, f.flat_e if self.use_ema else None, coef,
                                 self.h_dev)
                end(None)
        except Exception:
            if state["g"] is not None:
                try:
                    state["g"].capture_end()
                except Exception:   # noqa: BLE001
                    pass
            raise
        finally:
            ex.grad_hook = old_hook
        torch.cuda.current_stream().wait_stream(stream)
        self.segs = segs if gs is not None and not comm_in_graph else None
        self.graph, self.loss_s = segs[-1][0], loss.detach()
        self.flat = ex.flat

    def _replay(self):
        self.replays += 1
        if self.segs is None:
            self.graph.replay()
            return
        gs = self.tr.grad_sync
        works = []
        for g, bucket in self.segs:
            if bucket is None:
                if self.measure_comm:
                    e0 = torch.cuda.Event(enable_timing=True)
                    e0.record()       # after the backward's last bucketed segment
                for seg, w in works:
                    w.wait()          # the compute stream waits for RCCL; no host sync
                    if gs.post_div:
                        seg.div_(gs.world)
                if self.measure_comm:
                    e1 = torch.cuda.Event(enable_timing=True)
                    e1.record()
                    self.comm_events.append((e0, e1))
            g.replay()
            if bucket is not None:
                seg = self.flat[bucket[0]:bucket[1]]
                works.append((seg, dist.all_reduce(seg, op=gs.op, group=gs.pg, async_op=True)))

    def step(self, images, t, y):
        """One training step; returns the loss, or None when this step must run eagerly."""
        self.calls += 1
        if self.failed or self.calls <= self.WARM:
            return None
        tr = self.tr
        f = tr._flat
        if not f._bound or not f._valid():
            return None
        key = self._key(images, y)
        if self.graph is None or key != self.key:
            if self.graph is not None:
                return None           # one captured shape (the last, ragged batch of an epoch runs eagerly)
            prev = torch.cuda.current_stream()
            from ..diffusion._graph import gc_paused
            try:
                with gc_paused():   # a guard: the package's own objects hold no reference cycles
                    self._capture(images, y)
                self.key = key
            except Exception as e:    # noqa: BLE001
                # loud: round 3 saw the eager retry of a failed capture fail on the same stream ("operation
                # failed due to a previous error during capture"). A capture_begin that raises inside
                # torch.cuda.graph's __enter__ leaves its capture stream current: restore the caller's.
                torch.cuda.set_stream(prev)
                self.failed = True
                self.graph = None
                raise GraphCaptureError(
                    "training-step HIP graph capture failed; the step is not retried eagerly on a possibly "
                    "poisoned stream (set DMC_GRAPH=0 to train without graphs)") from e
        from ..models._unet_exec import _seed_from_torch
        self.x_s.copy_(images)
        self.t_s.copy_(t)
        self.n_s.copy_(torch.randn_like(images))       # p_losses' draw, same generator and order
        if y is not None:
            self.y_s.copy_(y)
        ema_decay = tr.ema_decay if tr.use_ema else None
        h = torch.zeros(16, dtype=torch.float32)
        h[:9] = torch.tensor(f.scalars(ema_decay), dtype=torch.float32)
        if self.drop_on:
            h.view(torch.int32)[9] = _seed_from_torch()
        k = self.slot % self.RING
        self.slot += 1
        if self.ring_ev[k] is not None:
            t0 = time.perf_counter()
            self.ring_ev[k].synchronize()      # the pinned slot's previous copy has been consumed
            self.ring_wait_s += time.perf_counter() - t0
        self.ring[k].copy_(h)
        self.h_dev.copy_(self.ring[k], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.ring_ev[k] = ev
        self._replay()
        f.bump(ema_decay)
        return self.loss_s.clone()

    def comm_ms(self):
        """Mean exposed-communication ms over the replays measured since the last call (measure_comm)."""
        if not self.comm_events:
            return None
        self.comm_events[-1][1].synchronize()
        v = sum(a.elapsed_time(b) for a, b in self.comm_events) / len(self.comm_events)
        self.comm_events = []
        return v


class DiffusionTrainer:
    """Trainer for diffusion models (utils/trainer.py:21-421)."""

    def __init__(self, model, diffusion, train_loader, optimizer, scheduler=None, device='cuda', config=None, rank=0,
                 world_size=1, resume_path=None):
        self.device = device
        self.rank = rank
        self.world_size = world_size
        self.is_distributed = world_size > 1
        self.is_main_process = rank == 0

        self.model = model.to(device)
        self._raw_model = self.model
        self.grad_sync = None
        if self.is_distributed:
            if _is_dmc_model(self.model):
                # DDP's init broadcast, then gradient averaging from inside the HIP backward
                with torch.no_grad():
                    for t in list(self.model.parameters()) + list(self.model.buffers()):
                        dist.broadcast(t, src=0)
                self.grad_sync = self._make_grad_sync(config)
            else:
                self.model = DDP(model)

        self.diffusion = diffusion
        self.train_loader = train_loader
        self.optimizer = optimizer
        self.scheduler = scheduler

        self.config = config or {}
        self.epochs = self.config.get('epochs', 100)
        self.save_dir = Path(self.config.get('save_dir', './checkpoints'))
        self.sample_dir = Path(self.config.get('sample_dir', './generated_images'))
        self.loss_type = self.config.get('loss_type', 'l2')
        self.gradient_accumulation_steps = self.config.get('gradient_accumulation_steps', 1)
        self.save_interval = self.config.get('save_interval', 10)
        self.sample_interval = self.config.get('sample_interval', 5)
        self.sample_start_epoch = self.config.get('sample_start_epoch', 20)
        self.num_samples = self.config.get('num_samples', 16)
        self.cfg_dropout_prob = self.config.get('cfg_dropout_prob', 0.2)
        self.cfg_scale = self.config.get('cfg_scale', 1.8)
        self.use_ema = self.config.get('use_ema', False)
        self.ema_decay = self.config.get('ema_decay', 0.9999)
        self.use_swanlab = self.config.get('use_swanlab', False)
        self.conditional = self.config.get('conditional', False)
        self.num_classes = self.config.get('num_classes', None)
        self.image_size = resolve_image_size(self.config.get('image_size', 32))
        self.model_type = self.config.get('model_type', 'unet').lower()
        self.model_params = self.config.get('model_params', {}).copy()
        self.in_channels = self.model_params.get('in_channels', 3)
        self.log_every = self.config.get('log_every', 20)

        if self.is_main_process:
            self.save_dir.mkdir(parents=True, exist_ok=True)
            self.sample_dir.mkdir(parents=True, exist_ok=True)

        if self.use_ema and self.is_main_process:
            self.ema_model = self._create_ema_model()
        else:
            self.ema_model = None
        self._ema_refs = None
        self._clip_refs = None
        self._flat = None
        if _is_dmc_model(self._module) and FlatAdamW.supported(self._module, optimizer) and (
                self.ema_model is None or _is_dmc_model(self.ema_model)):
            self._flat = FlatAdamW(self._module, optimizer, self.ema_model)
        self._graph = GraphedTrainStep(self) if GraphedTrainStep.supported(self) else None

        self.best_loss = float('inf')
        self.start_epoch = 1
        if resume_path:
            self.load_checkpoint(resume_path)

        if self.use_swanlab and self.is_main_process:
            import swanlab
            swanlab.init(project=self.config.get('project_name', 'diffusion-models'),
                         experiment_name=self.config.get('experiment_name', 'experiment'), config=self.config)

    # ------------------------------------------------------------------------------------------
    def _make_grad_sync(self, config, process_group=None, force_avg=False):
        # bucket size: the reference's DDP default (25 MB); 'ddp_bucket_mb' (not a reference key) or the
        # DMC_DDP_BUCKET_MB environment variable overrides. 'ddp_force_avg' (not a reference key): ReduceOp.AVG
        # even on a one-rank RCCL group (GradSync)
        import os
        bmb = float((config or {}).get('ddp_bucket_mb', os.environ.get('DMC_DDP_BUCKET_MB', 25)))
        force_avg = force_avg or bool((config or {}).get('ddp_force_avg', False))
        return GradSync(self.model.executor, process_group=process_group, bucket_bytes=int(bmb * 1024 * 1024),
                        force_avg=force_avg)

    def enable_grad_sync(self, process_group=None, force_avg=False):
        """Average gradients over `process_group` (default: the initialised default group) from inside the HIP
        backward even when this trainer was built with world_size 1 -- the data-parallel step (GradSync + the
        segmented graph) on a one-rank group, used to exercise and time the RCCL path on a single GPU
        (force_avg: the ReduceOp.AVG every multi-rank run takes instead of the one-rank SUM). On a group of more
        ranks the parameters and buffers are first broadcast from the group's first rank, as the constructor's
        distributed path does, and the trainer becomes distributed."""
        if not dist.is_initialized() or not _is_dmc_model(self._raw_model):
            raise RuntimeError("enable_grad_sync needs an initialised process group and a dmc backbone")
        if dist.get_world_size(process_group) > 1:
            src = dist.get_global_rank(process_group, 0) if process_group is not None else 0
            with torch.no_grad():
                for t in list(self._raw_model.parameters()) + list(self._raw_model.buffers()):
                    dist.broadcast(t, src=src, group=process_group)
            self.is_distributed = True
        self.grad_sync = self._make_grad_sync(self.config, process_group, force_avg)
        self._graph = GraphedTrainStep(self) if GraphedTrainStep.supported(self) else None
        return self.grad_sync

    @property
    def _module(self):
        return self.model.module if isinstance(self.model, DDP) else self.model

    def load_checkpoint(self, checkpoint_path):
        print(f"Loading checkpoint from {checkpoint_path}...")
        checkpoint = torch.load(checkpoint_path, map_location=self.device, weights_only=True)
        self._module.load_state_dict(checkpoint['model_state_dict'])
        if 'optimizer_state_dict' in checkpoint and self.optimizer:
            self.optimizer.load_state_dict(checkpoint['optimizer_state_dict'])
        if 'scheduler_state_dict' in checkpoint and self.scheduler:
            self.scheduler.load_state_dict(checkpoint['scheduler_state_dict'])
        if 'ema_model_state_dict' in checkpoint and self.ema_model:
            self.ema_model.load_state_dict(checkpoint['ema_model_state_dict'])
        self.start_epoch = checkpoint.get('epoch', 0) + 1
        self.best_loss = checkpoint.get('best_loss', float('inf'))
        print(f"Resuming training from epoch {self.start_epoch}")
        if self.start_epoch > self.epochs:
            print(f"Checkpoint epoch ({self.start_epoch-1}) is greater than configured epochs ({self.epochs}).")
            print(f"Extending training by {self.config.get('epochs', 100)} epochs...")
            self.epochs = self.start_epoch + self.config.get('epochs', 100)
            print(f"New target epochs: {self.epochs}")

    def _create_ema_model(self):
        src = self._module
        ema_model = type(src)(**self._get_model_params()).to(self.device)
        if hasattr(src, "compute_dtype") and hasattr(ema_model, "set_compute_dtype"):
            ema_model.set_compute_dtype("bf16" if src.compute_dtype == torch.bfloat16 else "fp32")
        ema_model.load_state_dict(src.state_dict())
        ema_model.eval()
        for param in ema_model.parameters():
            param.requires_grad = False
        return ema_model

    def _get_model_params(self):
        params = self.model_params.copy()
        params['num_classes'] = self.num_classes if self.conditional else None
        return params

    def _update_ema(self):
        """ema = d*ema + (1-d)*theta over the state_dict (utils/trainer.py:187-202), one fused launch."""
        if self.ema_model is None:
            return
        ema_sd = self.ema_model.state_dict()
        msd = self._module.state_dict()
        pairs = [(ema_sd[k], msd[k]) for k in ema_sd if ema_sd[k].is_floating_point()]
        key = tuple((a.data_ptr(), b.data_ptr()) for a, b in pairs)
        if self._ema_refs is None or self._ema_refs[0] != key:
            self._ema_refs = (key, K.TensorRefs(pairs, pairs[0][0].device))
        K.ema_update(self._ema_refs[1], self.ema_decay)
        if getattr(self.ema_model, "executor", None) is not None:
            self.ema_model.executor.wgen += 1      # raw-pointer update: the EMA executor must repack its weights

    def _clip(self, max_norm=1.0):
        """torch.nn.utils.clip_grad_norm_(params, max_norm) as one fused multi-tensor launch."""
        grads = [p.grad for p in self._module.parameters() if p.grad is not None]
        if not grads:
            return None
        key = tuple(g.data_ptr() for g in grads)
        if self._clip_refs is None or self._clip_refs[0] != key:
            self._clip_refs = (key, K.TensorRefs([(g, None) for g in grads], grads[0].device))
        return K.clip_grad_norm(self._clip_refs[1], max_norm)

    def train_step(self, batch, i=0):
        """One iteration of the reference loop body (utils/trainer.py:222-265); returns the scaled loss."""
        if self.conditional:
            images, labels = batch
            labels = labels.to(self.device)
            labels_for_loss = labels + 1
            if self.cfg_dropout_prob > 0 and self.num_classes is not None:
                drop_mask = torch.rand_like(labels.float()) < self.cfg_dropout_prob
                labels_for_loss = labels_for_loss.clone()
                labels_for_loss[drop_mask] = 0
        else:
            images = batch[0] if isinstance(batch, (list, tuple)) else batch
            labels_for_loss = None
        images = images.to(self.device, non_blocking=True)
        batch_size = images.shape[0]
        t = torch.randint(0, self.diffusion.num_timesteps, (batch_size,), device=self.device).long()
        if self._graph is not None and self._module.training:
            loss = self._graph.step(images, t, labels_for_loss)
            if loss is not None:
                return loss
        loss = self.diffusion.p_losses(self.model, images, t, labels_for_loss, loss_type=self.loss_type)
        loss = loss / self.gradient_accumulation_steps
        loss.backward()
        if (i + 1) % self.gradient_accumulation_steps == 0:
            fused = self._flat is not None and self._flat.step(
                1.0, self.ema_decay if (self.use_ema and self.ema_model is not None) else None) is not None
            if fused:
                self.optimizer.zero_grad()
            else:
                self._clip(1.0)
                self.optimizer.step()
                self.optimizer.zero_grad()
                if self.use_ema:
                    self._update_ema()
        return loss.detach()    # a caller holding it must not keep this step's autograd graph (and tape) alive

    def train_epoch(self, epoch):
        self.model.train()
        total_loss = torch.zeros((), dtype=torch.float32, device=self.device)
        num_batches = 0
        if self.is_distributed and hasattr(self.train_loader, "sampler") and hasattr(self.train_loader.sampler,
                                                                                     "set_epoch"):
            self.train_loader.sampler.set_epoch(epoch)
        elif hasattr(self.train_loader, "set_epoch"):
            self.train_loader.set_epoch(epoch)      # the device loader's flip hash is keyed by the epoch
        progress_bar = tqdm(self.train_loader, desc=f"Epoch {epoch}/{self.epochs}", disable=not self.is_main_process)
        self.optimizer.zero_grad()
        for i, batch in enumerate(progress_bar):
            loss = self.train_step(batch, i)
            total_loss += loss.detach() * self.gradient_accumulation_steps
            num_batches += 1
            if self.is_main_process and (i + 1) % self.log_every == 0:
                progress_bar.set_postfix({'loss': loss.item() * self.gradient_accumulation_steps})
        avg = total_loss / max(num_batches, 1)
        if self.is_distributed:
            dist.all_reduce(avg, op=dist.ReduceOp.AVG)
        return avg.item()

    @torch.no_grad()
    def sample_images(self, epoch, num_samples=None):
        from torchvision.utils import save_image  # optional dependency of the reference (image files)
        if num_samples is None:
            num_samples = self.num_samples
        model = self.ema_model if self.ema_model is not None else self._module
        model.eval()
        h, w = self.image_size
        shape = (num_samples, self.in_channels, h, w)
        nrow = max(1, int(math.sqrt(num_samples)))
        if self.conditional and self.num_classes:
            num_rows = (num_samples + nrow - 1) // nrow
            row_labels = torch.arange(num_rows, device=self.device) % self.num_classes
            labels = (row_labels + 1).repeat_interleave(nrow)[:num_samples]
            print(f"Sampling with labels: {labels.cpu().numpy()}")
            samples = self.diffusion.sample_with_cfg(model, shape, labels, cfg_scale=self.cfg_scale)
        else:
            samples = self.diffusion.sample(model, shape, None)
        samples = torch.clamp((samples + 1) / 2, 0, 1)
        save_image(samples, str(self.sample_dir / f'epoch_{epoch:04d}.png'), nrow=nrow)
        if self.use_swanlab:
            import swanlab
            swanlab.log({'samples': swanlab.Image(samples)}, step=epoch)
        return samples

    def save_checkpoint(self, epoch, is_best=False):
        if not self.is_main_process:
            return
        checkpoint = {
            'epoch': epoch,
            'model_state_dict': self._module.state_dict(),
            'optimizer_state_dict': self.optimizer.state_dict(),
            'best_loss': self.best_loss,
            'config': self.config,
        }
        if self.scheduler is not None:
            checkpoint['scheduler_state_dict'] = self.scheduler.state_dict()
        if self.ema_model is not None:
            checkpoint['ema_model_state_dict'] = self.ema_model.state_dict()
        torch.save(checkpoint, self.save_dir / 'current_model.pth')
        if is_best:
            torch.save(checkpoint, self.save_dir / 'best_model.pth')
        if epoch % self.save_interval == 0:
            torch.save(checkpoint, self.save_dir / f'model_epoch_{epoch:04d}.pth')

    def train(self):
        if self.is_main_process:
            print(f"Starting training for {self.epochs} epochs")
            print(f"Device: {self.device}")
            print(f"Distributed: {self.is_distributed} (World size: {self.world_size})")
        for epoch in range(self.start_epoch, self.epochs + 1):
            start_time = time.time()
            avg_loss = self.train_epoch(epoch)
            if self.scheduler is not None:
                self.scheduler.step()
            epoch_time = time.time() - start_time
            if self.is_main_process:
                lr = self.optimizer.param_groups[0]['lr']
                print(f"Epoch {epoch}/{self.epochs} - Loss: {avg_loss:.4f} - LR: {lr:.6f} - Time: {epoch_time:.2f}s")
                if self.use_swanlab:
                    import swanlab
                    swanlab.log({'train/loss': avg_loss, 'train/lr': lr, 'train/epoch_time': epoch_time}, step=epoch)
            is_best = avg_loss < self.best_loss
            if is_best:
                self.best_loss = avg_loss
            if self.is_main_process:
                self.save_checkpoint(epoch, is_best)
            if self.is_main_process and epoch >= self.sample_start_epoch and epoch % self.sample_interval == 0:
                print(f"Generating samples at epoch {epoch}...")
                self.sample_images(epoch)
        if self.is_main_process:
            print("Training completed!")
            if self.use_swanlab:
                import swanlab
                swanlab.finish()

    def cleanup(self):
        if self.is_distributed:
            dist.destroy_process_group()
