"""One sampling step captured as a HIP graph and replayed for the rest of a sampling loop.

A UNet sampling step is ~300 kernel launches whose Python/ctypes enqueue takes about as long as the GPU work
at small batch (the in-training sampler draws 16 images through 1000 DDPM steps, diffusion/ddpm.py:222-332,
utils/trainer.py:303-312). The step function is captured once with static input buffers; a replay copies the
new inputs in (device copies), launches the graph, and returns the static output (the next step copies it
back in, so the output buffer is never read and written by the same replay). Random draws happen OUTSIDE the
graph, eagerly and in the eager loop's order (`buf.normal_()` is what `torch.randn_like` does), so a graphed
loop computes bitwise what the eager loop computes (tests/test_gpu_model.py).

A loop whose step reads nothing but its inputs, the sampler's tables and the model's weights may keep its graph
on the sampler across sample() calls (`cache=`): the key holds the sampler's settings, the executor, the input
shapes and every parameter's (version, pointer) plus the executor's weight generation (bumped by the fused
optimizer / EMA kernels that write the parameters behind torch's back), so any weight update recaptures. The
entry holds the executor only weakly and is dropped once that executor is gone. Without a cache key a graph lives
for one call.

Destroying a HIP graph while this thread captures another is illegal. Round 5 saw exactly that: a dropped model
(then tied to its executor by a reference cycle) was freed by a cyclic collection that ran inside a capture. The
package's objects now hold no cycles (the executor refers to its model weakly), so they are freed at the `del`; as a
guard for cycles in user code, cyclic collection is paused during every capture (gc_paused).
"""
import collections
import contextlib
import gc
import os
import weakref

import torch


@contextlib.contextmanager
def gc_paused():
    """No cyclic garbage collection while a graph is captured: a collection can free an unreachable object's HIP
    graphs and memory, which is illegal on a capturing thread (seen as an abort inside a capture). No collection is
    forced here either (it would land inside whatever the caller times)."""
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


class StepGraph:
    def __init__(self, fn, *inputs, const=()):
        """const: positions of inputs that stay the same tensor through a loop (class labels): copied only when
        a different tensor, or a new torch version of it, is handed in."""
        self.static = [x.clone() for x in inputs]
        self.const = frozenset(const)
        # const inputs: (weak reference, version) of the tensor last copied in -- no strong reference to the caller's
        # tensors outlives the call
        self.seen = [(weakref.ref(x), x._version) if i in self.const else None for i, x in enumerate(inputs)]
        self.graph = torch.cuda.CUDAGraph()
        with gc_paused(), torch.cuda.graph(self.graph, capture_error_mode="thread_local"):   # see trainer.py begin()
            self.out = fn(*self.static)

    def step(self, *inputs):
        for i, (s, x) in enumerate(zip(self.static, inputs)):
            if x is None or x is s:
                continue
            if i in self.const and self.seen[i][0]() is x and self.seen[i][1] == x._version:
                continue
            s.copy_(x)
            if i in self.const:
                self.seen[i] = (weakref.ref(x), x._version)
        self.graph.replay()
        return self.out

    @staticmethod
    def eligible(model, x, deterministic, return_all):
        """DMC_GRAPH=0 / 1 turns the replay off / on; by default it is used for batches of <= 64, where the
        step's host enqueue (~2.8-3.1 ms for the CIFAR UNet) is at or above its GPU time. Measured DDIM-50 on one
        MI355X (scripts/ddim_probe.py, ms per call, eager / graphed / graph kept across calls): B=16 172 / 116 /
        110, B=64 155 / 143 / 134, B=128 178 / 187 / 179 -- at B=128 the step is GPU-bound and a replay runs no
        faster than the eager loop, so the first call's capture would only add its cost."""
        mode = os.environ.get("DMC_GRAPH")
        if mode == "0" or not deterministic or return_all or not x.is_cuda:
            return False
        if getattr(model, "executor", None) is None or model.training:
            return False
        return mode == "1" or x.shape[0] <= 64

    @staticmethod
    def weights_key(model):
        ex = getattr(model, "executor", None)
        return (getattr(ex, "wgen", None),) + tuple((p._version, p.data_ptr()) for p in model.parameters())


_CACHE_MAX = 2      # graphs kept per executor (each holds its activation pool)


def cache_for(model, tag, owner, x):
    """(store, key, executor) for run_loop(cache=...): the store lives on `owner`, the sampler whose tables the step
    reads. None for a model without an executor."""
    ex = getattr(model, "executor", None)
    if ex is None:
        return None
    store = owner.__dict__.setdefault("_step_graphs", collections.OrderedDict())
    for k in [k for k, (ref, _) in store.items() if ref() is None]:
        del store[k]       # a freed executor's graph (and its activation pool) goes with it
    return store, (tag, id(ex), tuple(x.shape), x.dtype, x.device, StepGraph.weights_key(model)), ex


def run_loop(x, nsteps, make_inputs, fn, use_graph, record=None, cache=None, const=()):
    """for i in range(nsteps): x = fn(*make_inputs(i, x)); eager for step 0 (caches and weight packs are then
    in place) and graphed afterwards when use_graph. make_inputs(i, x) -> tuple of tensors, x first. With a
    cache (cache_for) a graph from an earlier call with the same key replays from step 0."""
    graph = None
    if use_graph and cache is not None:
        store, key, ex = cache
        hit = store.get(key)
        if hit is not None and hit[0]() is ex:   # the same live executor (an id can be reused after a free)
            store.move_to_end(key)
            graph = hit[1]
    for i in range(nsteps):
        args = make_inputs(i, x)
        if graph is None and use_graph and i >= 1:
            prev = torch.cuda.current_stream()
            try:
                graph = StepGraph(fn, *args, const=const)
            except Exception as e:   # noqa: BLE001
                # loud, as the training step's capture (utils/trainer.py GraphCaptureError): the stream a failed
                # capture ran on may be poisoned, so the loop does not silently carry on eagerly on it. A failure in
                # capture_begin leaves torch.cuda.graph's side stream current (its __exit__ never runs): restore
                torch.cuda.set_stream(prev)
                from ..utils.trainer import GraphCaptureError
                raise GraphCaptureError(f"sampling step capture failed at step {i}: {e!r}") from e
            if cache is not None:
                store, key, ex = cache
                store[key] = (weakref.ref(ex), graph)
                while len(store) > _CACHE_MAX:
                    store.popitem(last=False)
        x = graph.step(*args) if graph is not None else fn(*args)
        if record is not None:
            record(i, x)
    return x.clone() if graph is not None else x
