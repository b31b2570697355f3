"""One sampling step captured as a HIP graph and replayed for the rest of a sampling loop.

A UNet sampling step is ~300 kernel launches whose Python/ctypes enqueue takes about as long as the GPU work
at small batch (the in-training sampler draws 16 images through 1000 DDPM steps, diffusion/ddpm.py:222-332,
utils/trainer.py:303-312). The step function is captured once with static input buffers; a replay copies the
new inputs in (device copies), launches the graph, and returns the static output (the next step copies it
back in, so the output buffer is never read and written by the same replay). Random draws happen OUTSIDE the
graph, eagerly and in the eager loop's order (`buf.normal_()` is what `torch.randn_like` does), so a graphed
loop computes bitwise what the eager loop computes (tests/test_gpu_model.py). A graph lives for one sample()
call: the weights may change between calls.
"""
import os

import torch


class StepGraph:
    def __init__(self, fn, *inputs):
        self.static = [x.clone() for x in inputs]
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):   # see utils/trainer.py begin()
            self.out = fn(*self.static)

    def step(self, *inputs):
        for s, x in zip(self.static, inputs):
            if x is not None and x is not s:
                s.copy_(x)
        self.graph.replay()
        return self.out

    @staticmethod
    def eligible(model, x, deterministic, return_all):
        """DMC_GRAPH=0 / 1 turns the replay off / on; by default it is used for batches of <= 32, where the
        step's host enqueue exceeds its GPU time (at B=128 the step is GPU-bound and a per-call capture only
        adds its own cost: 569 vs 602 img/s measured for DDIM-50)."""
        mode = os.environ.get("DMC_GRAPH")
        if mode == "0" or not deterministic or return_all or not x.is_cuda:
            return False
        if getattr(model, "executor", None) is None or model.training:
            return False
        return mode == "1" or x.shape[0] <= 32


def run_loop(x, nsteps, make_inputs, fn, use_graph, record=None):
    """for i in range(nsteps): x = fn(*make_inputs(i, x)); eager for step 0 (caches and weight packs are then
    in place) and graphed afterwards when use_graph. make_inputs(i, x) -> tuple of tensors, x first."""
    graph = None
    for i in range(nsteps):
        args = make_inputs(i, x)
        if graph is None and use_graph and i >= 1:
            prev = torch.cuda.current_stream()
            try:
                graph = StepGraph(fn, *args)
            except Exception as e:   # noqa: BLE001
                # loud, as the training step's capture (utils/trainer.py GraphCaptureError): the stream a failed
                # capture ran on may be poisoned, so the loop does not silently carry on eagerly on it. A failure in
                # capture_begin leaves torch.cuda.graph's side stream current (its __exit__ never runs): restore
                torch.cuda.set_stream(prev)
                from ..utils.trainer import GraphCaptureError
                raise GraphCaptureError(f"sampling step capture failed at step {i}: {e!r}") from e
        x = graph.step(*args) if graph is not None else fn(*args)
        if record is not None:
            record(i, x)
    return x.clone() if graph is not None else x
