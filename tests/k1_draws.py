"""Inputs of the 1000-step trainer protocol (tests/golden/trainer_1k.npz), in ONE place: the fixture generator
(tests/golden/gen_golden.py), the CPU oracle test (test_oracle.py) and the GPU protocol (test_gpu_protocol.py) all
draw them here, so the fixture and the tests cannot drift apart."""
import numpy as np
import torch


def k1_draws(seeds, batch, steps, hw=16):
    """numpy PCG64 draws in step order, host-independent: x0 ~ U(-1, 1), t ~ U{0..999}, noise ~ N(0, 1) (float32),
    from the (x0, t, noise) seeds."""
    rx, rt, rn = (np.random.default_rng(int(s)) for s in seeds)
    shape = (int(batch), 3, hw, hw)
    xs, ts, ns = [], [], []
    for _ in range(int(steps)):
        xs.append(torch.from_numpy(rx.random(shape, dtype=np.float32) * np.float32(2) - np.float32(1)))
        ts.append(torch.from_numpy(rt.integers(0, 1000, (int(batch),), dtype=np.int64)))
        ns.append(torch.from_numpy(rn.standard_normal(shape, dtype=np.float32)))
    return xs, ts, ns


def k1_inputs(g):
    """The draws of a loaded trainer_1k fixture (its seeds, batch and step count)."""
    return k1_draws(g["seeds"], g["batch"], len(g["losses"]))
