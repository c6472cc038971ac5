"""Deterministic per-step noise for long fixture trajectories (test infrastructure).

The reference draws `torch.randn_like(xt)` every step (diffusions/ddpm.py:251,
diffusions/ddim.py:76). Storing 1000 steps of CIFAR noise would make a 25 MB
fixture, so the generator (make_golden.py) replaces that draw with this
source while it runs the reference, and the GPU tests install the same source
as the engine's `noise_fn`: draw k of a trajectory is numpy PCG64 seeded
[seed, k], standard normal in float32 (numpy's float32 ziggurat is
platform-independent). Only the RNG is substituted; every arithmetic step of
the reference is unchanged.
"""
import numpy as np
import torch


class StepNoise:
    def __init__(self, seed: int):
        self.seed = seed
        self.k = 0

    def draw(self, shape) -> np.ndarray:
        rng = np.random.Generator(np.random.PCG64([self.seed, self.k]))
        self.k += 1
        return rng.standard_normal(tuple(shape), dtype=np.float32)

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        """randn_like replacement: same shape, x's dtype and device."""
        return torch.from_numpy(self.draw(x.shape)).to(device=x.device, dtype=x.dtype)
