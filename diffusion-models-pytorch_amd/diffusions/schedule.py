"""Beta schedules and respaced timestep sequences.

Host-side index/scalar arithmetic, kept bit-identical to the reference
(diffusions/schedule.py:5-73): the tables are built with the same torch CPU
ops and dtypes (float64 linspace for linear/quad/const, a float32 tensor from
a Python list for cosine, int64 index sequences), so every downstream
coefficient matches the reference bit for bit.
"""
import math

import torch

_BETA_SCHEDULES = ('linear', 'quad', 'const', 'cosine')
_RESPACE_TYPES = ('uniform', 'uniform-leading', 'uniform-linspace', 'uniform-trailing', 'quad', 'none', None)


def _cosine_alpha_bar(s: float) -> float:
    return math.cos((s + 0.008) / 1.008 * math.pi / 2) ** 2


def get_beta_schedule(
        total_steps: int = 1000,
        beta_schedule: str = 'linear',
        beta_start: float = 0.0001,
        beta_end: float = 0.02,
):
    """Return the [total_steps] beta table (reference schedule.py:5-38).

    'linear', 'quad', 'const' are float64; 'cosine' (improved DDPM) is built
    in Python floats and converted with torch.tensor (float32), as upstream.
    """
    if beta_schedule == 'linear':
        return torch.linspace(beta_start, beta_end, total_steps, dtype=torch.float64)
    if beta_schedule == 'quad':
        root = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, total_steps, dtype=torch.float64)
        return root ** 2
    if beta_schedule == 'const':
        return torch.full((total_steps, ), fill_value=beta_end, dtype=torch.float64)
    if beta_schedule == 'cosine':
        out = []
        for i in range(total_steps):
            ratio = _cosine_alpha_bar((i + 1) / total_steps) / _cosine_alpha_bar(i / total_steps)
            out.append(min(1 - ratio, 0.999))
        return torch.tensor(out)
    raise ValueError(f'Beta schedule {beta_schedule} is not supported.')


def get_respaced_seq(
        total_steps: int = 1000,
        respace_type: str = 'uniform',
        respace_steps: int = 100,
):
    """Timestep indices kept for sampling (reference schedule.py:41-73).

    Note the upstream quirks reproduced on purpose: 'uniform' uses
    arange(0, T, T // S) and may return more than S entries (1000/300 -> 334);
    'quad' may repeat indices.
    """
    if respace_type in ('uniform', 'uniform-leading'):
        return torch.arange(0, total_steps, total_steps // respace_steps).long()
    if respace_type == 'uniform-linspace':
        return torch.linspace(0, total_steps - 1, respace_steps).long()
    if respace_type == 'uniform-trailing':
        step = total_steps // respace_steps
        return torch.arange(total_steps - 1, -1, -step).long().flip(dims=[0])
    if respace_type == 'quad':
        grid = torch.linspace(0, math.sqrt(total_steps * 0.8), respace_steps) ** 2
        return torch.floor(grid).long()
    if respace_type is None or respace_type == 'none':
        return torch.arange(0, total_steps).long()
    raise ValueError(f'Respace type {respace_type} is not supported.')
