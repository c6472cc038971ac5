"""Deterministic synthetic weights.

No checkpoints are available offline, and the reference's own default init
makes some denoisers output exactly zero, so benchmarks and parity runs use
this rank-independent recipe over the reference state_dict keys, in order,
drawn from one numpy PCG64 stream (seed 0 by default):
  * tensors with ndim >= 2:   U(-1/sqrt(fan_in), +1/sqrt(fan_in)), fan_in = numel / shape[0]
  * 1-D '*.weight' (norms):   1
  * 1-D '*.bias':             U(-0.01, +0.01)
  * DiT 'pos_embed':          the fixed 2-D sin-cos table (dit/model.py:193-194), no draws
Each other tensor consumes numel float32 draws U[0,1) mapped to the range.
"""
import hashlib
from typing import Dict

import numpy as np
import torch


def _sincos_2d(embed_dim: int, grid_size: int) -> np.ndarray:
    """MAE / DiT fixed position table (dit/model.py:278-325), float64 [grid^2, embed_dim]."""
    def one_d(dim, pos):
        omega = np.arange(dim // 2, dtype=np.float64)
        omega /= dim / 2.
        omega = 1. / 10000 ** omega
        out = np.einsum('m,d->md', pos.reshape(-1), omega)
        return np.concatenate([np.sin(out), np.cos(out)], axis=1)
    gh = np.arange(grid_size, dtype=np.float32)
    gw = np.arange(grid_size, dtype=np.float32)
    grid = np.stack(np.meshgrid(gw, gh), axis=0).reshape([2, 1, grid_size, grid_size])
    return np.concatenate([one_d(embed_dim // 2, grid[0]), one_d(embed_dim // 2, grid[1])], axis=1)


def synthetic_state_dict(state_dict_like: Dict[str, torch.Tensor], seed: int = 0) -> Dict[str, torch.Tensor]:
    rng = np.random.Generator(np.random.PCG64(seed))
    out = {}
    for name, ref in state_dict_like.items():
        shape = tuple(ref.shape)
        n = int(np.prod(shape)) if shape else 1
        if name == 'pos_embed' or name.endswith('.pos_embed'):
            grid = int(round(np.sqrt(shape[-2])))
            vals = _sincos_2d(shape[-1], grid).astype(np.float32)
        elif len(shape) >= 2:
            bound = 1.0 / np.sqrt(n / shape[0])
            u = rng.random(n, dtype=np.float32)
            vals = ((u * 2.0 - 1.0) * bound).astype(np.float32)
        elif name.endswith('weight'):
            vals = np.ones(n, dtype=np.float32)
        else:
            u = rng.random(n, dtype=np.float32)
            vals = ((u * 2.0 - 1.0) * 0.01).astype(np.float32)
        out[name] = torch.from_numpy(vals.reshape(shape))
    return out


def init_synthetic_(model: torch.nn.Module, seed: int = 0):
    """Load the synthetic weights into `model` in place; returns their sha256."""
    sd = synthetic_state_dict(model.state_dict(), seed)
    model.load_state_dict(sd)
    return state_dict_sha256(sd)


def state_dict_sha256(sd: Dict[str, torch.Tensor]) -> str:
    h = hashlib.sha256()
    for k, v in sd.items():
        h.update(k.encode())
        h.update(v.detach().cpu().contiguous().numpy().tobytes())
    return h.hexdigest()
