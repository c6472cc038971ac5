"""Deterministic synthetic weights.

No checkpoints are available offline, and the reference's own default init
makes some denoisers output exactly zero, so benchmarks and parity runs use
this rank-independent recipe over the reference state_dict keys, in order,
drawn from one numpy PCG64 stream (seed 0 by default):
  * tensors with ndim >= 2:   U(-1/sqrt(fan_in), +1/sqrt(fan_in)), fan_in = numel / shape[0]
  * 1-D '*.weight' (norms):   1
  * 1-D '*.bias':             U(-0.01, +0.01)
Each tensor consumes numel float32 draws U[0,1) mapped to the range.
"""
import hashlib
from typing import Dict

import numpy as np
import torch


def synthetic_state_dict(state_dict_like: Dict[str, torch.Tensor], seed: int = 0) -> Dict[str, torch.Tensor]:
    rng = np.random.Generator(np.random.PCG64(seed))
    out = {}
    for name, ref in state_dict_like.items():
        shape = tuple(ref.shape)
        n = int(np.prod(shape)) if shape else 1
        if len(shape) >= 2:
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
