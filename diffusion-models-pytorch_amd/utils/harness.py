"""Data-parallel sampling harness (reference scripts/sample_uncond.py:179-195,
scripts/sample_cfg.py:157-182), independent of the launcher.

One process per GPU. Each rank draws its own init noise (seeded seed + rank,
as accelerate's set_seed(device_specific=True)), samples a fold of `bspp`
images fully independently, and the fold is gathered once over the process
group in rank order (on GPUs: the C-ABI RCCL all-gather `dm_allgather_f32`, dmhip/comm.py; DM_GATHER=torch
selects torch.distributed's `all_gather_into_tensor` instead; gloo on CPU);
only the first `bs` images of each fold are kept, exactly as
`accelerator.gather(samples)[:bs]`.
"""
import math
import os
from typing import Callable, Iterable, List, Optional

import torch
import torch.distributed as dist

from utils.misc import amortize


class DistEnv:
    """Process-group view taken from torchrun / accelerate style env vars."""

    def __init__(self, backend: Optional[str] = None):
        self.world = int(os.environ.get('WORLD_SIZE', '1'))
        self.rank = int(os.environ.get('RANK', '0'))
        self.local_rank = int(os.environ.get('LOCAL_RANK', '0'))
        if torch.cuda.is_available():
            # one GPU per rank; more ranks than GPUs (a rehearsal of the N-GPU path) share them round-robin
            self.device = torch.device('cuda', self.local_rank % torch.cuda.device_count())
            torch.cuda.set_device(self.device)
        else:
            self.device = torch.device('cpu')
        # RCCL ("nccl") on GPUs; DM_DIST_BACKEND=gloo rehearses the multi-rank path over host memory
        self.backend = backend or os.environ.get('DM_DIST_BACKEND') or (
            'nccl' if self.device.type == 'cuda' else 'gloo')
        if self.world > 1 and not dist.is_initialized():
            kw = dict(device_id=self.device) if self.backend == 'nccl' else {}
            dist.init_process_group(self.backend, **kw)
        self._comm = None  # the C-ABI communicator (None: not set up yet; False: the torch path on every rank)
        self._checked = False

    @property
    def is_main(self):
        return self.rank == 0

    def barrier(self):
        if self.world > 1:
            dist.barrier()

    def gather(self, x: torch.Tensor) -> torch.Tensor:
        """Concatenate every rank's tensor along dim 0 in rank order (accelerate.gather)."""
        if self.world == 1:
            return x
        x = x.contiguous()
        out = torch.empty((self.world * x.shape[0], *x.shape[1:]), dtype=x.dtype, device=x.device)
        if (x.device.type == 'cuda' and self.backend == 'nccl' and x.dtype == torch.float32
                and os.environ.get('DM_GATHER') != 'torch' and self._comm is not False):
            if self._comm is None:   # RCCL communicator of the C ABI, bootstrapped once over the process group
                from dmhip.comm import Comm
                self._comm = Comm.try_from_process_group() or False  # False: every rank takes the torch path
            if self._comm is not False:
                self._comm.allgather(x, out)   # one RCCL all-gather over xGMI (dm_allgather_f32)
                if not self._checked:
                    self._check_gather(x, out)
                if self._comm is not False:
                    return out
            dist.all_gather_into_tensor(out, x)
        elif x.device.type == 'cuda' and self.backend == 'nccl':
            dist.all_gather_into_tensor(out, x)   # other dtypes (dm_allgather_f32 is float32 only)
        else:
            host = out.cpu() if out.device.type != 'cpu' else out
            dist.all_gather(list(host.chunk(self.world)), x.cpu())
            if host is not out:
                out.copy_(host)
        return out

    def _check_gather(self, x: torch.Tensor, out: torch.Tensor) -> None:
        """First gather at world > 1: the C-ABI all-gather against all_gather_into_tensor of the same
        fold; if any rank sees a difference, every rank drops to the torch path (agreed by an all-reduce)."""
        ref = torch.empty_like(out)
        dist.all_gather_into_tensor(ref, x)
        same = torch.tensor([1 if torch.equal(ref, out) else 0], dtype=torch.int32, device=out.device)
        dist.all_reduce(same, op=dist.ReduceOp.MIN)
        self._checked = True
        if int(same.item()) == 0:
            import sys
            print('dm_comm: dm_allgather_f32 differs from all_gather_into_tensor; using torch.distributed',
                  file=sys.stderr)
            self._comm.close()
            self._comm = False
            out.copy_(ref)

    def close(self):
        if self._comm:
            self._comm.close()
        self._comm = None
        if self.world > 1 and dist.is_initialized():
            dist.destroy_process_group()


def per_process_batch(n_samples: int, batch_size: int, world: int) -> int:
    """bspp of sample_uncond.py:182."""
    return min(batch_size, math.ceil(n_samples / world))


def sample_folds(sample_fn: Callable[[torch.Tensor], torch.Tensor], img_shape, n_samples: int, batch_size: int,
                 env: DistEnv, noise_fn: Callable[[tuple], torch.Tensor],
                 sink: Optional[Callable[[int, torch.Tensor], None]] = None) -> List[int]:
    """Run the fold loop of sample_uncond.py:179-195.

    sample_fn(init_noise) -> samples on this rank; noise_fn(shape) draws this
    rank's init noise; sink(first_index, images) receives the gathered images
    of a fold on rank 0. Returns the fold sizes."""
    bspp = per_process_batch(n_samples, batch_size, env.world)
    folds = amortize(n_samples, bspp * env.world)
    idx = 0
    for bs in folds:
        init_noise = noise_fn((bspp, *img_shape))
        samples = sample_fn(init_noise).clamp(-1, 1)
        samples = env.gather(samples)[:bs]
        if env.is_main and sink is not None:
            sink(idx, samples)
        idx += bs
    return folds
