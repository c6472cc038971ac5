"""The C-ABI all-gather of the sampling harness (include/dm_hip.h dm_comm_*, csrc/comm.hip).

Replaces accelerate's `accelerator.gather(samples)` of each rank's finished fold (reference
scripts/sample_uncond.py:190, scripts/sample_cfg.py:177): one RCCL all-gather in rank order, enqueued on
the caller's HIP stream. The communicator is bootstrapped RCCL's way -- rank 0 draws the unique id, which
reaches the other ranks over the process group the launcher already set up (`from_process_group`); every
later gather goes through the C ABI only.
"""
import ctypes
from typing import Optional

import torch

from dmhip._lib import check, load, require_device_tensor, stream_handle

UID_BYTES = 128   # DM_COMM_UID_BYTES


def unique_id() -> bytes:
    """dm_comm_unique_id: the bootstrap id rank 0 hands to every rank."""
    buf = ctypes.create_string_buffer(UID_BYTES)
    check(load().dm_comm_unique_id(buf), 'dm_comm_unique_id')
    return buf.raw


class Comm:
    """One rank's RCCL communicator on the current HIP device (dm_comm_init)."""

    def __init__(self, uid: bytes, nranks: int, rank: int, device: Optional[torch.device] = None):
        if len(uid) != UID_BYTES:
            raise ValueError(f'unique id must be {UID_BYTES} bytes, got {len(uid)}')
        if device is not None:
            torch.cuda.set_device(device)
        self.device = torch.device('cuda', torch.cuda.current_device())
        h = ctypes.c_void_p()
        check(load().dm_comm_init(ctypes.create_string_buffer(uid, UID_BYTES), nranks, rank, ctypes.byref(h)),
              'dm_comm_init')
        self._h = h
        self.nranks, self.rank = nranks, rank

    @classmethod
    def from_process_group(cls, group=None) -> 'Comm':
        """Bootstrap over an initialised torch.distributed group (gloo or RCCL): rank 0's id is broadcast.
        Raises on every rank together if any rank could not set up its communicator (try_from_process_group)."""
        comm = cls.try_from_process_group(group)
        if comm is None:
            raise RuntimeError('dm_comm: the C-ABI communicator could not be set up on every rank')
        return comm

    @classmethod
    def try_from_process_group(cls, group=None) -> Optional['Comm']:
        """The communicator on every rank, or None on every rank (the ranks agree). Rank 0 always
        broadcasts -- the unique id, or None when RCCL cannot be loaded -- and the ranks then all-reduce whether
        their dm_comm_init succeeded, so a failure on any rank sends all of them to the torch.distributed path
        together instead of leaving collectives paired wrongly."""
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        uid = None
        if rank == 0:
            try:
                uid = unique_id()
            except (RuntimeError, ValueError, OSError):
                uid = None
        obj = [uid]
        dist.broadcast_object_list(obj, src=0, group=group)
        if obj[0] is None:
            return None
        comm = None
        try:
            comm = cls(obj[0], world, rank)
        except (RuntimeError, ValueError, OSError):
            comm = None
        backend = dist.get_backend(group)
        dev = torch.device('cuda', torch.cuda.current_device()) if backend == 'nccl' else torch.device('cpu')
        ok = torch.tensor([1 if comm is not None else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)
        if int(ok.item()) == 0:
            if comm is not None:
                comm.close()
            return None
        return comm

    def info(self):
        n, r, d = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(load().dm_comm_info(self._h, ctypes.byref(n), ctypes.byref(r), ctypes.byref(d)), 'dm_comm_info')
        return n.value, r.value, d.value

    def allgather(self, x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """[n, ...] float32 on this rank's device -> [nranks * n, ...], rank r's rows at r * n (accelerate's
        gather order)."""
        if self._h is None:
            raise RuntimeError('dm_comm: communicator already destroyed')
        require_device_tensor(x, 'x')
        shape = (self.nranks * x.shape[0], *x.shape[1:]) if x.dim() else (self.nranks, )
        if out is None:
            out = torch.empty(shape, dtype=torch.float32, device=x.device)
        else:
            require_device_tensor(out, 'out')
            if tuple(out.shape) != shape:
                raise ValueError(f'dm_comm: out must have shape {shape}, got {tuple(out.shape)}')
        check(load().dm_allgather_f32(self._h, x.data_ptr(), out.data_ptr(), x.numel(), stream_handle(x.device)),
              'dm_allgather_f32')
        return out

    def close(self):
        if self._h is not None:
            load().dm_comm_destroy(self._h)
            self._h = None
