"""The C-ABI all-gather (include/dm_hip.h dm_comm_*, csrc/comm.hip) that replaces accelerate's gather of each
rank's fold (reference scripts/sample_uncond.py:190, scripts/sample_cfg.py:177).

CPU: argument checks that need no RCCL or GPU. GPU: a one-rank communicator (the box has one GPU; RCCL does not
put two ranks on one device) -- bootstrap, rank/size, an all-gather that must return its input bit for bit, in
place and out of place; the N-rank gather order itself is covered by the gloo tests of the harness
(tests/test_distributed.py) and runs over RCCL in the driver's multi-GPU bench (bench.py, DM_GATHER=torch: the
torch.distributed path instead)."""
import ctypes
import os
import socket

import pytest
import torch

import dmhip
from dmhip._lib import DM_ERR_ARG


def test_comm_argument_checks_without_rccl_calls():
    L = dmhip.load()
    h = ctypes.c_void_p()
    uid = ctypes.create_string_buffer(128)
    assert L.dm_comm_init(None, 1, 0, ctypes.byref(h)) == DM_ERR_ARG
    assert L.dm_comm_init(uid, 2, 2, ctypes.byref(h)) == DM_ERR_ARG
    assert b'rank must lie' in L.dm_last_error()
    assert L.dm_comm_init(uid, 0, 0, ctypes.byref(h)) == DM_ERR_ARG
    assert L.dm_allgather_f32(None, None, None, 4, None) == DM_ERR_ARG
    assert L.dm_comm_unique_id(None) == DM_ERR_ARG
    assert L.dm_comm_info(None, None, None, None) == DM_ERR_ARG
    L.dm_comm_destroy(None)   # no-op


def test_comm_rejects_bad_uid_length():
    from dmhip.comm import Comm
    with pytest.raises(ValueError):
        Comm(b'x' * 16, 1, 0)


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_comm_one_rank_allgather_is_identity(cuda):
    import torch.distributed as dist
    from dmhip.comm import Comm
    dist.init_process_group('gloo', init_method=f'tcp://127.0.0.1:{_free_port()}', rank=0, world_size=1)
    try:
        comm = Comm.from_process_group()
        assert comm.info() == (1, 0, torch.device(cuda).index or 0)
        g = torch.Generator().manual_seed(5)
        x = torch.randn((3, 3, 32, 32), generator=g).to(cuda)
        y = comm.allgather(x)
        torch.cuda.synchronize()
        assert y.shape == x.shape and torch.equal(y, x)
        out = torch.empty_like(x)
        comm.allgather(x, out)
        buf = x.clone()
        comm.allgather(buf, buf)   # in place: send = recv + rank x count
        torch.cuda.synchronize()
        assert torch.equal(out, x) and torch.equal(buf, x)
        with pytest.raises(ValueError):
            comm.allgather(x, torch.empty((2, 3, 32, 32), device=cuda))
        assert comm.allgather(torch.empty((0, 3), device=cuda)).shape == (0, 3)
        comm.close()
        with pytest.raises(RuntimeError):
            comm.allgather(x)
    finally:
        dist.destroy_process_group()
