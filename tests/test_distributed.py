"""World-size-2 gloo rehearsal of the multi-GPU path (one process per GPU, batch
sharded, one all-gather per fold) — reference scripts/sample_uncond.py:179-195."""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'diffusion-models-pytorch_amd')


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir, n_samples, batch_size):
    sys.path.insert(0, PKG)
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    from utils.harness import DistEnv, sample_folds
    env = DistEnv(backend='gloo')
    gen = torch.Generator().manual_seed(2022 + env.rank)   # set_seed(seed, device_specific=True)
    received = []

    def sample_fn(z):
        # stand-in for diffuser.sample: tags every image with its rank and draws, values in (-1, 1)
        return torch.tanh(z) * 0.5 + 0.25 * env.rank

    def sink(idx, imgs):
        received.append((idx, imgs.clone()))

    folds = sample_folds(sample_fn, (1, 2, 2), n_samples, batch_size, env,
                         noise_fn=lambda shape: torch.randn(shape, generator=gen), sink=sink)
    torch.save(dict(folds=folds, received=received), os.path.join(out_dir, f'rank{rank}.pt'))
    env.close()


@pytest.mark.parametrize('n_samples,batch_size', [(10, 4), (8, 8), (3, 4)])
def test_gloo_world2_fold_gather(tmp_path, n_samples, batch_size):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), n_samples, batch_size), nprocs=world, join=True)
    r0 = torch.load(tmp_path / 'rank0.pt', weights_only=True)
    r1 = torch.load(tmp_path / 'rank1.pt', weights_only=True)
    import math
    bspp = min(batch_size, math.ceil(n_samples / world))
    full, rest = divmod(n_samples, bspp * world)
    assert r0['folds'] == [bspp * world] * full + ([rest] if rest else [])
    assert r1['received'] == []                 # only rank 0 writes images
    assert sum(imgs.shape[0] for _, imgs in r0['received']) == n_samples
    # regenerate each rank's noise stream and check the gathered order: rank 0's fold first, then rank 1's
    gens = [torch.Generator().manual_seed(2022 + r) for r in range(world)]
    for (idx, imgs), bs in zip(r0['received'], r0['folds']):
        parts = [torch.tanh(torch.randn((bspp, 1, 2, 2), generator=gens[r])) * 0.5 + 0.25 * r for r in range(world)]
        expect = torch.cat(parts)[:bs].clamp(-1, 1)
        assert torch.equal(imgs, expect)
