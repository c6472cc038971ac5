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


def _bench(args, env_extra):
    import json
    import subprocess
    env = dict(os.environ, DM_DIST_BACKEND='gloo', MASTER_ADDR='127.0.0.1')
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_PORT'):
        env.pop(k, None)
    env.update(env_extra)
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py')] + args, env=env, capture_output=True,
                       text=True, timeout=240)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{')]
    return p.returncode, [json.loads(ln) for ln in lines], p.stderr


def test_bench_gpus2_launches_two_ranks():
    """`bench.py --gpus 2` with no launcher starts the two ranks itself (fresh child processes, before any GPU
    call) and forwards rank 0's line: n_gpus 2, the global batch of both ranks, barrier + max-over-ranks timing."""
    rc, lines, err = _bench(['--gpus', '2', '--workload', 'stub', '--steps', '2', '--warmup', '1'], {})
    assert rc == 0, err
    assert len(lines) == 1, (lines, err)
    line = lines[0]
    assert line['n_gpus'] == 2 and line['config']['global_batch'] == 8 and line['config']['parallelism'] == 'dp2'
    assert line['value'] > 0 and line['steps'] == 2
    # the fold's gather path is named in the line (on GPUs: the C-ABI RCCL all-gather, dm_allgather_f32)
    assert line['config']['gather'] == 'gloo (host)', line['config']
    # the per-rank record: every rank's device and own fold time, the group's size, the
    # gather check's outcome; on GPUs also the RCCL communicator's own rank count (dm_comm_info)
    rk = line['ranks']
    assert rk['process_group_size'] == 2 and rk['backend'] == 'gloo', rk
    assert [r['rank'] for r in rk['per_rank']] == [0, 1], rk
    assert all(r['device'] == 'cpu' and r['fold_ms'] > 0 for r in rk['per_rank']), rk
    assert max(r['fold_ms'] for r in rk['per_rank']) <= line['ms_per_step'] + 0.01, (rk, line['ms_per_step'])
    assert rk['gather_check'].startswith('not run (gloo'), rk
    assert rk['comm_nranks'] is None, rk


def test_bench_single_rank_has_no_rank_record():
    rc, lines, err = _bench(['--workload', 'stub', '--steps', '1', '--warmup', '0'], {})
    assert rc == 0, err
    assert lines[0]['ranks'] is None and lines[0]['n_gpus'] == 1


def test_bench_rejects_gpus_world_mismatch():
    rc, lines, err = _bench(['--gpus', '1', '--workload', 'stub'], {'WORLD_SIZE': '2', 'RANK': '0'})
    assert rc == 2 and not lines and 'WORLD_SIZE=2' in err
