"""ADM UNetModel / UNetCombined (models/adm/) on the MI355X path vs the reference.

Golden fixtures: tests/golden/adm.npz, made by tests/golden/make_golden.py from
the reference modules themselves (reduced archs at 16x16 and the full-size
RePaint CelebA-HQ / guided-diffusion combined 256x256 configs at B=1).
Tolerance: fp32 max-abs <= 1e-4 (north_star).
"""
import ctypes

import numpy as np
import pytest
import torch

from diffusions import DDIMCFG, DDPM
from models.adm.unet import UNetModel
from models.adm.unet_combined import UNetCombined
from utils.synthetic import init_synthetic_

TOL = 1e-4
TINY = ['adm_tiny', 'adm_tiny_conv', 'adm_tiny_pool']
FULL = ['adm256_celebahq', 'adm256_combined']


def _build(meta, name):
    arch = meta['archs'][name]
    return (UNetCombined if name.endswith('combined') else UNetModel)(**arch).eval()


@pytest.mark.parametrize('name', TINY)
def test_adm_state_dict_layout(golden, name):
    _, meta = golden('adm')
    m = _build(meta, name)
    assert [[k, list(v.shape)] for k, v in m.state_dict().items()] == meta[f'{name}_state_dict']


def test_adm_combined_state_dict_layout(golden):
    _, meta = golden('adm')
    m = UNetCombined(**meta['archs']['adm_tiny'])
    assert [[k, list(v.shape)] for k, v in m.state_dict().items()] == meta['combined_tiny_state_dict']


@pytest.mark.parametrize('name', TINY + FULL)
def test_adm_param_count_matches_abi(golden, name):
    from dmhip._lib import load
    _, meta = golden('adm')
    m = _build(meta, name)
    for sub in ([m.unet_cond, m.unet_uncond] if isinstance(m, UNetCombined) else [m]):
        n = ctypes.c_int()
        assert load().dm_unet_param_count(ctypes.byref(sub._arch_struct()), ctypes.byref(n)) == 0
        assert n.value == len(sub.state_dict()), name


def test_adm_refuses_fp16():
    with pytest.raises(NotImplementedError):
        UNetModel(32, 3, 32, 3, 1, [], use_fp16=True)


@pytest.mark.gpu
@pytest.mark.parametrize('name', TINY + FULL)
def test_adm_forward_vs_reference(cuda, golden, report, name):
    g, meta = golden('adm')
    model = _build(meta, name)
    assert init_synthetic_(model) == meta[f'{name}_weights_sha256']
    model = model.to(cuda)
    x = torch.from_numpy(g[f'{name}_x']).to(cuda)
    t = torch.from_numpy(g[f'{name}_t']).to(cuda)
    y = torch.from_numpy(g[f'{name}_labels']).to(cuda) if f'{name}_labels' in g else None
    out = model(x, t, y).cpu()
    err = (out - torch.from_numpy(g[f'{name}_out'])).abs().max().item()
    report(f'adm_forward_{name}_maxabs_vs_reference', err)
    assert err <= TOL, err
    del model
    torch.cuda.empty_cache()


@pytest.mark.gpu
def test_adm_label_contract(cuda, golden):
    _, meta = golden('adm')
    model = _build(meta, 'adm_tiny').to(cuda)
    x = torch.zeros((1, 3, 16, 16), device=cuda)
    t = torch.zeros((1, ), dtype=torch.long, device=cuda)
    with pytest.raises(AssertionError):
        model(x, t)  # class-conditional model needs y (adm/unet.py:662-664)
    with pytest.raises(IndexError):
        model(x, t, torch.tensor([5], device=cuda))


@pytest.mark.gpu
def test_adm_ddpm_learned_range_trajectory(cuda, golden, report):
    g, meta = golden('adm')
    model = _build(meta, 'adm_tiny')
    init_synthetic_(model)
    model = model.to(cuda)
    d = DDPM(var_type='learned_range', respace_type='uniform', respace_steps=8, device=cuda)
    noises = iter([torch.from_numpy(g[f'ddpm8_step{i}_noise']).to(cuda) for i in range(8)])
    d.noise_fn = lambda x: next(noises)
    d.skip_unused_noise = False
    labels = torch.from_numpy(g['ddpm8_labels']).to(cuda)
    worst = 0.0
    for i, out in enumerate(d.sample_loop(model, torch.from_numpy(g['ddpm8_init']).to(cuda),
                                          model_kwargs=dict(y=labels))):
        err = float(np.abs(out['sample'].cpu().numpy() - g[f'ddpm8_step{i}_sample']).max())
        worst = max(worst, err)
        assert err <= TOL, (i, err)
    report('adm_ddpm8_learned_range_maxabs_vs_reference', worst)


@pytest.mark.gpu
def test_adm_combined_ddimcfg_trajectory(cuda, golden, report):
    """Free-running DDIMCFG-6 through UNetCombined. Per-step parity is checked teacher-forced (each
    step starts from the reference's previous sample, so the bound is the single-step error); the
    free-running trajectory compounds the 3e-6 forward difference through x0 = sqrt(1/a_t) x - ...
    (sqrt(1/a_t) ~ 160 at t = 996) and the CFG combine (s = 2.5), so it gets a 5x looser bound."""
    g, meta = golden('adm')
    model = UNetCombined(**meta['archs']['adm_tiny']).eval()
    assert init_synthetic_(model) == meta['combined_tiny_weights_sha256']
    model = model.to(cuda)
    cfg = meta['cfg6']
    d = DDIMCFG(guidance_scale=cfg['guidance_scale'], respace_type=cfg['respace_type'],
                respace_steps=cfg['respace_steps'], eta=cfg['eta'], device=cuda)
    labels = torch.from_numpy(g['ddpm8_labels']).to(cuda)
    init = torch.from_numpy(g['cfg6_init']).to(cuda)
    # teacher-forced single steps
    seq = d.respaced_seq.tolist()
    pairs = list(zip(reversed(seq), reversed([-1] + seq[:-1])))
    worst_step = 0.0
    for i, (t, tp) in enumerate(pairs):
        x = init if i == 0 else torch.from_numpy(g[f'cfg6_step{i - 1}_sample']).to(cuda)
        tb = torch.full((2, ), t, dtype=torch.long, device=cuda)
        out = d._step(model(x, tb, labels), x, t, tp, model_output_uncond=model(x, tb, None),
                      guidance_scale=d.guidance_scale)
        err = float(np.abs(out['sample'].cpu().numpy() - g[f'cfg6_step{i}_sample']).max())
        worst_step = max(worst_step, err)
        assert err <= TOL, (i, err)
    report('adm_combined_ddimcfg6_single_step_maxabs_vs_reference', worst_step)
    worst = 0.0
    for i, out in enumerate(d.sample_loop(model, init, model_kwargs=dict(y=labels))):
        err = float(np.abs(out['sample'].cpu().numpy() - g[f'cfg6_step{i}_sample']).max())
        worst = max(worst, err)
        assert err <= 5 * TOL, (i, err)
    report('adm_combined_ddimcfg6_free_running_maxabs_vs_reference', worst)
