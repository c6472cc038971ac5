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
    """DDIMCFG-6 through UNetCombined. Every step teacher-forced (from the reference's previous
    sample) <= 1e-4; free-running, tests/conftest.py check_free_running: the reference's own fp32 run
    drifts 1.6e-4 from its float64 run on this trajectory (x0 = sqrt(1/a_t) x - ... with
    sqrt(1/a_t) ~ 160 at t = 996, times the (2s - 1) CFG gain; tests/golden/drift.npz cfg6)."""
    from tests.conftest import check_chaos_envelope, check_free_running
    dg = golden('drift')[0]
    drift = dg['cfg6_drift_sample']
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
    worst, worst64 = 0.0, 0.0
    for i, out in enumerate(d.sample_loop(model, init, model_kwargs=dict(y=labels))):
        e32, e64 = check_free_running(out['sample'].cpu().numpy(), g[f'cfg6_step{i}_sample'],
                                      dg['cfg6_sample64'][i], drift, i)
        worst, worst64 = max(worst, e32), max(worst64, e64)
    report('adm_combined_ddimcfg6_free_running_maxabs_vs_reference', worst)
    report('adm_combined_ddimcfg6_free_running_maxabs_vs_reference_float64', worst64)
    report('adm_combined_ddimcfg6_reference_fp32_vs_fp64_drift', float(drift.max()))
    check_chaos_envelope(golden, 'cfg6', worst64, report, 'adm_combined_ddimcfg6')


@pytest.mark.gpu
def test_adm_combined_ddpmcfg_learned_range_trajectory(cuda, golden, report):
    """DDPMCFG-8 (s = 2.5) with var_type learned_range through UNetCombined (two weight sets, two calls
    per step, reference diffusions/ddpm.py:319-351): eps halves combined, the CONDITIONAL branch's
    variance channels concatenated (:344-345), learned-range variance (:240-246), noise pinned per
    step (tests/golden/ddpmcfg.npz). Every step teacher-forced (from the reference's previous sample):
    sample and pred_eps <= 1e-4; free-running: tests/conftest.py check_free_running on the sample."""
    from diffusions import DDPMCFG
    from tests.conftest import check_free_running
    from tests.golden.noise import StepNoise
    g, meta = golden('ddpmcfg')
    model = UNetCombined(**golden('adm')[1]['archs']['adm_tiny']).eval()
    assert init_synthetic_(model) == meta['combined_tiny_weights_sha256']
    model = model.to(cuda)
    c = meta['adm']
    d = DDPMCFG(guidance_scale=c['guidance_scale'], var_type=c['var_type'], respace_type=c['respace_type'],
                respace_steps=c['respace_steps'], device=cuda)
    labels = torch.from_numpy(g['adm_labels']).to(cuda)
    seq = d.respaced_seq.tolist()
    worst_step = 0.0
    for i, (t, tp) in enumerate(zip(reversed(seq), reversed([-1] + seq[:-1]))):
        x = torch.from_numpy(g['adm_init'] if i == 0 else g[f'adm_step{i - 1}_sample']).to(cuda)
        src = StepNoise(c['noise_seed'])
        src.k = i   # the i-th draw of the trajectory
        d.noise_fn = src
        tb = torch.full((2, ), t, dtype=torch.long, device=cuda)
        out = d._step(model(x, tb, labels), x, t, tp, model_output_uncond=model(x, tb, None),
                      guidance_scale=d.guidance_scale)
        for k in ('sample', 'pred_eps'):
            err = float(np.abs(out[k].cpu().numpy() - g[f'adm_step{i}_{k}']).max())
            worst_step = max(worst_step, err)
            assert err <= TOL, (i, k, err)
    src = StepNoise(c['noise_seed'])
    d.noise_fn = src
    worst = 0.0
    for i, out in enumerate(d.sample_loop(model, torch.from_numpy(g['adm_init']).to(cuda),
                                          model_kwargs=dict(y=labels))):
        e32, _ = check_free_running(out['sample'].cpu().numpy(), g[f'adm_step{i}_sample'], g['adm_sample64'][i],
                                    g['adm_drift_sample'], i)
        worst = max(worst, e32)
    assert i + 1 == len(seq) and src.k == i + 1
    report('adm_combined_ddpmcfg8_learned_range_single_step_maxabs_vs_reference', worst_step)
    report('adm_combined_ddpmcfg8_learned_range_free_running_maxabs_vs_reference', worst)


@pytest.mark.gpu
def test_adm256_batch_invariance(cuda, golden, report):
    """BASELINE config C4's model (the guided-diffusion 256x256 UNetCombined arch) at its batch size:
    a B=64 forward of the conditional network, whose row 0 is the pinned B=1 reference input
    (tests/golden/adm.npz adm256_combined, checked <= 1e-4 against the reference), equals B=1
    forwards of rows 0, 31 and 63 bit for bit, so the B=1 reference parity extends to B=64."""
    g, meta = golden('adm')
    model = UNetCombined(**meta['archs']['adm256_combined']).eval()
    init_synthetic_(model)
    net = model.unet_cond.to(cuda)
    gen = torch.Generator().manual_seed(64)
    B = 64
    x = torch.randn((B, 3, 256, 256), generator=gen)
    x[0] = torch.from_numpy(g['adm256_combined_x'][0])
    t = torch.randint(0, 1000, (B, ), generator=gen)
    t[0] = int(g['adm256_combined_t'][0])
    y = torch.randint(0, 1000, (B, ), generator=gen)
    y[0] = int(g['adm256_combined_labels'][0])
    x, t, y = x.to(cuda), t.to(cuda), y.to(cuda)
    big = net(x, t, y)
    err = (big[0].cpu() - torch.from_numpy(g['adm256_combined_out'][0])).abs().max().item()
    report('adm256_combined_B64_row0_maxabs_vs_reference', err)
    assert err <= TOL, err
    for r in (0, 31, 63):
        one = net(x[r:r + 1].contiguous(), t[r:r + 1].contiguous(), y[r:r + 1].contiguous())
        assert torch.equal(big[r:r + 1], one), r
    assert torch.isfinite(big).all()
    del net, model, big
    torch.cuda.empty_cache()
