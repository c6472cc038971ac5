"""UNetCategorialAdaGN (models/unet_categorial_adagn.py) on the MI355X path vs the reference.

Golden fixtures: tests/golden/adagn.npz, made by tests/golden/make_golden.py from
the reference module itself. Tolerance: fp32 max-abs <= 1e-4 (north_star).
"""
import numpy as np
import pytest
import torch

from diffusions import DDIMCFG
from models.unet_categorial_adagn import UNetCategorialAdaGN
from utils.synthetic import init_synthetic_

TOL = 1e-4
NAMES = ['tiny_updown', 'tiny_conv', 'cfg_cifar10']


def _model(meta, name):
    m = UNetCategorialAdaGN(**meta['archs'][name]).eval()
    sha = init_synthetic_(m)
    return m, sha


@pytest.mark.parametrize('name', NAMES)
def test_adagn_state_dict_layout(golden, name):
    _, meta = golden('adagn')
    m = UNetCategorialAdaGN(**meta['archs'][name])
    assert [[k, list(v.shape)] for k, v in m.state_dict().items()] == meta[f'{name}_state_dict']


def test_adagn_param_count_matches_abi(golden):
    """dm_unet_param_count (no GPU needed) walks the same registration order as the module."""
    import ctypes
    from dmhip._lib import load
    _, meta = golden('adagn')
    for name in NAMES:
        m = UNetCategorialAdaGN(**meta['archs'][name])
        n = ctypes.c_int()
        rc = load().dm_unet_param_count(ctypes.byref(m._arch_struct()), ctypes.byref(n))
        assert rc == 0 and n.value == len(m.state_dict()), name


@pytest.mark.gpu
@pytest.mark.parametrize('name', NAMES)
def test_adagn_forward_vs_reference(cuda, golden, report, name):
    g, meta = golden('adagn')
    model, sha = _model(meta, name)
    assert sha == meta[f'{name}_weights_sha256']
    model = model.to(cuda)
    x = torch.from_numpy(g[f'{name}_x']).to(cuda)
    t = torch.from_numpy(g[f'{name}_t']).to(cuda)
    y = torch.from_numpy(g[f'{name}_labels']).to(cuda)
    out_y = model(x, t, y).cpu()
    out_n = model(x, t, None).cpu()
    e_y = (out_y - torch.from_numpy(g[f'{name}_out_y'])).abs().max().item()
    e_n = (out_n - torch.from_numpy(g[f'{name}_out_none'])).abs().max().item()
    report(f'adagn_forward_{name}_y_maxabs_vs_reference', e_y)
    report(f'adagn_forward_{name}_none_maxabs_vs_reference', e_n)
    assert e_y <= TOL and e_n <= TOL, (e_y, e_n)
    # per-row null label (y = -1, inside the CFG samplers' scope) equals the y=None call
    import dmhip
    with dmhip.null_label_scope():
        mixed = model(x, t, torch.tensor([-1, int(g[f'{name}_labels'][1])], device=cuda)).cpu()
    assert torch.equal(mixed[0], out_n[0])
    assert torch.equal(mixed[1], out_y[1])


@pytest.mark.gpu
def test_adagn_label_out_of_range(cuda, golden):
    _, meta = golden('adagn')
    model, _ = _model(meta, 'tiny_updown')
    model = model.to(cuda)
    x = torch.zeros((1, 3, 16, 16), device=cuda)
    t = torch.zeros((1, ), dtype=torch.long, device=cuda)
    with pytest.raises(IndexError):
        model(x, t, torch.tensor([5], device=cuda))


@pytest.mark.gpu
@pytest.mark.parametrize('batched', [True, False])
def test_ddimcfg_trajectory_vs_reference(cuda, golden, report, batched):
    """DDIMCFG-10 (s = 3). Every step is checked teacher-forced (from the reference's previous
    sample) against the 1e-4 bound, and free-running with tests/conftest.py check_free_running
    (tests/golden/drift.npz adagn_cfg10: the reference's fp32 and float64 runs)."""
    from tests.conftest import check_chaos_envelope, check_free_running
    dg = golden('drift')[0]
    drift = dg['adagn_cfg10_drift_sample']
    g, meta = golden('adagn')
    model, _ = _model(meta, 'tiny_updown')
    model = model.to(cuda)
    cfg = meta['cfg']
    d = DDIMCFG(guidance_scale=cfg['guidance_scale'], respace_type=cfg['respace_type'],
                respace_steps=cfg['respace_steps'], eta=cfg['eta'], device=cuda)
    d.batch_cfg = batched
    init = torch.from_numpy(g['cfg_init']).to(cuda)
    labels = torch.from_numpy(g['cfg_labels']).to(cuda)
    seq = d.respaced_seq.tolist()
    pairs = list(zip(reversed(seq), reversed([-1] + seq[:-1])))
    worst_step = 0.0
    for i, (t, tp) in enumerate(pairs):
        x = init if i == 0 else torch.from_numpy(g[f'cfg_step{i - 1}_sample']).to(cuda)
        out = _one_step(d, model, x, labels, t, tp, batched)
        err = float(np.abs(out['sample'].cpu().numpy() - g[f'cfg_step{i}_sample']).max())
        worst_step = max(worst_step, err)
        assert err <= TOL, (i, err)
    worst, worst64 = 0.0, 0.0
    for i, out in enumerate(d.sample_loop(model, init, model_kwargs=dict(y=labels))):
        e32, e64 = check_free_running(out['sample'].cpu().numpy(), g[f'cfg_step{i}_sample'],
                                      dg['adagn_cfg10_sample64'][i], drift, i)
        worst, worst64 = max(worst, e32), max(worst64, e64)
    tag = 'batched' if batched else 'two_calls'
    report(f'ddimcfg10_adagn_{tag}_free_running_maxabs_vs_reference_float64', worst64)
    check_chaos_envelope(golden, 'adagn_cfg10', worst64, report, f'ddimcfg10_adagn_{tag}')
    report(f'ddimcfg10_adagn_{tag}_single_step_maxabs_vs_reference', worst_step)
    report(f'ddimcfg10_adagn_{tag}_free_running_maxabs_vs_reference', worst)


def _one_step(d, model, x, labels, t, tp, batched):
    """One DDIMCFG step from x at (t, tp): cond + uncond forwards (one 2B call with null labels when
    batched, as the sampler does), then the fused CFG update."""
    B = x.shape[0]
    if batched:
        tb = torch.full((2 * B, ), t, dtype=torch.long, device=x.device)
        import dmhip
        with dmhip.null_label_scope():
            both = model(torch.cat([x, x]), tb, torch.cat([labels, torch.full_like(labels, -1)]))
        oc, ou = both[:B], both[B:]
    else:
        tb = torch.full((B, ), t, dtype=torch.long, device=x.device)
        oc, ou = model(x, tb, labels), model(x, tb, None)
    return d._step(oc, x, t, tp, model_output_uncond=ou, guidance_scale=d.guidance_scale)


@pytest.mark.gpu
def test_adagn_batch_invariance(cuda, golden):
    """Row b of a B=64 batch equals the same row run at B=2 (no cross-row reduction anywhere)."""
    g, meta = golden('adagn')
    model, _ = _model(meta, 'cfg_cifar10')
    model = model.to(cuda)
    gen = torch.Generator().manual_seed(3)
    x = torch.randn((64, 3, 32, 32), generator=gen).to(cuda)
    t = torch.randint(0, 1000, (64, ), generator=gen).to(cuda)
    y = torch.randint(-1, 10, (64, ), generator=gen).to(cuda)
    import dmhip
    with dmhip.null_label_scope():
        big = model(x, t, y)
        small = model(x[5:7].contiguous(), t[5:7].contiguous(), y[5:7].contiguous())
    assert torch.equal(big[5:7], small)


@pytest.mark.gpu
@pytest.mark.parametrize('batched', [True, False])
def test_ddpmcfg_learned_range_trajectory(cuda, golden, report, batched):
    """DDPMCFG-6 with var_type learned_range (reference diffusions/ddpm.py:319-351) on a learned-sigma
    UNetCategorialAdaGN (out_channels = 2C, cosine schedule), noise pinned per step: the CFG combine of
    the eps halves, the concat of the CONDITIONAL branch's variance channels (:344-345) and the
    learned-range variance (:240-246), through the batched 2B forward (null-label rows) and the
    two-call path (tests/golden/ddpmcfg.npz, make_golden_r2.py). Every step teacher-forced: sample and
    pred_eps <= 1e-4; free-running: tests/conftest.py check_free_running on the sample."""
    from diffusions import DDPMCFG
    from tests.conftest import check_free_running
    g, meta = golden('ddpmcfg')
    model = UNetCategorialAdaGN(**meta['adagn_learned_arch']).eval()
    assert init_synthetic_(model) == meta['adagn_learned_weights_sha256']
    model = model.to(cuda)
    c = meta['adagn']
    d = DDPMCFG(guidance_scale=c['guidance_scale'], beta_schedule=c['beta_schedule'], var_type=c['var_type'],
                respace_type=c['respace_type'], respace_steps=c['respace_steps'], device=cuda)
    d.batch_cfg = batched
    n = len(d.respaced_seq)
    from tests.golden.noise import StepNoise
    labels = torch.from_numpy(g['adagn_labels']).to(cuda)
    seq = d.respaced_seq.tolist()
    worst_step = 0.0
    for i, (t, tp) in enumerate(zip(reversed(seq), reversed([-1] + seq[:-1]))):
        x = torch.from_numpy(g['adagn_init'] if i == 0 else g[f'adagn_step{i - 1}_sample']).to(cuda)
        src = StepNoise(c['noise_seed'])
        src.k = i
        d.noise_fn = src
        out = _one_step(d, model, x, labels, t, tp, batched)
        for k in ('sample', 'pred_eps'):
            err = float(np.abs(out[k].cpu().numpy() - g[f'adagn_step{i}_{k}']).max())
            worst_step = max(worst_step, err)
            assert err <= TOL, (i, k, err)
    d.noise_fn = StepNoise(c['noise_seed'])
    worst = 0.0
    for i, out in enumerate(d.sample_loop(model, torch.from_numpy(g['adagn_init']).to(cuda),
                                          model_kwargs=dict(y=labels))):
        e32, _ = check_free_running(out['sample'].cpu().numpy(), g[f'adagn_step{i}_sample'], g['adagn_sample64'][i],
                                    g['adagn_drift_sample'], i)
        worst = max(worst, e32)
    assert i + 1 == n
    report(f'ddpmcfg6_learned_adagn_{"batched" if batched else "two_calls"}_single_step_maxabs_vs_reference',
           worst_step)
    report(f'ddpmcfg6_learned_adagn_{"batched" if batched else "two_calls"}_maxabs_vs_reference', worst)

