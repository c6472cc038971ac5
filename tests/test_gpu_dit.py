"""DiT (models/dit/model.py) on the MI355X path.

PARITY UNPINNED: the reference DiT needs timm (absent), so the expected
outputs (tests/golden/dit.npz) come from oracle/dit.py, a restatement of
model.py + timm 0.9.12 (tests/golden/make_dit_golden.py). Tolerance: fp32
max-abs <= 1e-4, as for the pinned paths.
"""
import ctypes

import numpy as np
import pytest
import torch

from diffusions import DDIMCFG
from models.dit.model import DiT, DiT_models
from utils.synthetic import init_synthetic_

TOL = 1e-4
NAMES = ['dit_tiny', 'dit_s2', 'dit_xl2']


def _model(meta, name):
    m = DiT(**meta['archs'][name]).eval()
    return m, init_synthetic_(m)


@pytest.mark.parametrize('name', NAMES)
def test_dit_state_dict_layout(golden, name):
    _, meta = golden('dit')
    m = DiT(**meta['archs'][name])
    assert [[k, list(v.shape)] for k, v in m.state_dict().items()] == meta[f'{name}_state_dict']
    n = ctypes.c_int()
    from dmhip._lib import load
    assert load().dm_dit_param_count(ctypes.byref(m._arch_struct()), ctypes.byref(n)) == 0
    assert n.value == len(m.state_dict())


def test_dit_models_table():
    assert set(DiT_models) == {f'DiT-{s}/{p}' for s in ('XL', 'L', 'B', 'S') for p in (2, 4, 8)}


@pytest.mark.gpu
@pytest.mark.parametrize('name', NAMES)
def test_dit_forward_vs_oracle(cuda, golden, report, name):
    g, meta = golden('dit')
    model, sha = _model(meta, name)
    assert sha == meta[f'{name}_weights_sha256']
    model = model.to(cuda)
    x = torch.from_numpy(g[f'{name}_x']).to(cuda)
    t = torch.from_numpy(g[f'{name}_t']).to(cuda)
    y = torch.from_numpy(g[f'{name}_labels']).to(cuda)
    out_y = model(x, t, y).cpu()
    out_n = model(x, t, None).cpu()
    e_y = (out_y - torch.from_numpy(g[f'{name}_out_y'])).abs().max().item()
    e_n = (out_n - torch.from_numpy(g[f'{name}_out_null'])).abs().max().item()
    report(f'dit_forward_{name}_y_maxabs_vs_oracle', e_y)
    report(f'dit_forward_{name}_null_maxabs_vs_oracle', e_n)
    assert e_y <= TOL and e_n <= TOL, (e_y, e_n)
    # inside the CFG samplers' null-label scope y[b] = -1 selects the null class row, the same as
    # y=None; outside it a negative label is an IndexError (nn.Embedding upstream)
    import dmhip
    with dmhip.null_label_scope():
        neg = model(x, t, torch.full_like(y, -1)).cpu()
    assert torch.equal(neg, out_n)
    with pytest.raises(IndexError):
        model(x, t, torch.full_like(y, -1))
    # the null class index itself is a valid label (model.py:241-242)
    nul = model(x, t, torch.full_like(y, meta['archs'][name]['num_classes'])).cpu()
    assert torch.equal(nul, out_n)
    del model
    torch.cuda.empty_cache()


@pytest.mark.gpu
@pytest.mark.parametrize('batched', [True, False])
def test_dit_ddimcfg_trajectory_vs_oracle(cuda, golden, report, batched):
    g, meta = golden('dit')
    model, _ = _model(meta, 'dit_tiny')
    model = model.to(cuda)
    cfg = meta['cfg5']
    d = DDIMCFG(guidance_scale=cfg['guidance_scale'], respace_type=cfg['respace_type'],
                respace_steps=cfg['respace_steps'], eta=cfg['eta'], device=cuda)
    d.batch_cfg = batched
    labels = torch.from_numpy(g['cfg5_labels']).to(cuda)
    worst = 0.0
    for i, out in enumerate(d.sample_loop(model, torch.from_numpy(g['cfg5_init']).to(cuda),
                                          model_kwargs=dict(y=labels))):
        err = float(np.abs(out['sample'].cpu().numpy() - g[f'cfg5_step{i}_sample']).max())
        worst = max(worst, err)
        assert err <= TOL, (i, err)
    report(f'dit_ddimcfg5_{"batched" if batched else "two_calls"}_maxabs_vs_oracle', worst)


@pytest.mark.gpu
def test_dit_forward_with_cfg(cuda, golden):
    _, meta = golden('dit')
    model, _ = _model(meta, 'dit_tiny')
    model = model.to(cuda)
    gen = torch.Generator().manual_seed(5)
    x = torch.randn((4, 4, 8, 8), generator=gen).to(cuda)
    t = torch.full((4, ), 500, dtype=torch.long, device=cuda)
    nc = meta['archs']['dit_tiny']['num_classes']
    y = torch.tensor([1, 2, nc, nc], device=cuda)   # null class for the second half, as reference callers pass it
    out = model.forward_with_cfg(x, t, y, 1.5)
    full = model(torch.cat([x[:2], x[:2]]), t, y)
    ce, ue = full[:2, :3], full[2:, :3]
    torch.testing.assert_close(out[:2, :3], ue + 1.5 * (ce - ue), rtol=0, atol=1e-6)
    assert torch.equal(out[:, 3:], full[:, 3:])


@pytest.mark.gpu
@pytest.mark.parametrize('math', ['fp16x2', 'fp32'])
def test_dit_math_vs_oracle(cuda, golden, report, math):
    """The token GEMMs in fp16x2 (default) and fp32 both meet the tolerance on DiT-XL/2 geometry."""
    import dmhip
    g, meta = golden('dit')
    model, _ = _model(meta, 'dit_xl2')
    model = model.to(cuda)
    h = model.native_handle(torch.device(cuda))
    assert dmhip.dit_math(h) == 'fp16x2'
    assert dmhip.dit_math(h, math) == math
    x, t, y = (torch.from_numpy(g[f'dit_xl2_{k}']).to(cuda) for k in ('x', 't', 'labels'))
    err = (model(x, t, y).cpu() - torch.from_numpy(g['dit_xl2_out_y'])).abs().max().item()
    report(f'dit_forward_dit_xl2_{math}_maxabs_vs_oracle', err)
    assert err <= TOL, err
    assert dmhip.dit_math(h) == math


@pytest.mark.gpu
def test_dit_range_fallback(cuda, golden):
    """fc1 weights x 1e5 push the GELU output (fc2's input, x 2^6) beyond fp16: the fp16x2 forward is
    re-run in fp32 and equals a forward forced to fp32; the model's arithmetic stays fp16x2 (not sticky)."""
    import dmhip
    g, meta = golden('dit')
    x, t, y = (torch.from_numpy(g[f'dit_tiny_{k}']).to(cuda) for k in ('x', 't', 'labels'))
    outs = {}
    for math in ('fp16x2', 'fp32'):
        model, _ = _model(meta, 'dit_tiny')
        with torch.no_grad():
            for k, v in model.state_dict(keep_vars=True).items():
                if k.endswith('mlp.fc1.weight'):
                    v.mul_(1e5)
        model = model.to(cuda)
        h = model.native_handle(torch.device(cuda))
        dmhip.dit_math(h, math)
        outs[math] = model(x, t, y).cpu()
        assert dmhip.dit_math(h) == math
        assert dmhip.range_stats(h, abi='dm_dit') == ((1, 'fp16x2') if math == 'fp16x2' else (0, 'fp32'))
    assert torch.equal(outs['fp16x2'], outs['fp32'])
