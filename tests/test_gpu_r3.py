"""Round-3 GPU tests: the closed-form sampler conversions, the plan cache and the shared workspace, the
deferred range check across a re-pack, DiT-XL/2 at its benchmark batch, and per-step accuracy against
float64 for each arithmetic.

Fixtures: tests/golden/convert.npz and stepacc.npz (the reference itself, make_golden_r3.py),
dit.npz / dit_r3.npz (oracle/dit.py: DiT parity UNPINNED, timm absent).
"""
import numpy as np
import pytest
import torch

import dmhip
from diffusions import DDIM, DDIMCFG, DDPM
from tests.test_gpu_parity import TOL, _model
from utils.synthetic import init_synthetic_

pytestmark = pytest.mark.gpu


# ------------------------------------------------------------------ conversions (ddpm.py:102-172)
@pytest.mark.parametrize('case', ['linear1000', 'cosine1000'])
def test_conversions_vs_reference(cuda, golden, case):
    """pred_x0_from_eps / pred_eps_from_x0 / pred_x0_from_v / pred_eps_from_v / get_v / diffuse on the engine
    (dm_lincomb): bit-identical to the oracle's torch CPU expressions on this host, within a few ulp of the
    reference outputs generated on the build container's CPU (host-dependent 0-dim pow rounding: a 1-ulp
    coefficient difference times sqrt(1/ac) ~ 160 at t = 999, or divided by sqrt(1/ac - 1) ~ 0.01 at t = 0, is
    within 1e-6 of the output's scale)."""
    from oracle import diffusion as od
    g, meta = golden('convert')
    c = meta['cases'][case]
    d = DDPM(total_steps=c['total_steps'], beta_schedule=c['beta_schedule'], device=cuda)
    ac = od.alphas_cumprod(od.beta_schedule(c['total_steps'], c['beta_schedule']))
    x0, eps, xt = (torch.from_numpy(g[f'{case}_{k}']) for k in ('x0', 'eps', 'xt'))
    tvec = torch.from_numpy(g[f'{case}_tvec'])
    X0, EPS, XT = x0.to(cuda), eps.to(cuda), xt.to(cuda)

    def check(got, ref, gold):
        got = got.cpu().numpy()
        assert np.array_equal(got, ref.numpy()), np.abs(got - ref.numpy()).max()
        assert np.abs(got - gold).max() <= 1e-6 * np.abs(gold).max() + 1e-7, np.abs(got - gold).max()
    check(d.diffuse(X0, tvec.to(cuda), EPS), od.diffuse(ac, x0, tvec, eps), g[f'{case}_diffuse'])
    check(d.get_v(X0, EPS, tvec.to(cuda)), od.get_v(ac, x0, eps, tvec), g[f'{case}_get_v'])
    for t in c['ts']:
        check(d.pred_x0_from_eps(XT, t, EPS), od.pred_x0_from_eps(ac, xt, t, eps), g[f'{case}_t{t}_x0_from_eps'])
        check(d.pred_eps_from_x0(XT, t, X0), od.pred_eps_from_x0(ac, xt, t, x0), g[f'{case}_t{t}_eps_from_x0'])
        check(d.pred_x0_from_v(XT, t, EPS), od.pred_x0_from_v(ac, xt, t, eps), g[f'{case}_t{t}_x0_from_v'])
        check(d.pred_eps_from_v(XT, t, EPS), od.pred_eps_from_v(ac, xt, t, eps), g[f'{case}_t{t}_eps_from_v'])
    # an int timestep for diffuse (0-dim coefficients, as the reference's 0-dim indexing gives)
    got = d.diffuse(X0, 500, EPS).cpu().numpy()
    assert np.array_equal(got, od.diffuse(ac, x0, torch.tensor(500), eps).numpy())
    with pytest.raises(ValueError):
        d.diffuse(X0, torch.tensor([1, 2], device=cuda), EPS)   # one timestep per image


# ------------------------------------------------------------------ plan cache / shared workspace
def test_plan_cache_alternating_shapes(cuda, golden):
    """Alternating batch sizes reuse their cached plans (no rebuild after the first forward of each shape;
    reference sample_cfg.py:169-171 folds, batched vs two-call CFG), and every result equals a fresh
    model's forward at that shape bit for bit; a 4th shape evicts the least recently used plan."""
    _, meta = golden('forward')
    model, _ = _model(meta, 'tiny', cuda)
    h = model.native_handle(torch.device(cuda))
    gen = torch.Generator().manual_seed(3)
    xs = {B: torch.randn((B, 3, 16, 16), generator=gen).to(cuda) for B in (2, 3, 4, 5)}
    ts = {B: torch.randint(0, 1000, (B, ), generator=gen).to(cuda) for B in (2, 3, 4, 5)}
    first = {}
    for B in (2, 3, 4):
        first[B] = model(xs[B], ts[B])
    builds, cached = dmhip.plan_stats(h)
    assert (builds, cached) == (3, 3)
    for B in (2, 4, 3, 2, 3, 4):
        assert torch.equal(model(xs[B], ts[B]), first[B]), B
    assert dmhip.plan_stats(h) == (3, 3)
    model(xs[5], ts[5])   # evicts B = 2 (least recently used: 3 and 4 ran after it)
    assert dmhip.plan_stats(h) == (4, 3)
    assert torch.equal(model(xs[4], ts[4]), first[4])
    assert dmhip.plan_stats(h) == (4, 3)
    assert torch.equal(model(xs[2], ts[2]), first[2])
    assert dmhip.plan_stats(h) == (5, 3)
    fresh, _ = _model(meta, 'tiny', cuda)
    for B in (2, 3, 4):
        assert torch.equal(fresh(xs[B], ts[B]), first[B])


def test_combined_shared_workspace(cuda, golden):
    """UNetCombined's two networks run over ONE plan scratch slab (dm_unet_share_workspace): interleaved
    cond / uncond forwards equal those of two separate networks with the same weights bit for bit, and the
    two handles report the same (single) workspace."""
    from models.adm.unet import UNetModel
    from models.adm.unet_combined import UNetCombined
    _, meta = golden('adm')
    arch = meta['archs']['adm_tiny']
    comb = UNetCombined(**arch).eval()
    init_synthetic_(comb)
    sep_c = UNetModel(**arch).eval()
    sep_u = UNetModel(**dict(arch, num_classes=None)).eval()
    sep_c.load_state_dict(comb.unet_cond.state_dict())
    sep_u.load_state_dict(comb.unet_uncond.state_dict())
    comb, sep_c, sep_u = comb.to(cuda), sep_c.to(cuda), sep_u.to(cuda)
    gen = torch.Generator().manual_seed(8)
    y = torch.tensor([2, 3], device=cuda)
    for i in range(3):
        x = torch.randn((2, 3, 16, 16), generator=gen).to(cuda)
        t = torch.full((2, ), 900 - 300 * i, dtype=torch.long, device=cuda)
        assert torch.equal(comb(x, t, y), sep_c(x, t, y))
        assert torch.equal(comb(x, t, None), sep_u(x, t, None))
        x3 = torch.randn((3, 3, 16, 16), generator=gen).to(cuda)   # a second shape on the shared slab
        t3 = torch.full((3, ), 500, dtype=torch.long, device=cuda)
        assert torch.equal(comb(x3, t3, None), sep_u(x3, t3, None))
    import ctypes
    ws = []
    for net in (comb.unet_cond, comb.unet_uncond):
        w, s = ctypes.c_int64(), ctypes.c_int64()
        dmhip.load().dm_unet_memory(net.native_handle(torch.device(cuda)), ctypes.byref(w), ctypes.byref(s))
        ws.append(s.value)
    assert ws[0] == ws[1] > 0


# ------------------------------------------------------------------ deferred range check
def test_deferred_range_repack_mid_loop(cuda, golden):
    """A model re-packed inside DDPM.sample (a parameter's version bumped mid-loop) has its old handle
    polled before it is freed: the overflow it flagged is not lost, the loop re-runs, and sample() equals a
    model forced to bf16x3 bit for bit (no use of the freed handle)."""
    _, meta = golden('forward')
    outs = {}
    for case in ('repack', 'bf16x3'):
        model, _ = _model(meta, 'tiny', cuda)
        with torch.no_grad():
            model.first_conv.weight.mul_(1e5)   # activations beyond the fp16 range
        if case == 'bf16x3':
            dmhip.unet_conv_math(model.native_handle(torch.device(cuda)), 'bf16x3')
        calls = [0]

        def net(x, t, **kw):
            calls[0] += 1
            if case == 'repack' and calls[0] == 2:
                with torch.no_grad():
                    model.first_conv.bias.mul_(1.0)   # bumps _version: the next forward re-packs
            return model(x, t, **kw)
        d = DDIM(respace_type='uniform', respace_steps=4, eta=0.7, device=cuda)
        torch.manual_seed(9)
        init = torch.randn((2, 3, 16, 16), device=cuda)
        outs[case] = d.sample(net, init, tqdm_kwargs=dict(disable=True)).cpu()
        if case == 'repack':
            assert calls[0] == 8   # the loop ran twice
    assert torch.isfinite(outs['bf16x3']).all()
    assert torch.equal(outs['repack'], outs['bf16x3'])


def test_dit_deferred_range_fallback(cuda):
    """DiT-S/2 on 32x32 latents (T = 256, 2B * T = 8192 tokens: the pre-split linear_k32 path and the fc1
    pre-split epilogue run): fc1 weights x 1e5 overflow fp16 inside DDIMCFG.sample (eta > 0, deferred range
    check); the loop re-runs in fp32 from the same RNG state and equals a model forced to fp32."""
    from models.dit.model import DiT
    outs = {}
    for math in ('fp16x2', 'fp32'):
        m = DiT(input_size=32, patch_size=2, in_channels=4, hidden_size=384, depth=2, num_heads=6,
                num_classes=1000, learn_sigma=True).eval()
        init_synthetic_(m)
        with torch.no_grad():
            for k, v in m.state_dict(keep_vars=True).items():
                if k.endswith('mlp.fc1.weight'):
                    v.mul_(1e5)
        m = m.to(cuda)
        dmhip.dit_math(m.native_handle(torch.device(cuda)), math)
        d = DDIMCFG(guidance_scale=4.0, respace_type='uniform', respace_steps=3, eta=0.5, clip_denoised=False,
                    device=cuda)
        torch.manual_seed(11)
        init = torch.randn((16, 4, 32, 32), device=cuda)
        y = torch.arange(16, device=cuda)
        outs[math] = d.sample(m, init, model_kwargs=dict(y=y), tqdm_kwargs=dict(disable=True)).cpu()
        h = m.native_handle(torch.device(cuda))
        assert dmhip.dit_math(h) == math
        assert dmhip.range_stats(h, abi='dm_dit') == ((1, 'fp16x2') if math == 'fp16x2' else (0, 'fp32'))
    assert torch.isfinite(outs['fp32']).all()
    assert torch.equal(outs['fp16x2'], outs['fp32'])


# ------------------------------------------------------------------ DiT-XL/2 at the C5 batch
def _xl2(cuda, golden):
    from models.dit.model import DiT
    _, meta = golden('dit')
    m = DiT(**meta['archs']['dit_xl2']).eval()
    assert init_synthetic_(m) == meta['dit_xl2_weights_sha256']
    return m.to(cuda), meta


@pytest.mark.parametrize('sk', ['1', '0'])
def test_dit_xl2_cfg_batch64(cuda, golden, report, monkeypatch, sk):
    """BASELINE config C5's forward: DiT-XL/2, 32 images per GPU as one CFG batch of 2B = 64 rows (rows
    32..63 the null class, y = -1 inside the samplers' null-label scope). Row 0 / row 32 are the pinned
    dit_xl2 input with its label / the null class: within 1e-4 of oracle/dit.py; rows 0, 31, 32 and 63 against
    B = 1 / B = 2 forwards, so the B = 1 oracle parity extends to the benchmark batch: bit for bit with every tile
    over the whole K (DM_LIN_SK=0); with linear_k32's split-K tail (the default) a tile's sum is re-associated
    when it falls in a launch's last partial round -- which tiles do depends on the batch -- so within 2e-6 of
    the output's max (fp32 re-association; measured ~5e-7)."""
    monkeypatch.setenv('DM_LIN_SK', sk)
    g, _ = golden('dit')
    model, meta = _xl2(cuda, golden)
    gen = torch.Generator().manual_seed(64)
    B = 32
    x = torch.randn((B, 4, 32, 32), generator=gen)
    x[0] = torch.from_numpy(g['dit_xl2_x'][0])
    t = torch.randint(0, 1000, (B, ), generator=gen)
    t[0] = int(g['dit_xl2_t'][0])
    y = torch.randint(0, 1000, (B, ), generator=gen)
    y[0] = int(g['dit_xl2_labels'][0])
    x2, t2 = torch.cat([x, x]).to(cuda), torch.cat([t, t]).to(cuda)
    y2 = torch.cat([y, torch.full_like(y, -1)]).to(cuda)
    with dmhip.null_label_scope():
        big = model(x2, t2, y2)
        e_c = (big[0].cpu() - torch.from_numpy(g['dit_xl2_out_y'][0])).abs().max().item()
        e_u = (big[B].cpu() - torch.from_numpy(g['dit_xl2_out_null'][0])).abs().max().item()
        report('dit_xl2_2B64_row0_cond_maxabs_vs_oracle', e_c)
        report('dit_xl2_2B64_row32_null_maxabs_vs_oracle', e_u)
        assert e_c <= TOL and e_u <= TOL, (e_c, e_u)
        scale = big.abs().max().item()
        worst = 0.0
        for r in (0, 31, 32, 63):
            one = model(x2[r:r + 1].contiguous(), t2[r:r + 1].contiguous(), y2[r:r + 1].contiguous())
            if sk == '0':
                assert torch.equal(big[r:r + 1], one), r
            worst = max(worst, (big[r:r + 1] - one).abs().max().item() / scale)
        two = model(x2[[0, 63]].contiguous(), t2[[0, 63]].contiguous(), y2[[0, 63]].contiguous())
        if sk == '0':
            assert torch.equal(two, big[[0, 63]])
        worst = max(worst, (two - big[[0, 63]]).abs().max().item() / scale)
        report(f'dit_xl2_2B64_rows_vs_B1_rel_sk{sk}', worst)
        assert worst <= 2e-6, worst
    assert torch.isfinite(big).all()
    del model, big
    torch.cuda.empty_cache()


def test_dit_xl2_ddimcfg3_trajectory(cuda, golden, report):
    """DiT-XL/2 DDIMCFG-3 (s = 4, clip_denoised false as the DiT-XL/2 YAML sets, batched 2B forward) vs
    oracle/dit.py (tests/golden/dit_r3.npz; parity unpinned). Unclipped, x0 = sqrt(1/ac_t) x - ... carries
    the model's rounding times sqrt(1/ac_999) ~ 157 times the CFG gain 2s - 1 = 7 into the sample, so the
    oracle's own fp32 run sits ~1e-4 from its float64 run after one step: the bound is check_free_running's
    (tests/conftest.py) against both runs."""
    from tests.conftest import check_free_running
    g, meta = golden('dit_r3')
    model, _ = _xl2(cuda, golden)
    c = meta['xl2_cfg3']
    d = DDIMCFG(guidance_scale=c['guidance_scale'], respace_type=c['respace_type'], respace_steps=c['respace_steps'],
                eta=c['eta'], clip_denoised=c['clip_denoised'], device=cuda)
    labels = torch.from_numpy(g['xl2_cfg3_labels']).to(cuda)
    worst, worst64 = 0.0, 0.0
    for i, out in enumerate(d.sample_loop(model, torch.from_numpy(g['xl2_cfg3_init']).to(cuda),
                                          model_kwargs=dict(y=labels), tqdm_kwargs=dict(disable=True))):
        e32, e64 = check_free_running(out['sample'].cpu().numpy(), g[f'xl2_cfg3_step{i}_sample'],
                                      g['xl2_cfg3_sample64'][i], g['xl2_cfg3_drift_sample'], i)
        worst, worst64 = max(worst, e32), max(worst64, e64)
    report('dit_xl2_ddimcfg3_maxabs_vs_oracle', worst)
    report('dit_xl2_ddimcfg3_maxabs_vs_oracle_float64', worst64)
    report('dit_xl2_ddimcfg3_oracle_fp32_vs_fp64_drift', float(g['xl2_cfg3_drift_sample'].max()))
    del model
    torch.cuda.empty_cache()


# ------------------------------------------------------------------ per-step accuracy vs float64
def _stepacc_model(golden, name, cuda):
    from models.adm.unet_combined import UNetCombined
    from models.unet import UNet
    from models.unet_categorial_adagn import UNetCategorialAdaGN
    if name == 'cfg6':
        m = UNetCombined(**golden('adm')[1]['archs']['adm_tiny']).eval()
        nets = lambda mm: [mm.unet_cond, mm.unet_uncond]   # noqa: E731
    elif name == 'adagn_cfg10':
        m = UNetCategorialAdaGN(**golden('adagn')[1]['archs']['tiny_updown']).eval()
        nets = lambda mm: [mm]   # noqa: E731
    else:
        arch = golden('forward')[1]['archs']['tiny' if name == 'invrec' else 'cifar10']
        m = UNet(**arch).eval()
        nets = lambda mm: [mm]   # noqa: E731
    sha = init_synthetic_(m)
    return m.to(cuda), nets, sha


def _engine_step(name, model, meta, x, kind, t, tn, cuda):
    B = x.shape[0]
    tb = torch.full((B, ), t, dtype=torch.long, device=cuda)
    if name == 'cfg6':
        d = DDIMCFG(guidance_scale=2.5, respace_type='uniform', respace_steps=6, eta=0.0, device=cuda)
        y = torch.tensor([2, 3], device=cuda)
        return d._step(model(x, tb, y), x, t, tn, model_output_uncond=model(x, tb, None), guidance_scale=2.5)
    if name == 'adagn_cfg10':
        d = DDIMCFG(guidance_scale=3.0, respace_type='uniform', respace_steps=10, eta=0.0, device=cuda)
        y = torch.tensor(meta['adagn_cfg10_labels'], device=cuda)
        return d._step(model(x, tb, y), x, t, tn, model_output_uncond=model(x, tb, None), guidance_scale=3.0)
    d = DDIM(respace_type='uniform', respace_steps=5 if name == 'invrec' else 50, eta=0.0, device=cuda)
    if kind == 'inv':
        return d.denoise_inversion(model(x, tb), x, t, tn)
    return d.denoise(model(x, tb), x, t, tn)


@pytest.mark.parametrize('name', ['cfg6', 'adagn_cfg10', 'invrec', 'ddim50'])
def test_step_accuracy_vs_float64(cuda, golden, report, name):
    """Per step, from the same input (the reference's float64 trajectory state rounded to float32): the
    engine's distance to the float64 step against the fp32 reference's, for each conv arithmetic
    (tests/golden/stepacc.npz). This is the accuracy comparison the free-running trajectories cannot make
    (their end points scatter by chaos: DESIGN.md §5). Recorded per math; asserted: every step within 1e-4
    of the float64 step, and the default arithmetic's rms error at most 2x the fp32 reference's."""
    g, meta = golden('stepacc')
    info = meta[name]
    steps = info['steps']
    for math in ('fp16x2', 'bf16x3', 'fp32'):
        model, nets, _ = _stepacc_model(golden, name, cuda)
        for n in nets(model):
            dmhip.unet_conv_math(n.native_handle(torch.device(cuda)), math)
        e_max, e_rms = [], []
        for i, (kind, t, tn) in enumerate(steps):
            x = torch.from_numpy(g[f'{name}_x'][i]).to(cuda)
            got = _engine_step(name, model, meta, x, kind, t, tn, cuda)['sample'].cpu().double().numpy()
            diff = np.abs(got - g[f'{name}_ref64'][i])
            e_max.append(float(diff.max()))
            e_rms.append(float(np.sqrt((diff ** 2).mean())))
            assert e_max[-1] <= TOL, (math, i, e_max[-1])
        r_max, r_rms = np.array(info['ref32_max']), np.array(info['ref32_rms'])
        ratio_rms = float(np.max(np.array(e_rms) / r_rms))
        ratio_max = float(np.max(np.array(e_max) / r_max))
        report(f'stepacc_{name}_{math}_max_err_vs_float64', max(e_max))
        report(f'stepacc_{name}_{math}_worst_step_rms_ratio_to_fp32_reference', ratio_rms)
        report(f'stepacc_{name}_{math}_worst_step_max_ratio_to_fp32_reference', ratio_max)
        report(f'stepacc_{name}_{math}_mean_rms_ratio_to_fp32_reference', float(np.mean(np.array(e_rms) / r_rms)))
        if math == 'fp16x2':
            assert ratio_rms <= 2.0, (math, e_rms, list(r_rms))
        del model
    report(f'stepacc_{name}_fp32_reference_max_err_vs_float64', float(np.max(info['ref32_max'])))


def test_gpu_library_is_built_from_this_tree(cuda):
    """The library this GPU run loads was built from the sources in the snapshot (not a stale build)."""
    assert dmhip._lib.build_info().split()[0] == 'src=' + dmhip._lib.source_hash()


# ------------------------------------------------------------------ flash attention (attention.hip)
_FLASH_DIT_EXTRA = {   # head dims on the 16x16x32 P V tail: 80 (a whole 16-row tail), 72 at L = 64 (2-wave blocks)
    'dit_dh80': dict(input_size=16, patch_size=2, in_channels=4, hidden_size=320, depth=2, num_heads=4,
                     mlp_ratio=4.0, class_dropout_prob=0.1, num_classes=10, learn_sigma=True),
    'dit_dh72_l64': dict(input_size=16, patch_size=2, in_channels=4, hidden_size=576, depth=2, num_heads=8,
                         mlp_ratio=4.0, class_dropout_prob=0.1, num_classes=10, learn_sigma=True),
}


@pytest.mark.parametrize('case', ['adm_tiny', 'dit_s2', 'dit_xl2', 'adm256', 'adagn', 'dit_dh80', 'dit_dh72_l64'])
def test_flash_attention_vs_unfused(cuda, golden, report, monkeypatch, case):
    """attn_flash_kernel (online softmax, S never in HBM) against the unfused S GEMM -> softmax_rows -> PV
    GEMM path it replaces, which stays as the test oracle: ADM's 8^2 blocks (adm_tiny: L = 64, heads of 32,
    zero-padded to a 64-deep contraction), DiT-S/2 at 16^2 latents (L = 64, heads of 64), DiT-XL/2 (L = 256,
    16 heads of 72: an 80-deep contraction, O^T rows 64 .. 71 on the 16x16x32 tail; also 72 at L = 64 on 2-wave
    blocks and 80 with a whole 16-row tail), the guided-diffusion 256^2 UNet (L = 1024 at
    32^2 and L = 64 at 8^2, heads of 64), CFG-CIFAR AdaGN (8^2 blocks, heads of 64). Forwards within 1e-5 of
    each other (the attention core alone differs by exp2 vs expf and the online rescaling, a few 1e-7
    relative)."""
    from models.adm.unet import UNetModel
    from models.dit.model import DiT
    from models.unet_categorial_adagn import UNetCategorialAdaGN
    outs = {}
    for mode in ('flash', 'unfused'):
        if mode == 'unfused':
            monkeypatch.setenv('DM_ATTN', 'unfused')
        gen = torch.Generator().manual_seed(21)
        if case == 'adagn':
            m = UNetCategorialAdaGN(**golden('adagn')[1]['archs']['cfg_cifar10']).eval()
            B = 2
            x = torch.randn((B, 3, 32, 32), generator=gen)
            y = torch.tensor([1, 3])
        elif case.startswith('adm'):
            arch = golden('adm')[1]['archs']['adm_tiny' if case == 'adm_tiny' else 'adm256_combined']
            m = UNetModel(**arch).eval()
            S, B = arch['image_size'], 2 if case == 'adm_tiny' else 1
            x = torch.randn((B, 3, S, S), generator=gen)
            y = torch.tensor([1, 3][:B])
        else:
            arch = _FLASH_DIT_EXTRA.get(case) or golden('dit')[1]['archs'][case]
            m = DiT(**arch).eval()
            S, B = arch['input_size'], 2
            x = torch.randn((B, 4, S, S), generator=gen)
            y = torch.tensor([5, 9])
        init_synthetic_(m)
        m = m.to(cuda)
        t = torch.tensor([999, 40][:B])
        outs[mode] = m(x.to(cuda), t.to(cuda), y.to(cuda)).cpu()
        labels = [op['label'] for op in dmhip.unet_profile_read(m.native_handle(torch.device(cuda)), m._abi)]
        assert any(lb.startswith('attn_flash_kernel') for lb in labels) == (mode == 'flash'), labels
        del m
        torch.cuda.empty_cache()
    err = (outs['flash'] - outs['unfused']).abs().max().item()
    report(f'flash_attention_{case}_maxabs_vs_unfused', err)
    assert torch.isfinite(outs['flash']).all()
    assert err <= 1e-5, err


# ------------------------------------------------------------------ small-map conv kernel (conv_k32.hip)
@pytest.mark.parametrize('arch', ['cifar10', 'adagn'])
def test_small_map_conv_vs_splitk(cuda, golden, report, monkeypatch, arch):
    """The 4 x 4 level's convs on conv_k32s_kernel (one launch, K split inside the block, GroupNorm statistics
    per image from its epilogue; DM_CONV_WINO=0) against the two-launch split-K path with its reduction
    (DM_CONV_K32S=0) and against the default since round 6, which puts the up path's 512-channel conv1s on the split-K
    Winograd kernel (conv_wino_kernel<4, ..> + conv_splitk_reduce, GroupNorm statistics from the reduction; its in-kernel
    GroupNorm finalize over a split's channels): whole forwards within 1e-5 (the partial sums
    group differently), and each kernel is the one the plan runs."""
    from models.unet_categorial_adagn import UNetCategorialAdaGN
    outs = {}
    for mode in ('small', 'splitk', 'wino'):
        monkeypatch.setenv('DM_CONV_WINO', '1' if mode == 'wino' else '0')
        monkeypatch.setenv('DM_CONV_K32S', '0' if mode == 'splitk' else '1')
        if arch == 'cifar10':
            m, _ = _model(golden('forward')[1], 'cifar10', cuda)
        else:
            m = UNetCategorialAdaGN(**golden('adagn')[1]['archs']['cfg_cifar10']).eval()
            init_synthetic_(m)
            m = m.to(cuda)
        g = torch.Generator().manual_seed(6)
        x = torch.randn((8, 3, 32, 32), generator=g).to(cuda)
        t = torch.tensor([999, 800, 600, 400, 200, 100, 10, 0], device=cuda)
        outs[mode] = (m(x, t) if arch == 'cifar10' else m(x, t, torch.arange(8, device=cuda) % 10)).cpu()
        h = m.native_handle(torch.device(cuda))
        dmhip.unet_profile_enable(h, 1)
        dmhip.unet_profile_enable(h, 0)
        labels = [op['label'] for op in dmhip.unet_profile_read(h)]
        assert dmhip.range_stats(h)[0] == 0  # (a range fallback would re-run the forward in bf16x3)
        k32s = any(lb.startswith('conv_k32s_kernel') for lb in labels)
        wino4 = any(lb.startswith('conv_wino_kernel<4,') for lb in labels)
        # (the Winograd mode keeps conv_k32s for the convs with < 12 K steps per split: unet_exec.hip maybe_split)
        assert (k32s, wino4) == {'small': (True, False), 'splitk': (False, False), 'wino': (k32s, True)}[mode], labels
        del m
    for other in ('splitk', 'wino'):
        err = (outs['small'] - outs[other]).abs().max().item()
        report(f'small_map_conv_{arch}_maxabs_vs_{other}', err)
        assert torch.isfinite(outs[other]).all()
        assert err <= 1e-5, (other, err)


# ------------------------------------------------------------------ first conv row split
@pytest.mark.parametrize('dim,size', [(320, 32), (192, 16), (96, 8)])
def test_first_conv_wide_channels(cuda, dim, size):
    """The first conv's block covers R = 64 / W rows; with dim / 2 channel pairs not dividing 256 its pixel
    groups split those rows unevenly (dim 320 at 32^2: one group of 160 lanes, 96 leftover threads; dim 192 at
    16^2: two groups, 64 leftover). Every row is computed once and no thread writes past its block: a UNet
    with that first layer matches the oracle (reference models/unet.py:72, 121-152)."""
    from models.unet import UNet
    from oracle.unet import OracleUNet
    arch = dict(dim=dim, dim_mults=[1], use_attn=[False], num_res_blocks=1, n_heads=1, dropout=0.0)
    m = UNet(**arch).eval()
    init_synthetic_(m)
    oracle = OracleUNet(m.state_dict(), **arch)
    m = m.to(cuda)
    g = torch.Generator().manual_seed(12)
    x = torch.randn((2, 3, size, size), generator=g)
    t = torch.tensor([5, 640])
    # the output buffer is followed by other plan scratch: a write past the last block would land there
    out = m(x.to(cuda), t.to(cuda)).cpu()
    ref = oracle(x, t)
    err = (out - ref).abs().max().item()
    assert err <= TOL, err
    assert torch.equal(m(x.to(cuda), t.to(cuda)).cpu(), out)


def test_combined_shared_workspace_two_streams(cuda, golden):
    """The cond and uncond networks of a UNetCombined share one scratch slab; forwards issued on two different
    streams without any host sync are ordered by the engine (a forward on a new stream waits for the previous
    forward over the slab) and equal separate networks' forwards bit for bit."""
    from models.adm.unet import UNetModel
    from models.adm.unet_combined import UNetCombined
    _, meta = golden('adm')
    arch = meta['archs']['adm_tiny']
    comb = UNetCombined(**arch).eval()
    init_synthetic_(comb)
    sep_c = UNetModel(**arch).eval()
    sep_u = UNetModel(**dict(arch, num_classes=None)).eval()
    sep_c.load_state_dict(comb.unet_cond.state_dict())
    sep_u.load_state_dict(comb.unet_uncond.state_dict())
    comb, sep_c, sep_u = comb.to(cuda), sep_c.to(cuda), sep_u.to(cuda)
    gen = torch.Generator().manual_seed(21)
    y = torch.tensor([1, 4], device=cuda)
    xs = [torch.randn((2, 3, 16, 16), generator=gen).to(cuda) for _ in range(4)]
    t = torch.tensor([700, 90], device=cuda)
    comb(xs[0], t, y), comb(xs[0], t, None)   # plans
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = []
    for i, x in enumerate(xs):
        with torch.cuda.stream(s1 if i % 2 == 0 else s2):
            outs.append((comb(x, t, y), comb(x, t, None)))
    torch.cuda.synchronize()
    for x, (oc, ou) in zip(xs, outs):
        assert torch.equal(oc, sep_c(x, t, y))
        assert torch.equal(ou, sep_u(x, t, None))
