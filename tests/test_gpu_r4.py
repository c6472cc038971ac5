"""Round-4 GPU tests.

* the folded single-head attention block (attn_block.hip, variants 3 and 4) against the unfolded path (q / k / v /
  proj as the reference computes them, DM_ATTN=0) and the reference fixtures (models/modules.py:77-102,
  models/unet.py:121-152);
* DiT-XL/2 per-step accuracy vs float64 and the 2^-20 chaos envelope (models/dit/model.py:234-252; parity
  unpinned, timm absent);
* the K32 convs added this round: small-map 8 waves, stride-2 tiles (models/modules.py:70-72), 2-D tiles of
  wide maps incl. the sub-pixel upsample (models/adm/unet.py:162-275), each against the path it replaces.
"""
import numpy as np
import pytest
import torch

import dmhip
from tests.test_gpu_parity import TOL, _model
from utils.synthetic import init_synthetic_

pytestmark = pytest.mark.gpu


def _profile_labels(model, cuda):
    h = model.native_handle(torch.device(cuda))
    dmhip.unet_profile_enable(h, 1)
    return h


def _labels(h):
    return [op['label'] for op in dmhip.unet_profile_read(h)]


@pytest.mark.parametrize('B,variant', [(2, '3'), (7, '3'), (5, '4'), (3, '4')])
def test_folded_attention_vs_unfolded(cuda, golden, monkeypatch, B, variant):
    """The CIFAR-10 UNet's five 16 x 16 attention blocks run folded (variant 4, the default, and 3:
    attn_block4_kernel / attn_block3_kernel alone, no q / k / v planes): whole forwards within 1e-5 of the
    unfolded path (same weights, same inputs), and the folded kernels are the ones in the plan."""
    monkeypatch.setenv('DM_ATTN', variant)
    kname = {'3': 'attn_block3_kernel', '4': 'attn_block4_kernel<8>'}[variant]
    _, meta = golden('forward')
    g = torch.Generator().manual_seed(31)
    x = torch.randn((B, 3, 32, 32), generator=g).to(cuda)
    t = torch.randint(0, 1000, (B, ), generator=g).to(cuda)
    folded, _ = _model(meta, 'cifar10', cuda)
    out_f = folded(x, t)
    h = folded.native_handle(torch.device(cuda))
    dmhip.unet_profile_enable(h, 1)
    folded(x, t)
    labels = _labels(h)
    dmhip.unet_profile_enable(h, 0)
    assert labels.count(kname) == 5, labels
    assert not any(lb.startswith('linear_k32_kernel') for lb in labels)
    assert not any(lb.startswith('attn_presplit_kernel') for lb in labels)
    monkeypatch.setenv('DM_ATTN', '0')
    unfolded, _ = _model(meta, 'cifar10', cuda)
    out_u = unfolded(x, t)
    err = (out_f - out_u).abs().max().item()
    assert err <= 1e-5, err
    assert torch.isfinite(out_f).all()


def test_folded_attention_vs_reference(cuda, golden, report):
    """Reference fixture (tests/golden/forward.npz, the reference UNet itself at B = 2): the folded forward
    within 1e-4 (north_star tolerance)."""
    arrays, meta = golden('forward')
    model, _ = _model(meta, 'cifar10', cuda)
    y = model(torch.from_numpy(arrays['cifar10_x']).to(cuda), torch.from_numpy(arrays['cifar10_t']).to(cuda))
    err = (y.cpu() - torch.from_numpy(arrays['cifar10_y'])).abs().max().item()
    report('forward_cifar10_folded_attention_maxabs_vs_reference', err)
    assert err <= TOL, err


@pytest.mark.parametrize('variant', ['3', '4'])
def test_folded_attention_batch_invariance(cuda, golden, monkeypatch, variant):
    """B = 256 (the benchmark batch) rows equal the B = 3 forward's rows bit for bit: every work-group is one
    (image, query half) and reads only its image."""
    monkeypatch.setenv('DM_ATTN', variant)
    _, meta = golden('forward')
    model, _ = _model(meta, 'cifar10', cuda)
    g = torch.Generator().manual_seed(32)
    x = torch.randn((256, 3, 32, 32), generator=g).to(cuda)
    t = torch.randint(0, 1000, (256, ), generator=g).to(cuda)
    big = model(x, t)
    idx = [0, 129, 255]
    small = model(x[idx].contiguous(), t[idx].contiguous())
    assert torch.equal(big[idx], small)


def test_folded_attention_8_waves_bit_identical(cuda, golden, monkeypatch):
    """Variant 4 (8 waves of 16 queries) runs variant 3's MFMA sequence per output element with the same staging
    layouts and scales: whole forwards equal bit for bit."""
    _, meta = golden('forward')
    g = torch.Generator().manual_seed(34)
    x = torch.randn((4, 3, 32, 32), generator=g).to(cuda)
    t = torch.randint(0, 1000, (4, ), generator=g).to(cuda)
    outs = {}
    for v in ('3', '4'):
        monkeypatch.setenv('DM_ATTN', v)
        model, _ = _model(meta, 'cifar10', cuda)
        outs[v] = model(x, t)
        del model
    assert torch.equal(outs['3'], outs['4'])


def test_attention_in_kernel_gn_finalize_bit_identical(cuda, golden, monkeypatch):
    """Variant 4 computes its GroupNorm affine from the chunk partials in the kernel (gn_finalize's expressions
    and summation order): whole forwards equal the separate gn_finalize launch's (DM_ATTN_GNFIN=1) bit for bit,
    with five gn_finalize launches fewer per forward."""
    _, meta = golden('forward')
    g = torch.Generator().manual_seed(35)
    x = torch.randn((3, 3, 32, 32), generator=g).to(cuda)
    t = torch.randint(0, 1000, (3, ), generator=g).to(cuda)
    outs, nfin = {}, {}
    for mode in ('kernel', 'launch'):
        if mode == 'launch':
            monkeypatch.setenv('DM_ATTN_GNFIN', '1')
        model, _ = _model(meta, 'cifar10', cuda)
        outs[mode] = model(x, t)
        h = _profile_labels(model, cuda)
        model(x, t)
        nfin[mode] = _labels(h).count('gn_finalize')
        dmhip.unet_profile_enable(h, 0)
        del model
    assert nfin['launch'] == nfin['kernel'] + 5, nfin
    assert torch.equal(outs['kernel'], outs['launch'])


# ------------------------------------------------------------------ DiT accuracy evidence
def _dit_xl2(cuda, golden):
    from models.dit.model import DiT
    _, meta = golden('dit')
    g, ameta = golden('dit_acc')
    m = DiT(**meta['archs']['dit_xl2']).eval()
    assert init_synthetic_(m) == ameta['dit_xl2_weights_sha256']
    return m.to(cuda), g, ameta


def test_dit_step_accuracy_vs_float64(cuda, golden, report):
    """DiT-XL/2 DDIMCFG-3 (s = 4, clip_denoised false: the C5 config), per step from the same input (the
    oracle's float64 trajectory state rounded to float32; tests/golden/dit_acc.npz, make_golden_r4.py): the
    engine's distance to the float64 step against the fp32 oracle's. Asserted: every step's rms error at most
    2x the fp32 oracle's (parity unpinned: oracle/dit.py restates the reference, timm absent)."""
    from diffusions import DDIMCFG
    model, g, meta = _dit_xl2(cuda, golden)
    s = meta['guidance_scale']
    d = DDIMCFG(guidance_scale=s, respace_type='uniform', respace_steps=meta['respace_steps'], eta=0.0,
                clip_denoised=meta['clip_denoised'], device=cuda)
    y = torch.tensor(meta['labels'], device=cuda)
    ratios, e_max = [], []
    for i, (t, tn) in enumerate(meta['steps']):
        x = torch.from_numpy(g['x'][i]).to(cuda)
        tb = torch.full((x.shape[0], ), t, dtype=torch.long, device=cuda)
        got = d._step(model(x, tb, y), x, t, tn, model_output_uncond=model(x, tb, None),
                      guidance_scale=s)['sample'].cpu().double().numpy()
        diff = np.abs(got - g['ref64'][i])
        rms = float(np.sqrt((diff ** 2).mean()))
        e_max.append(float(diff.max()))
        ratios.append(rms / meta['ref32_rms'][i])
    report('dit_xl2_stepacc_max_err_vs_float64', max(e_max))
    report('dit_xl2_stepacc_fp32_oracle_max_err_vs_float64', max(meta['ref32_max']))
    report('dit_xl2_stepacc_worst_step_rms_ratio_to_fp32_oracle', max(ratios))
    report('dit_xl2_stepacc_mean_rms_ratio_to_fp32_oracle', float(np.mean(ratios)))
    assert max(ratios) <= 2.0, ratios
    del model
    torch.cuda.empty_cache()


def test_dit_trajectory_chaos_envelope(cuda, golden, report):
    """The DiT-XL/2 DDIMCFG-3 free-running trajectory (batched 2B CFG forward, as the sampler runs it)
    against the oracle's float64 run: its worst distance must lie inside the envelope of the fp32 oracle's own
    runs with the model output perturbed by 2^-20 relative (8 seeds, the level at which the engine's forwards
    differ from the oracle's) -- the check_chaos_envelope criterion of the UNet CFG trajectories."""
    from diffusions import DDIMCFG
    model, g, meta = _dit_xl2(cuda, golden)
    d = DDIMCFG(guidance_scale=meta['guidance_scale'], respace_type='uniform', respace_steps=meta['respace_steps'],
                eta=0.0, clip_denoised=meta['clip_denoised'], device=cuda)
    y = torch.tensor(meta['labels'], device=cuda)
    worst = 0.0
    for i, out in enumerate(d.sample_loop(model, torch.from_numpy(g['init']).to(cuda), model_kwargs=dict(y=y),
                                          tqdm_kwargs=dict(disable=True))):
        worst = max(worst, float(np.abs(out['sample'].cpu().double().numpy() - g['traj64'][i]).max()))
    env20 = g['e64_p20'].max(axis=1)
    report('dit_xl2_free_running_maxabs_vs_oracle_float64', worst)
    report('dit_xl2_fp32_oracle_unperturbed_vs_float64', float(g['e64_p0'].max()))
    report('dit_xl2_chaos_envelope_2^-20_max', float(env20.max()))
    report('dit_xl2_chaos_envelope_2^-22_max', float(g['e64_p22'].max()))
    report('dit_xl2_perturbed_oracle_runs_further_than_engine', float(np.mean(env20 > worst)))
    assert worst <= max(TOL, float(env20.max())), (worst, list(env20))
    del model
    torch.cuda.empty_cache()


# ------------------------------------------------------------------ small-map conv, 8 waves (conv_k32.hip)
def test_small_map_conv_8_waves_bit_identical(cuda, golden, monkeypatch):
    """The 4x4-level convs (conv_k32s_kernel) with 8 waves (two per SIMD, 32 x 32 wave tiles) give the same bits
    as the 4-wave form (same K split, same MFMA sequence per output element): whole CIFAR forwards equal, and the
    8-wave kernel is the one in the plan."""
    _, meta = golden('forward')
    g = torch.Generator().manual_seed(33)
    x = torch.randn((5, 3, 32, 32), generator=g).to(cuda)
    t = torch.randint(0, 1000, (5, ), generator=g).to(cuda)
    outs, labels = {}, {}
    for w4 in ('0', '1'):
        monkeypatch.setenv('DM_K32S_W4', w4)
        model, _ = _model(meta, 'cifar10', cuda)
        outs[w4] = model(x, t)
        h = model.native_handle(torch.device(cuda))
        dmhip.unet_profile_enable(h, 1)
        model(x, t)
        labels[w4] = _labels(h)
        dmhip.unet_profile_enable(h, 0)
        del model
    assert any(lb.startswith('conv_k32s_kernel<') and lb.endswith(',8>') for lb in labels['0']), labels['0']
    assert torch.equal(outs['0'], outs['1'])


# ------------------------------------------------------------------ stride-2 downsample on K32 (conv_k32.hip S2)
S2_LABEL = 'conv_k32_kernel<64,128,32,32,false,false,false,512,392,2048,true>'


@pytest.mark.parametrize('B,Cin,Cout,H', [(2, 32, 64, 32), (3, 64, 128, 16), (2, 128, 256, 16), (1, 96, 160, 32),
                                          (3, 128, 128, 32)])
def test_stride2_k32_exact(cuda, B, Cin, Cout, H):
    """The stride-2 3x3 (models/modules.py:70-72) on the K32 tiles (tile 18: 64-pixel output tiles of whole
    rows, parity-split patch columns, 8 waves of 32 x 32, ragged Cout tails): bit-exact on integer operands."""
    from tests.test_gpu_ops import _ints, _nhwc, _pack, _run_conv
    import torch.nn.functional as F
    x = _ints((B, Cin, H, H), -2, 3, seed=44)
    w = _ints((Cout, Cin, 3, 3), -2, 3, seed=45)
    b = _ints((Cout, ), seed=46)
    ref = F.conv2d(x.double(), w.double(), b.double(), stride=2, padding=1).float()
    Ho = ref.shape[-1]
    y = _run_conv(cuda, _nhwc(x).to(cuda), _pack(w, cuda), Cout, Ho, Ho, 9, 2, 0, b.to(cuda), split='fp16x2', tile=18)
    assert torch.equal(y.cpu(), _nhwc(ref))


def test_stride2_k32_fp32_accuracy(cuda):
    """Random stride-2 conv on the K32 tiles: error vs fp64 within 2x the fp32 kernel's."""
    from tests.test_gpu_ops import _nhwc, _pack, _run_conv
    import torch.nn.functional as F
    g = torch.Generator().manual_seed(47)
    B, Cin, Cout, H = 8, 256, 256, 16
    x = torch.randn((B, Cin, H, H), generator=g) * 3
    w = torch.randn((Cout, Cin, 3, 3), generator=g) * (1.0 / (9 * Cin) ** 0.5)
    ref = _nhwc(F.conv2d(x.double(), w.double(), stride=2, padding=1))
    errs = []
    for split, tile in ((False, 0), ('fp16x2', 18)):
        y = _run_conv(cuda, _nhwc(x).to(cuda), _pack(w, cuda), Cout, H // 2, H // 2, 9, 2, split=split, tile=tile)
        errs.append((y.cpu().double() - ref).abs().max().item())
    assert errs[1] < 2.0 * errs[0] + 1e-7 * ref.abs().max().item(), errs


def test_downsample_k32_vs_patch3(cuda, golden, report, monkeypatch):
    """The CIFAR UNet's 32->16 and 16->8 Downsample convs on the K32 stride-2 tiles (with the consumer's
    GroupNorm statistics from their epilogue) against conv_patch3 MODE 4 + gn_partial (DM_CONV_K32S2=0): whole
    forwards within 1e-5, and the K32 kernel is the one in the plan."""
    _, meta = golden('forward')
    g = torch.Generator().manual_seed(48)
    x = torch.randn((6, 3, 32, 32), generator=g).to(cuda)
    t = torch.randint(0, 1000, (6, ), generator=g).to(cuda)
    outs = {}
    for mode in ('k32', 'patch3'):
        if mode == 'patch3':
            monkeypatch.setenv('DM_CONV_K32S2', '0')
        model, _ = _model(meta, 'cifar10', cuda)
        outs[mode] = model(x, t)
        h = _profile_labels(model, cuda)
        model(x, t)
        labels = _labels(h)
        dmhip.unet_profile_enable(h, 0)
        assert labels.count(S2_LABEL) == (2 if mode == 'k32' else 0), labels
        del model
    err = (outs['k32'] - outs['patch3']).abs().max().item()
    report('downsample_k32_maxabs_vs_patch3', err)
    assert torch.isfinite(outs['k32']).all()
    assert err <= 1e-5, err


# ------------------------------------------------------------------ 2-D tiles of wide maps (conv_k32.hip T2D)
@pytest.mark.parametrize('B,Cin,Cout,H,W', [(1, 32, 64, 4, 256), (2, 64, 96, 8, 64), (1, 64, 32, 12, 128),
                                            (3, 32, 128, 4, 96)])
def test_t2d_tiles_exact(cuda, B, Cin, Cout, H, W):
    """Wide maps (ADM 64^2 .. 256^2) on 2-D tiles (tile 19: 4 rows x 32 columns per 128-row tile, the GEMM rows
    enumerating pixels tile by tile): bias, integer operands bit-exact vs fp64."""
    from tests.test_gpu_ops import _ints, _nhwc, _pack, _run_conv
    import torch.nn.functional as F
    x = _ints((B, Cin, H, W), -2, 3, seed=110)
    w = _ints((Cout, Cin, 3, 3), -2, 3, seed=111)
    b = _ints((Cout, ), seed=112)
    ref = F.conv2d(x.double(), w.double(), b.double(), padding=1).float()
    y = _run_conv(cuda, _nhwc(x).to(cuda), _pack(w, cuda), Cout, H, W, 9, 1, 0, b.to(cuda), tile=19, split='fp16x2')
    assert torch.equal(y.cpu(), _nhwc(ref))


@pytest.mark.parametrize('B,Cin,Cout,H,W', [(1, 32, 64, 4, 64), (2, 64, 32, 8, 128)])
def test_t2d_tiles_subpixel_exact(cuda, B, Cin, Cout, H, W):
    """The sub-pixel upsample (nearest-2x + 3x3, models/modules.py:60-63) of a wide low-res map on 2-D tiles
    (tile 19: 4 x 32 low-res pixels per tile, 4 parity convs of 4 taps, rows scattered to 2 iy + py, 2 ix + px):
    integer operands bit-exact vs fp64."""
    from tests.test_gpu_ops import _ints, _nhwc, _pack_subpix, _run_conv
    import torch.nn.functional as F
    x = _ints((B, Cin, H, W), -2, 3, seed=120)
    w = _ints((Cout, Cin, 3, 3), -1, 2, seed=121)
    b = _ints((Cout, ), seed=122)
    ref = F.conv2d(F.interpolate(x, scale_factor=2, mode='nearest').double(), w.double(), b.double(),
                   padding=1).float()
    y = _run_conv(cuda, _nhwc(x).to(cuda), _pack_subpix(w, cuda), Cout, 2 * H, 2 * W, 9, 1, 2, b.to(cuda), tile=19,
                  split='fp16x2')
    assert torch.equal(y.cpu(), _nhwc(ref))


def test_t2d_tiles_shortcut_residual_rowvec(cuda):
    """2-D tiles with the ResBlock epilogue pieces: the 1x1 shortcut segment (its rows mapped through the tile
    order), per-image row vector, residual, output pitch."""
    from tests.test_gpu_ops import _ints, _nhwc, _pack, _run_conv
    import torch.nn.functional as F
    B, C1, C2, Cout, H, W = 2, 64, 32, 64, 8, 128
    h = _ints((B, C1, H, W), seed=113)
    x = _ints((B, C2, H, W), seed=114)
    w2 = _ints((Cout, C1, 3, 3), -2, 3, seed=115)
    ws = _ints((Cout, C2, 1, 1), seed=116)
    b = _ints((Cout, ), seed=117)
    rv = _ints((B, Cout), seed=118)
    res = _ints((B, Cout, H, W), seed=119)
    K = 9 * C1 + C2
    wp = torch.zeros((Cout, K), device=cuda)
    _pack(w2, cuda, K, 0, wp)
    _pack(ws, cuda, K, 9 * C1, wp)
    ref = (F.conv2d(h.double(), w2.double(), b.double(), padding=1) + rv.double()[:, :, None, None]
           + F.conv2d(x.double(), ws.double()) + res.double()).float()
    y = _run_conv(cuda, _nhwc(h).to(cuda), wp, Cout, H, W, 9, bias=b.to(cuda), rowvec=rv.to(cuda),
                  res=_nhwc(res).to(cuda), x2=_nhwc(x).to(cuda), Cin2=C2, y_pitch=72, tile=19, split='fp16x2')
    assert torch.equal(y[..., :Cout].cpu(), _nhwc(ref))
    assert torch.isnan(y[..., Cout:]).all()


def test_adm256_t2d_vs_row_segments(cuda, golden, report, monkeypatch):  # noqa: C901
    """The RePaint CelebA-HQ ADM-256 (reference fixture config, B = 1) with its 64^2 .. 256^2 convs on the 2-D
    tiles (their GroupNorm partials from the epilogue, chunks = 64 pixels of a tile) against the 128-pixel row
    segments (DM_CONV_K32T2=0): within 1e-5, and the 2-D kernel is in the plan."""
    from models.adm.unet import UNetModel
    g, meta = golden('adm')
    name = 'adm256_celebahq'
    x = torch.from_numpy(g[f'{name}_x']).to(cuda)
    t = torch.from_numpy(g[f'{name}_t']).to(cuda)
    y = torch.from_numpy(g[f'{name}_labels']).to(cuda) if f'{name}_labels' in g else None
    outs = {}
    for mode in ('t2d', 'rows'):
        if mode == 'rows':
            monkeypatch.setenv('DM_CONV_K32T2', '0')
        model = UNetModel(**meta['archs'][name]).eval()
        init_synthetic_(model)
        model = model.to(cuda)
        outs[mode] = model(x, t, y).cpu()
        h = model.native_handle(torch.device(cuda))
        dmhip.unet_profile_enable(h, 1)
        model(x, t, y)
        labels = _labels(h)
        dmhip.unet_profile_enable(h, 0)
        assert any(lb.startswith('conv_k32_kernel<128,128,64,64,') and lb.endswith(',2048,false,true>')
                   for lb in labels) == (mode == 't2d'), labels
        del model
        torch.cuda.empty_cache()
    err = (outs['t2d'] - outs['rows']).abs().max().item()
    report('adm256_t2d_maxabs_vs_row_segments', err)
    ref_err = (outs['t2d'] - torch.from_numpy(g[f'{name}_out'])).abs().max().item()
    report('adm256_t2d_maxabs_vs_reference', ref_err)
    assert err <= 1e-5, err
    assert ref_err <= TOL, ref_err


def test_k32_8x8_single_image_tiles_bit_identical(cuda, golden, monkeypatch):
    """The 8^2 convs on 64-row single-image tiles (4 waves of 32 x 64, two blocks per CU; the default) give the
    same bits as the 128 x 128 two-image tiles (DM_K32_8X=0; same K order per output element), GroupNorm partials
    included."""
    _, meta = golden('forward')
    g = torch.Generator().manual_seed(37)
    x = torch.randn((4, 3, 32, 32), generator=g).to(cuda)
    t = torch.randint(0, 1000, (4, ), generator=g).to(cuda)
    outs = {}
    for mode in ('base', '8x'):
        if mode == 'base':
            monkeypatch.setenv('DM_K32_8X', '0')
        else:
            monkeypatch.delenv('DM_K32_8X', raising=False)
        model, _ = _model(meta, 'cifar10', cuda)
        outs[mode] = model(x, t)
        del model
    assert torch.equal(outs['base'], outs['8x'])
