"""Round-6 GPU tests: the Winograd F(2,3) conv on maps wider than 32 columns (conv_wino_wide_kernel: 4 x 32-pixel
2-D tiles, the GEMM row index enumerating pixels tile by tile, the halo columns from the neighbouring tiles through
an LDS edge buffer; ADM's 64^2 .. 256^2 ResBlock convs, models/adm/unet.py:162-275).

* integer operands bit for bit against float64: zero padding only at the map's edges, the tile seams carry the real
  neighbours (every tile column and row position, single-row-of-tiles maps, several tiles per image row);
* the GroupNorm-affine prologue, temb row vector, residual, pitched tensors, the ResBlock shortcut segment;
* random operands with GroupNorm + SiLU at fp32-class accuracy against float64;
* whole ADM forwards against the direct conv (DM_CONV_WINO=0) and the reference fixture live in test_gpu_r5 / r4 /
  adm (they now take the wide kernel for their 64^2+ convs; the launch log below proves it).
"""
import pytest
import torch
import torch.nn.functional as F

import dmhip
from tests.test_gpu_ops import _ints, _nhwc, _pack, _run_conv

pytestmark = pytest.mark.gpu

WINO = 21  # ConvDesc.tile: force the Winograd kernel

WIDE_SHAPES = [(1, 64, 128, 8, 64), (2, 32, 128, 12, 96), (1, 96, 256, 16, 128), (3, 64, 128, 4, 64),
               (1, 160, 128, 8, 256)]


def _conv_logged(cuda, *args, **kw):
    dmhip.launch_log(True)
    y = _run_conv(cuda, *args, **kw)
    log = dmhip.launch_log_read()
    dmhip.launch_log(False)
    return y, log


@pytest.mark.parametrize('B,Cin,Cout,H,W', WIDE_SHAPES)
@pytest.mark.parametrize('pro', [False, True])
def test_wino_wide_exact(cuda, B, Cin, Cout, H, W, pro):
    """Integer operands (and integer GroupNorm-affine tables, no SiLU): V, U, their fp16 pieces and the fp32 sums are
    exact, so the wide-map Winograd conv equals the float64 conv bit for bit -- the halo columns at every tile seam
    included, zero padding at the map's edges only."""
    x = _ints((B, Cin, H, W), -2, 3, seed=150)
    w = _ints((Cout, Cin, 3, 3), -2, 3, seed=151)
    b = _ints((Cout, ), seed=152)
    xin, prot = x, None
    if pro:
        xin = x * 2 - 1
        prot = (torch.full((B, Cin), 2.0, device=cuda), torch.full((B, Cin), -1.0, device=cuda))
    ref = F.conv2d(xin.double(), w.double(), b.double(), padding=1).float()
    y, log = _conv_logged(cuda, _nhwc(x).to(cuda), _pack(w, cuda), Cout, H, W, 9, 1, 0, b.to(cuda), tile=WINO,
                          split='fp16x2', wino=True, pro=prot, pro_nosilu=1 if pro else 0)
    assert log == [f'conv_wino_wide_kernel<{1 if pro else 0},false>'], log
    assert torch.equal(y.cpu(), _nhwc(ref))


@pytest.mark.parametrize('H,W', [(8, 64), (4, 96)])
def test_wino_wide_rowvec_residual_pitch(cuda, H, W):
    """temb row vector, residual, pitched input and output (untouched beyond Cout), integer-exact."""
    B, Cin, Cout = 3, 64, 128
    x = _ints((B, Cin, H, W), seed=160)
    w = _ints((Cout, Cin, 3, 3), -2, 3, seed=161)
    b = _ints((Cout, ), seed=162)
    rv = _ints((B, Cout), seed=163)
    res = _ints((B, Cout, H, W), seed=164)
    ref = (F.conv2d(x.double(), w.double(), b.double(), padding=1) + rv.double()[:, :, None, None]
           + res.double()).float()
    xp = torch.full((B, H, W, 96), float('nan'), device=cuda)
    xp[..., :Cin] = _nhwc(x).to(cuda)
    y = _run_conv(cuda, xp[..., :Cin], _pack(w, cuda), Cout, H, W, 9, bias=b.to(cuda), rowvec=rv.to(cuda),
                  res=_nhwc(res).to(cuda), y_pitch=160, x_pitch=96, tile=WINO, split='fp16x2', wino=True)
    assert torch.equal(y[..., :Cout].cpu(), _nhwc(ref))
    assert torch.isnan(y[..., Cout:]).all()


@pytest.mark.parametrize('C1,C2,H,W,Cout,pro', [(64, 64, 8, 64, 128, False), (128, 256, 4, 128, 256, True),
                                                (32, 128, 12, 96, 128, False)])
def test_wino_wide_shortcut_exact(cuda, C1, C2, H, W, Cout, pro):
    """ResBlock conv2 with the 1x1 shortcut of x as a second K segment on the 2-D tiles (the shortcut rows mapped
    tile by tile), temb row vector, residual: integer-exact."""
    B = 2
    h = _ints((B, C1, H, W), seed=170)
    x = _ints((B, C2, H, W), seed=171)
    w2 = _ints((Cout, C1, 3, 3), -2, 3, seed=172)
    ws = _ints((Cout, C2, 1, 1), seed=173)
    b = _ints((Cout, ), seed=174)
    rv = _ints((B, Cout), seed=175)
    res = _ints((B, Cout, H, W), seed=176)
    K = 9 * C1 + C2
    wp = torch.zeros((Cout, K), device=cuda)
    _pack(w2, cuda, K, 0, wp)
    _pack(ws, cuda, K, 9 * C1, wp)
    hin, prot = h, None
    if pro:
        hin = h * 2 - 1
        prot = (torch.full((B, C1), 2.0, device=cuda), torch.full((B, C1), -1.0, device=cuda))
    ref = (F.conv2d(hin.double(), w2.double(), b.double(), padding=1) + rv.double()[:, :, None, None]
           + F.conv2d(x.double(), ws.double()) + res.double()).float()
    y, log = _conv_logged(cuda, _nhwc(h).to(cuda), wp, Cout, H, W, 9, bias=b.to(cuda), rowvec=rv.to(cuda),
                          res=_nhwc(res).to(cuda), x2=_nhwc(x).to(cuda), Cin2=C2, tile=WINO, split='fp16x2',
                          wino=True, pro=prot, pro_nosilu=1 if pro else 0)
    assert log == [f'conv_wino_wide_kernel<{1 if pro else 0},true>'], log
    assert torch.equal(y.cpu(), _nhwc(ref))


@pytest.mark.parametrize('B,Cin,Cout,H,W', [(2, 128, 128, 16, 64), (1, 256, 256, 8, 128), (1, 64, 128, 32, 256)])
def test_wino_wide_fp32_accuracy(cuda, report, B, Cin, Cout, H, W):
    """GroupNorm + SiLU prologue on random data: the wide-map Winograd conv's error vs float64 is at most that of the
    direct fp16x2 2-D-tile conv it replaces (conv_k32 T2D, tile 19; max and rms) -- the fp32 MFMA kernels take no fused
    prologue on wide maps; on the whole-row tiles the Winograd error is 0.28-0.47x the fp32 kernel's
    (test_gpu_r5.test_wino_fp32_accuracy)."""
    g = torch.Generator().manual_seed(180 + W)
    x = torch.randn((B, Cin, H, W), generator=g) * 2 + 0.3
    gamma, beta = torch.randn(Cin, generator=g), torch.randn(Cin, generator=g)
    w = torch.randn((Cout, Cin, 3, 3), generator=g) * (1.0 / (9 * Cin) ** 0.5)
    b = torch.randn(Cout, generator=g) * 0.01
    a = F.silu(F.group_norm(x.double(), 32, gamma.double(), beta.double(), 1e-5))
    ref = _nhwc(F.conv2d(a, w.double(), b.double(), padding=1))
    xd = _nhwc(x).to(cuda)
    pro = dmhip.groupnorm_affine(xd, B, H * W, Cin, 32, 1e-5, gamma.to(cuda), beta.to(cuda))
    wp = _pack(w, cuda)
    errs, rms = {}, {}
    for name, split, tile, wino in (('k32', 'fp16x2', 19, False), ('wino', 'fp16x2', WINO, True)):
        y = _run_conv(cuda, xd, wp, Cout, H, W, 9, 1, 0, b.to(cuda), pro=pro, split=split, tile=tile, wino=wino)
        d = y.cpu().double() - ref
        errs[name] = d.abs().max().item()
        rms[name] = d.pow(2).mean().sqrt().item()
    scale = ref.abs().max().item()
    for k in errs:
        report(f'wino_wide_accuracy_{B}_{Cin}_{Cout}_{H}x{W}_{k}_max_rel', errs[k] / scale)
        report(f'wino_wide_accuracy_{B}_{Cin}_{Cout}_{H}x{W}_{k}_rms_rel', rms[k] / scale)
    assert errs['wino'] <= errs['k32'], errs
    assert rms['wino'] <= rms['k32'], rms
    assert errs['wino'] < 4e-6 * scale, (errs, scale)


def test_adm256_wide_wino_forward(cuda, golden, report, monkeypatch):
    """The RePaint CelebA-HQ ADM-256 (reference fixture config, B = 1): its 64^2 .. 256^2 ResBlock convs on the wide-map
    Winograd kernel (the launch log shows it, with GroupNorm partials from its epilogue over the tile halves) within
    1e-5 of the direct 2-D-tile convs (DM_CONV_WINO=0) and within TOL of the reference."""
    from models.adm.unet import UNetModel
    from tests.test_gpu_parity import TOL
    from utils.synthetic import init_synthetic_
    g, meta = golden('adm')
    name = 'adm256_celebahq'
    x = torch.from_numpy(g[f'{name}_x']).to(cuda)
    t = torch.from_numpy(g[f'{name}_t']).to(cuda)
    y = torch.from_numpy(g[f'{name}_labels']).to(cuda) if f'{name}_labels' in g else None
    outs, logs = {}, {}
    for mode in ('wino', 'direct'):
        if mode == 'direct':
            monkeypatch.setenv('DM_CONV_WINO', '0')
        model = UNetModel(**meta['archs'][name]).eval()
        init_synthetic_(model)
        model = model.to(cuda)
        dmhip.launch_log(True)
        outs[mode] = model(x, t, y).cpu()
        logs[mode] = dmhip.launch_log_read()
        dmhip.launch_log(False)
        del model
        torch.cuda.empty_cache()
    monkeypatch.delenv('DM_CONV_WINO')
    assert any(lb.startswith('conv_wino_wide_kernel<2,') for lb in logs['wino']), sorted(set(logs['wino']))
    assert not any('conv_wino' in lb for lb in logs['direct'])
    err = (outs['wino'] - outs['direct']).abs().max().item()
    ref_err = (outs['wino'] - torch.from_numpy(g[f'{name}_out'])).abs().max().item()
    report('adm256_wide_wino_maxabs_vs_direct', err)
    report('adm256_wide_wino_maxabs_vs_reference', ref_err)
    assert err <= 1e-5, err
    assert ref_err <= TOL, ref_err


# ---- 4 x 4 maps (the CIFAR UNet's 4^2 level, models/unet.py:121-152): eight images per 128-pixel tile, split-K over
# the input channels (conv_wino_kernel<4, ..>: raw partial sums per split, conv_splitk_reduce adds them in split order
# with the epilogue); the plan takes it with 4 splits in place of the direct conv_k32s_kernel
SMALL_SHAPES = [(1, 64, 128, 2), (8, 256, 256, 4), (11, 128, 256, 4), (3, 512, 128, 3), (16, 96, 128, 3)]


@pytest.mark.parametrize('B,Cin,Cout,ks', SMALL_SHAPES)
@pytest.mark.parametrize('pro', [False, True])
def test_wino_small_exact(cuda, B, Cin, Cout, ks, pro):
    """Integer operands: every split's partial sums are exact, so the split-K Winograd conv on 4 x 4 maps equals the
    float64 conv bit for bit (zero padding at every image edge -- eight images side by side in a tile's patch -- a
    group's images past B, uneven splits)."""
    x = _ints((B, Cin, 4, 4), -2, 3, seed=190)
    w = _ints((Cout, Cin, 3, 3), -2, 3, seed=191)
    b = _ints((Cout, ), seed=192)
    xin, prot = x, None
    if pro:
        xin = x * 2 - 1
        prot = (torch.full((B, Cin), 2.0, device=cuda), torch.full((B, Cin), -1.0, device=cuda))
    ref = F.conv2d(xin.double(), w.double(), b.double(), padding=1).float()
    y, log = _conv_logged(cuda, _nhwc(x).to(cuda), _pack(w, cuda), Cout, 4, 4, 9, 1, 0, b.to(cuda), tile=WINO,
                          split='fp16x2', wino=True, pro=prot, pro_nosilu=1 if pro else 0, ksplit=ks)
    assert log == [f'conv_wino_kernel<4,{1 if pro else 0},false>'], log
    assert torch.equal(y.cpu(), _nhwc(ref))


def test_wino_small_rowvec_residual_pitch(cuda):
    """temb row vector, residual (added once, in the reduction), pitched input and output, integer-exact."""
    B, Cin, Cout = 9, 64, 128
    x = _ints((B, Cin, 4, 4), seed=200)
    w = _ints((Cout, Cin, 3, 3), -2, 3, seed=201)
    b = _ints((Cout, ), seed=202)
    rv = _ints((B, Cout), seed=203)
    res = _ints((B, Cout, 4, 4), seed=204)
    ref = (F.conv2d(x.double(), w.double(), b.double(), padding=1) + rv.double()[:, :, None, None]
           + res.double()).float()
    xp = torch.full((B, 4, 4, 96), float('nan'), device=cuda)
    xp[..., :Cin] = _nhwc(x).to(cuda)
    y = _run_conv(cuda, xp[..., :Cin], _pack(w, cuda), Cout, 4, 4, 9, bias=b.to(cuda), rowvec=rv.to(cuda),
                  res=_nhwc(res).to(cuda), y_pitch=160, x_pitch=96, tile=WINO, split='fp16x2', wino=True, ksplit=2)
    assert torch.equal(y[..., :Cout].cpu(), _nhwc(ref))
    assert torch.isnan(y[..., Cout:]).all()


@pytest.mark.parametrize('C1,C2,Cout,ks,pro', [(256, 512, 256, 4, False), (64, 64, 128, 2, True),
                                               (128, 192, 256, 4, False)])
def test_wino_small_shortcut_exact(cuda, C1, C2, Cout, ks, pro):
    """ResBlock conv2 with the 1x1 shortcut segment on 4 x 4 maps: each split takes its share of the shortcut steps
    (none for some splits), integer-exact."""
    B = 10
    h = _ints((B, C1, 4, 4), seed=210)
    x = _ints((B, C2, 4, 4), seed=211)
    w2 = _ints((Cout, C1, 3, 3), -2, 3, seed=212)
    ws = _ints((Cout, C2, 1, 1), seed=213)
    b = _ints((Cout, ), seed=214)
    rv = _ints((B, Cout), seed=215)
    res = _ints((B, Cout, 4, 4), seed=216)
    K = 9 * C1 + C2
    wp = torch.zeros((Cout, K), device=cuda)
    _pack(w2, cuda, K, 0, wp)
    _pack(ws, cuda, K, 9 * C1, wp)
    hin, prot = h, None
    if pro:
        hin = h * 2 - 1
        prot = (torch.full((B, C1), 2.0, device=cuda), torch.full((B, C1), -1.0, device=cuda))
    ref = (F.conv2d(hin.double(), w2.double(), b.double(), padding=1) + rv.double()[:, :, None, None]
           + F.conv2d(x.double(), ws.double()) + res.double()).float()
    y, log = _conv_logged(cuda, _nhwc(h).to(cuda), wp, Cout, 4, 4, 9, bias=b.to(cuda), rowvec=rv.to(cuda),
                          res=_nhwc(res).to(cuda), x2=_nhwc(x).to(cuda), Cin2=C2, tile=WINO, split='fp16x2',
                          wino=True, pro=prot, pro_nosilu=1 if pro else 0, ksplit=ks)
    assert log == [f'conv_wino_kernel<4,{1 if pro else 0},true>'], log
    assert torch.equal(y.cpu(), _nhwc(ref))


@pytest.mark.parametrize('B,Cin,Cout', [(64, 256, 256), (24, 512, 256)])
def test_wino_small_fp32_accuracy(cuda, report, B, Cin, Cout):
    """GroupNorm + SiLU prologue on random data at 4 x 4: the split-K Winograd conv's error vs float64 is at most the
    fp32 MFMA kernel's and its rms at most the direct fp16x2 small-map kernel's (conv_k32s, tile 15)."""
    from tests.test_gpu_conv_split import _rand_case
    xd, wp, b, pro, ref = _rand_case(cuda, B, Cin, Cout, 4, 0, seed=220)
    errs, rms = {}, {}
    for name, split, tile, wino, ks in (('fp32', False, 0, False, 0), ('k32s', 'fp16x2', 15, False, 2),
                                        ('wino', 'fp16x2', WINO, True, 4)):
        y = _run_conv(cuda, xd, wp, Cout, 4, 4, 9, 1, 0, b.to(cuda), pro=pro, split=split, tile=tile, wino=wino,
                      ksplit=ks)
        d = y.cpu().double() - _nhwc(ref)
        errs[name] = d.abs().max().item()
        rms[name] = d.pow(2).mean().sqrt().item()
    scale = ref.abs().max().item()
    for k in errs:
        report(f'wino_small_accuracy_{B}_{Cin}_{Cout}_{k}_max_rel', errs[k] / scale)
        report(f'wino_small_accuracy_{B}_{Cin}_{Cout}_{k}_rms_rel', rms[k] / scale)
    assert errs['wino'] <= errs['fp32'], errs
    assert rms['wino'] <= rms['fp32'], rms
    assert rms['wino'] <= rms['k32s'], rms
    assert errs['wino'] < 6e-6 * scale, (errs, scale)


# ------------------------------------------------------------------ the 4 x 4 middle attention block (attn_small)
def _cifar_forward_labels(cuda, golden, x, t):
    from tests.test_gpu_parity import _model
    _, meta = golden('forward')
    model, _ = _model(meta, 'cifar10', cuda)
    out = model(x, t)
    h = model.native_handle(torch.device(cuda))
    dmhip.unet_profile_enable(h, 1)
    model(x, t)
    labels = [op['label'] for op in dmhip.unet_profile_read(h)]
    dmhip.unet_profile_enable(h, 0)
    return out, labels


@pytest.mark.parametrize('B', [3, 8])
def test_small_attention_vs_unfolded(cuda, golden, monkeypatch, B):
    """The CIFAR-10 UNet's middle attention block (one head of 256 channels on the 4 x 4 map, models/unet.py:97-99,
    models/modules.py:77-102) runs as one attn_small_kernel launch -- folded T / S / softmax / P xn / Wg, fp32 -- in
    place of the unfolded qkv conv, S GEMM, softmax_rows, PV GEMM and projection launches (DM_ATTN_SMALL=0): whole
    forwards within 1e-5 of each other, and the consumer's GroupNorm statistics come from the kernel (no gn_partial
    pass after it)."""
    g = torch.Generator().manual_seed(61)
    x = torch.randn((B, 3, 32, 32), generator=g).to(cuda)
    t = torch.randint(0, 1000, (B, ), generator=g).to(cuda)
    out_s, lab_s = _cifar_forward_labels(cuda, golden, x, t)
    monkeypatch.setenv('DM_ATTN_SMALL', '0')
    out_u, lab_u = _cifar_forward_labels(cuda, golden, x, t)
    assert lab_s.count('attn_small_kernel') == 1, lab_s
    assert 'attn_small_kernel' not in lab_u and 'softmax_rows' in lab_u, lab_u
    assert 'softmax_rows' not in lab_s, lab_s
    assert lab_s.count('gn_partial') < lab_u.count('gn_partial'), (lab_s, lab_u)
    assert len(lab_s) <= len(lab_u) - 5, (len(lab_s), len(lab_u))
    err = (out_s - out_u).abs().max().item()
    assert err <= 1e-5, err
    assert torch.isfinite(out_s).all()


def test_small_attention_vs_reference(cuda, golden, report):
    """Reference fixture (tests/golden/forward.npz, the reference UNet at B = 2): the forward with the small-map block
    within 1e-4 (north_star tolerance); the label proves the kernel ran."""
    from tests.test_gpu_parity import TOL
    arrays, _ = golden('forward')
    y, labels = _cifar_forward_labels(cuda, golden, torch.from_numpy(arrays['cifar10_x']).to(cuda),
                                      torch.from_numpy(arrays['cifar10_t']).to(cuda))
    assert labels.count('attn_small_kernel') == 1, labels
    err = (y.cpu() - torch.from_numpy(arrays['cifar10_y'])).abs().max().item()
    report('forward_cifar10_small_attention_maxabs_vs_reference', err)
    assert err <= TOL, err


# ------------------------------------------------------------------ the time MLP / temb projections (linear_rows)
@pytest.mark.parametrize('B', [2, 256])
def test_linear_rows_vs_gemm(cuda, golden, monkeypatch, B):
    """The time MLP and the ResBlocks' temb projections (models/unet.py:64-69, :18-21) run on linear_rows_kernel
    (16 lanes per output over K, fp32 FMAs) where gemm_kernel's tiles would not fill the CUs: the two 512-wide time
    MLP launches per forward (the 4992-wide temb projection stays on gemm_kernel), whole forwards within 1e-5 of the
    gemm_kernel path (DM_LIN_ROWS=0, fp32 MFMA), and rows of the B = 256 forward equal the B = 3 forward's bit for
    bit (per-row sums depend on K only)."""
    g = torch.Generator().manual_seed(62)
    x = torch.randn((B, 3, 32, 32), generator=g).to(cuda)
    t = torch.randint(0, 1000, (B, ), generator=g).to(cuda)
    out_r, lab_r = _cifar_forward_labels(cuda, golden, x, t)
    assert lab_r.count('linear_rows_kernel') == 2, lab_r
    if B == 256:
        idx = [0, 77, 255]
        small, _ = _cifar_forward_labels(cuda, golden, x[idx].contiguous(), t[idx].contiguous())
        assert torch.equal(out_r[idx], small)
    monkeypatch.setenv('DM_LIN_ROWS', '0')
    out_g, lab_g = _cifar_forward_labels(cuda, golden, x, t)
    assert 'linear_rows_kernel' not in lab_g, lab_g
    err = (out_r - out_g).abs().max().item()
    assert err <= 1e-5, err
