"""The split halo-patch convolutions (conv_patch3.hip: bf16x3 and fp16x2) against fp64 torch references.

Structure: integer operands in [-2, 3) are exact in bf16 and fp16 (the low pieces are zero; the fp16x2
weight row scales are powers of two), so indexing, padding, tap walk, segments and epilogues compare bit
for bit as for the fp32 kernel. Numerics: on random fp32 operands both splits must be as accurate as the
fp32 MFMA kernel (same order of error vs fp64), i.e. fp32-level, never bf16/fp16-level (~1e-2 / 1e-3
relative). fp16x2 range: an activation beyond 65504 must raise the range flag."""
import pytest
import torch
import torch.nn.functional as F

import dmhip
from tests.test_gpu_ops import _ints, _nhwc, _pack, _pack_subpix, _run_conv

pytestmark = pytest.mark.gpu
KINDS = ['bf16x3', 'fp16x2']


@pytest.mark.parametrize('kind', KINDS)
@pytest.mark.parametrize('tile', [0, 4, 5, 6, 7, 8])
@pytest.mark.parametrize('B,Cin,Cout,H,up', [
    (2, 32, 64, 8, 0), (1, 128, 256, 16, 0), (5, 64, 64, 4, 0), (3, 32, 96, 5, 0), (4, 64, 128, 32, 1 - 1),
    (3, 64, 64, 16, 1), (2, 32, 64, 8, 1), (2, 48, 32, 8, 0),
])
def test_split_conv3x3_exact(cuda, B, Cin, Cout, H, up, tile, kind):
    x = _ints((B, Cin, H, H), -2, 3, seed=10)
    w = _ints((Cout, Cin, 3, 3), -2, 3, seed=11)
    b = _ints((Cout, ), seed=12)
    xin = F.interpolate(x, scale_factor=2, mode='nearest') if up else x
    ref = F.conv2d(xin.double(), w.double(), b.double(), padding=1).float()
    Ho = ref.shape[-1]
    wp = _pack(w, cuda) if Cin % 32 == 0 else None
    if wp is None:
        pytest.skip('packing needs Cin % 32 == 0')
    y = _run_conv(cuda, _nhwc(x).to(cuda), wp, Cout, Ho, Ho, 9, 1, up, b.to(cuda), tile=tile, split=kind)
    assert torch.equal(y.cpu(), _nhwc(ref))


@pytest.mark.parametrize('kind', KINDS)
@pytest.mark.parametrize('tile', [0, 4, 5, 6, 7, 8])
def test_split_conv_segments_rowvec_residual_pitch(cuda, tile, kind):
    B, C1, C2, Cout, H = 3, 64, 32, 64, 8
    h = _ints((B, C1, H, H), seed=20)
    x = _ints((B, C2, H, H), seed=21)
    w2 = _ints((Cout, C1, 3, 3), -2, 3, seed=22)
    ws = _ints((Cout, C2, 1, 1), seed=23)
    b = _ints((Cout, ), seed=24)
    rv = _ints((B, Cout), seed=25)
    res = _ints((B, Cout, H, H), seed=26)
    K = 9 * C1 + C2
    wp = torch.zeros((Cout, K), device=cuda)
    _pack(w2, cuda, K, 0, wp)
    _pack(ws, cuda, K, 9 * C1, wp)
    ref = (F.conv2d(h.double(), w2.double(), b.double(), padding=1) + rv.double()[:, :, None, None]
           + F.conv2d(x.double(), ws.double()) + res.double()).float()
    y = _run_conv(cuda, _nhwc(h).to(cuda), wp, Cout, H, H, 9, bias=b.to(cuda), rowvec=rv.to(cuda),
                  res=_nhwc(res).to(cuda), x2=_nhwc(x).to(cuda), Cin2=C2, y_pitch=96, tile=tile, split=kind)
    assert torch.equal(y[..., :Cout].cpu(), _nhwc(ref))
    assert torch.isnan(y[..., Cout:]).all()


@pytest.mark.parametrize('kind', KINDS)
@pytest.mark.parametrize('tile', [0, 4, 5, 6, 7, 8])
@pytest.mark.parametrize('B,Cin,Cout,H', [(3, 64, 64, 16), (2, 32, 64, 8), (4, 64, 128, 8), (2, 96, 64, 4)])
def test_split_conv_subpixel_exact(cuda, B, Cin, Cout, H, tile, kind):
    x = _ints((B, Cin, H, H), -2, 3, seed=70)
    w = _ints((Cout, Cin, 3, 3), -1, 2, seed=71)  # summed sub-pixel weights stay within bf16's exact range
    b = _ints((Cout, ), seed=72)
    ref = F.conv2d(F.interpolate(x, scale_factor=2, mode='nearest').double(), w.double(), b.double(),
                   padding=1).float()
    try:
        y = _run_conv(cuda, _nhwc(x).to(cuda), _pack_subpix(w, cuda), Cout, 2 * H, 2 * H, 9, 1, 2, b.to(cuda),
                      tile=tile, split=kind)
    except ValueError as e:
        pytest.skip(str(e))
    assert torch.equal(y.cpu(), _nhwc(ref))


def _rand_case(cuda, B, Cin, Cout, H, up, seed, wscale=1.0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn((B, Cin, H, H), generator=g) * 2 + 0.3
    gamma, beta = torch.randn(Cin, generator=g), torch.randn(Cin, generator=g)
    w = torch.randn((Cout, Cin, 3, 3), generator=g) * (wscale / (9 * Cin) ** 0.5)
    b = torch.randn(Cout, generator=g) * 0.01 * wscale
    a = F.silu(F.group_norm(x.double(), 32, gamma.double(), beta.double(), 1e-5))
    if up:
        a = F.interpolate(a, scale_factor=2, mode='nearest')
    ref = F.conv2d(a, w.double(), b.double(), padding=1)
    xd = _nhwc(x).to(cuda)
    pro = dmhip.groupnorm_affine(xd, B, H * H, Cin, 32, 1e-5, gamma.to(cuda), beta.to(cuda))
    wp = _pack_subpix(w, cuda) if up else _pack(w, cuda)
    return xd, wp, b, pro, ref


@pytest.mark.parametrize('B,Cin,Cout,H,up', [(4, 128, 128, 32, 0), (8, 256, 256, 16, 0), (16, 256, 256, 8, 0),
                                             (4, 256, 128, 16, 2), (2, 384, 128, 32, 0)])
def test_split_conv_fp32_accuracy(cuda, B, Cin, Cout, H, up):
    """fused GN+SiLU conv on random data: split errors vs fp64 within 2x the fp32 kernel's error."""
    xd, wp, b, pro, ref = _rand_case(cuda, B, Cin, Cout, H, up, seed=90)
    Ho = ref.shape[-1]
    errs = []
    for split in (False, 'bf16x3', 'fp16x2'):
        y = _run_conv(cuda, xd, wp, Cout, Ho, Ho, 9, 1, up, b.to(cuda), pro=pro, split=split)
        errs.append((y.cpu().double() - _nhwc(ref)).abs().max().item())
    scale = ref.abs().max().item()
    for e in errs[1:]:
        assert e < 2.0 * errs[0] + 1e-7 * scale, errs
        assert e < 4e-6 * scale, (errs, scale)


@pytest.mark.parametrize('wscale', [1.0, 1e-6, 3e4])
def test_fp16x2_weight_scale_range(cuda, wscale):
    """fp16x2 row scales: weights far below / above fp16's normal range keep fp32-level accuracy
    (relative to the output scale), as the bf16x3 path does."""
    xd, wp, b, pro, ref = _rand_case(cuda, 4, 64, 64, 8, 0, seed=91, wscale=wscale)
    errs = []
    for split in (False, 'bf16x3', 'fp16x2'):
        y = _run_conv(cuda, xd, wp, 64, 8, 8, 9, 1, 0, b.to(cuda), pro=pro, split=split)
        errs.append((y.cpu().double() - _nhwc(ref)).abs().max().item())
    scale = ref.abs().max().item()
    assert errs[2] < 2.0 * errs[0] + 1e-7 * scale, errs


@pytest.mark.parametrize('peak,flagged', [(6.0e4, False), (1.0e5, True)])
def test_fp16x2_range_flag(cuda, peak, flagged):
    """an activation beyond fp16's largest finite value (65504) raises the range flag; below it the
    fp16x2 result is fp32-accurate."""
    B, C, H = 2, 64, 8
    g = torch.Generator().manual_seed(92)
    x = torch.randn((B, C, H, H), generator=g)
    x[1, 5, 3, 4] = peak
    w = torch.randn((C, C, 3, 3), generator=g) * 0.01
    ref = F.conv2d(x.double(), w.double(), padding=1)
    flag = torch.zeros(1, dtype=torch.int32, device=cuda)
    y = _run_conv(cuda, _nhwc(x).to(cuda), _pack(w, cuda), C, H, H, 9, split='fp16x2', range_flag=flag)
    assert bool(flag.item()) == flagged
    if not flagged:
        assert (y.cpu().double() - _nhwc(ref)).abs().max().item() < 4e-6 * ref.abs().max().item()


@pytest.mark.parametrize('B,Cin,Cout,H', [(2, 64, 96, 16), (3, 256, 768, 16), (5, 32, 64, 4), (1, 128, 256, 8),
                                          (3, 96, 40, 5)])
def test_split_pointwise_exact(cuda, B, Cin, Cout, H):
    """1x1 conv on the split kernel (MODE 3, the attention qkv / proj): bias, residual, output pitch and
    ragged M (rows not a multiple of the 128-row tile) bit-exact on integer operands."""
    x = _ints((B, Cin, H, H), -2, 3, seed=30)
    w = _ints((Cout, Cin, 1, 1), -2, 3, seed=31)
    b = _ints((Cout, ), seed=32)
    res = _ints((B, Cout, H, H), seed=33)
    ref = (F.conv2d(x.double(), w.double(), b.double()) + res.double()).float()
    y = _run_conv(cuda, _nhwc(x).to(cuda), _pack(w, cuda), Cout, H, H, 1, bias=b.to(cuda), res=_nhwc(res).to(cuda),
                  y_pitch=Cout + 8, split='fp16x2')
    assert torch.equal(y[..., :Cout].cpu(), _nhwc(ref))
    assert torch.isnan(y[..., Cout:]).all()


@pytest.mark.parametrize('silu', [0, 1])
def test_split_pointwise_groupnorm_accuracy(cuda, silu):
    """GroupNorm (+ optional SiLU) prologue + 1x1 conv on random data: fp32-level error vs fp64."""
    B, C, Cout, H = 4, 256, 768, 16
    g = torch.Generator().manual_seed(34)
    x = torch.randn((B, C, H, H), generator=g) * 2 + 0.3
    gamma, beta = torch.randn(C, generator=g), torch.randn(C, generator=g)
    w = torch.randn((Cout, C, 1, 1), generator=g) * C ** -0.5
    b = torch.randn(Cout, generator=g) * 0.01
    a = F.group_norm(x.double(), 32, gamma.double(), beta.double(), 1e-5)
    if silu:
        a = F.silu(a)
    ref = _nhwc(F.conv2d(a, w.double(), b.double()))
    xd = _nhwc(x).to(cuda)
    pro = dmhip.groupnorm_affine(xd, B, H * H, C, 32, 1e-5, gamma.to(cuda), beta.to(cuda))
    y = _run_conv(cuda, xd, _pack(w, cuda), Cout, H, H, 1, bias=b.to(cuda), pro=pro, pro_nosilu=1 - silu,
                  split='fp16x2')
    err = (y.cpu().double() - ref).abs().max().item()
    assert err < 2e-6 * ref.abs().max().item(), err


@pytest.mark.parametrize('B,Cin,Cout,H', [(2, 32, 64, 32), (3, 64, 128, 16), (5, 64, 64, 8), (3, 96, 32, 4),
                                          (2, 128, 256, 16)])
def test_split_conv_stride2_exact(cuda, B, Cin, Cout, H):
    """stride-2 3x3 (Downsample) on the split kernel (MODE 4, parity-split patch columns, several images
    per tile at 4x4 outputs) bit-exact on integer operands."""
    x = _ints((B, Cin, H, H), -2, 3, seed=40)
    w = _ints((Cout, Cin, 3, 3), -2, 3, seed=41)
    b = _ints((Cout, ), seed=42)
    ref = F.conv2d(x.double(), w.double(), b.double(), stride=2, padding=1).float()
    Ho = ref.shape[-1]
    y = _run_conv(cuda, _nhwc(x).to(cuda), _pack(w, cuda), Cout, Ho, Ho, 9, 2, 0, b.to(cuda), split='fp16x2')
    assert torch.equal(y.cpu(), _nhwc(ref))


def test_split_conv_stride2_fp32_accuracy(cuda):
    """random stride-2 conv: split error vs fp64 within 2x the fp32 kernel's."""
    g = torch.Generator().manual_seed(43)
    B, Cin, Cout, H = 8, 128, 128, 32
    x = torch.randn((B, Cin, H, H), generator=g) * 3
    w = torch.randn((Cout, Cin, 3, 3), generator=g) * (1.0 / (9 * Cin) ** 0.5)
    ref = _nhwc(F.conv2d(x.double(), w.double(), stride=2, padding=1))
    errs = []
    for split in (False, 'fp16x2'):
        y = _run_conv(cuda, _nhwc(x).to(cuda), _pack(w, cuda), Cout, H // 2, H // 2, 9, 2, split=split)
        errs.append((y.cpu().double() - ref).abs().max().item())
    assert errs[1] < 2.0 * errs[0] + 1e-7 * ref.abs().max().item(), errs


@pytest.mark.parametrize('tile', [0, 9])
@pytest.mark.parametrize('B,Cin,Cout,H,W', [(1, 32, 64, 4, 256), (2, 64, 32, 3, 128), (1, 32, 64, 4, 64),
                                            (1, 32, 32, 2, 512)])
def test_split_conv_row_segments_exact(cuda, B, Cin, Cout, H, W, tile):
    """Wide maps (ADM 256^2 / 128^2 / 64^2) on the fp16x2 split kernel: 128-pixel row segments with a
    3 x 130 halo patch (or two whole 64-wide rows), bias + GroupNorm-free prologue, integer operands
    exact (bit-equal to the fp64 reference)."""
    x = _ints((B, Cin, H, W), -2, 3, seed=90)
    w = _ints((Cout, Cin, 3, 3), -2, 3, seed=91)
    b = _ints((Cout, ), seed=92)
    if Cin % 32:
        pytest.skip('packing needs Cin % 32 == 0')
    ref = F.conv2d(x.double(), w.double(), b.double(), padding=1).float()
    y = _run_conv(cuda, _nhwc(x).to(cuda), _pack(w, cuda), Cout, H, W, 9, 1, 0, b.to(cuda), tile=tile,
                  split='fp16x2')
    assert torch.equal(y.cpu(), _nhwc(ref))


@pytest.mark.parametrize('tile', [0, 9])
def test_split_conv_row_segments_shortcut_residual_prologue(cuda, tile):
    """Row segments with the ResBlock epilogue pieces: 1x1 shortcut as a second K segment, per-image
    rowvec, residual, and the GroupNorm-affine + SiLU prologue (scale 1, shift 0 on small integers:
    SiLU values are not integers, so this part checks against an fp64 SiLU with fp32 tolerance)."""
    B, C1, C2, Cout, H, W = 2, 64, 32, 64, 3, 256
    h = _ints((B, C1, H, W), seed=94)
    x = _ints((B, C2, H, W), seed=95)
    w2 = _ints((Cout, C1, 3, 3), -2, 3, seed=96)
    ws = _ints((Cout, C2, 1, 1), seed=97)
    b = _ints((Cout, ), seed=98)
    rv = _ints((B, Cout), seed=99)
    K = 9 * C1 + C2
    wp = torch.zeros((Cout, K), device=cuda)
    _pack(w2, cuda, K, 0, wp)
    _pack(ws, cuda, K, 9 * C1, wp)
    ref = (F.conv2d(h.double(), w2.double(), b.double(), padding=1) + rv.double()[:, :, None, None]
           + F.conv2d(x.double(), ws.double())).float()
    y = _run_conv(cuda, _nhwc(h).to(cuda), wp, Cout, H, W, 9, bias=b.to(cuda), rowvec=rv.to(cuda),
                  x2=_nhwc(x).to(cuda), Cin2=C2, tile=tile, split='fp16x2')
    assert torch.equal(y.cpu(), _nhwc(ref))
    sc = torch.ones((B, C1), device=cuda)
    sh = torch.zeros((B, C1), device=cuda)
    refp = (F.conv2d(F.silu(h.double()), w2.double(), b.double(), padding=1)).float()
    y2 = _run_conv(cuda, _nhwc(h).to(cuda), _pack(w2, cuda), Cout, H, W, 9, bias=b.to(cuda), tile=tile,
                   pro=(sc, sh), split='fp16x2')
    assert (y2.cpu() - _nhwc(refp)).abs().max().item() <= 2e-4 * float(refp.abs().max())
