"""The K = 32 fp16x2 split conv (conv_k32.hip: v_mfma_f32_16x16x32_f16, 32-channel chunks) against fp64
torch references, as tests/test_gpu_conv_split.py does for conv_patch3: integer operands compare bit for
bit (indexing, padding, tap walk, both K segments, epilogue), random operands must keep fp32-level
accuracy (within 2x of the fp32 MFMA kernel's error vs fp64), and an activation beyond fp16's range must
raise the range flag. Tiles: 10 = 128 x 128, 11 = 128 x 64, 12 / 13 = 64 x 64 / 64 x 128 split-K (forced);
0 = the automatic choice, which takes this kernel for the 8- / 16- / 32-pixel-wide maps the UNets run at
128-row tiles and for the split-K convs of maps of <= 16 pixels."""
import pytest
import torch
import torch.nn.functional as F

from tests.test_gpu_conv_split import _rand_case
from tests.test_gpu_ops import _ints, _nhwc, _pack, _pack_subpix, _run_conv

pytestmark = pytest.mark.gpu
TILES = [10, 11, 0]


@pytest.mark.parametrize('tile', TILES)
@pytest.mark.parametrize('B,Cin,Cout,H', [
    (1, 128, 256, 16), (2, 32, 64, 16), (2, 96, 96, 32), (1, 64, 128, 32), (3, 160, 64, 16), (1, 256, 160, 32),
    (3, 64, 64, 8), (2, 256, 128, 8),
])
def test_k32_conv3x3_exact(cuda, B, Cin, Cout, H, tile):
    x = _ints((B, Cin, H, H), -2, 3, seed=10)
    w = _ints((Cout, Cin, 3, 3), -2, 3, seed=11)
    b = _ints((Cout, ), seed=12)
    ref = F.conv2d(x.double(), w.double(), b.double(), padding=1).float()
    y = _run_conv(cuda, _nhwc(x).to(cuda), _pack(w, cuda), Cout, H, H, 9, 1, 0, b.to(cuda), tile=tile,
                  split='fp16x2')
    assert torch.equal(y.cpu(), _nhwc(ref))


@pytest.mark.parametrize('tile', TILES)
@pytest.mark.parametrize('C1,C2,H', [(64, 32, 16), (96, 64, 32), (32, 128, 16), (64, 64, 8)])
def test_k32_segments_rowvec_residual_pitch(cuda, tile, C1, C2, H):
    """ResBlock conv2: 3x3 over h + the 1x1 shortcut of x as a second K segment, temb row vector,
    residual, pitched output (untouched beyond Cout)."""
    B, Cout = 3, 64
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
                  res=_nhwc(res).to(cuda), x2=_nhwc(x).to(cuda), Cin2=C2, y_pitch=96, tile=tile, split='fp16x2')
    assert torch.equal(y[..., :Cout].cpu(), _nhwc(ref))
    assert torch.isnan(y[..., Cout:]).all()


@pytest.mark.parametrize('B,Cin,Cout,H', [(4, 128, 128, 32), (8, 256, 256, 16), (2, 384, 128, 32),
                                          (4, 512, 256, 16), (5, 256, 256, 8)])
def test_k32_fp32_accuracy(cuda, B, Cin, Cout, H):
    """fused GroupNorm + SiLU conv on random data: the K = 32 kernel's error vs fp64 is within 2x the
    fp32 MFMA kernel's (and of the same size as conv_patch3's fp16x2 128-row tile)."""
    xd, wp, b, pro, ref = _rand_case(cuda, B, Cin, Cout, H, 0, seed=90)
    errs = {}
    for name, split, tile in (('fp32', False, 0), ('patch3', 'fp16x2', 4), ('k32', 'fp16x2', 10),
                              ('k32_64', 'fp16x2', 11)):
        y = _run_conv(cuda, xd, wp, Cout, H, H, 9, 1, 0, b.to(cuda), pro=pro, split=split, tile=tile)
        errs[name] = (y.cpu().double() - _nhwc(ref)).abs().max().item()
    scale = ref.abs().max().item()
    for k in ('k32', 'k32_64'):
        assert errs[k] < 2.0 * errs['fp32'] + 1e-7 * scale, errs
        assert errs[k] < 4e-6 * scale, (errs, scale)


def test_k32_range_flag(cuda):
    """An activation beyond 65504 (no fp16 image) raises the range flag; in range it stays clear."""
    B, C, H = 2, 64, 16
    g = torch.Generator().manual_seed(5)
    x = torch.randn((B, C, H, H), generator=g)
    w = torch.randn((C, C, 3, 3), generator=g) * 0.05
    wp = _pack(w, cuda)
    for scale, expect in ((1.0, 0), (1e5, 1)):
        flag = torch.zeros(1, dtype=torch.int32, device=cuda)
        _run_conv(cuda, _nhwc(x * scale).to(cuda), wp, C, H, H, 9, 1, 0, tile=10, split='fp16x2', range_flag=flag)
        assert int(flag.item()) == expect


@pytest.mark.parametrize('tile', [12, 13, 0])
@pytest.mark.parametrize('ksplit', [2, 4])
@pytest.mark.parametrize('B,Cin,Cout,H', [(5, 256, 256, 4), (3, 128, 64, 4), (2, 256, 128, 2)])
def test_k32_splitk_exact(cuda, B, Cin, Cout, H, ksplit, tile):
    """split-K tiles (maps of <= 16 pixels): partial sums over input-channel ranges, reduced with bias."""
    x = _ints((B, Cin, H, H), -2, 3, seed=30)
    w = _ints((Cout, Cin, 3, 3), -2, 3, seed=31)
    b = _ints((Cout, ), seed=32)
    ref = F.conv2d(x.double(), w.double(), b.double(), padding=1).float()
    y = _run_conv(cuda, _nhwc(x).to(cuda), _pack(w, cuda), Cout, H, H, 9, 1, 0, b.to(cuda), tile=tile,
                  split='fp16x2', ksplit=ksplit)
    assert torch.equal(y.cpu(), _nhwc(ref))


@pytest.mark.parametrize('tile', [12, 13])
def test_k32_splitk_segments_rowvec_residual(cuda, tile):
    B, C1, C2, Cout, H = 3, 256, 64, 128, 4
    h = _ints((B, C1, H, H), seed=40)
    x = _ints((B, C2, H, H), seed=41)
    w2 = _ints((Cout, C1, 3, 3), -2, 3, seed=42)
    ws = _ints((Cout, C2, 1, 1), seed=43)
    b = _ints((Cout, ), seed=44)
    rv = _ints((B, Cout), seed=45)
    res = _ints((B, Cout, H, H), seed=46)
    K = 9 * C1 + C2
    wp = torch.zeros((Cout, K), device=cuda)
    _pack(w2, cuda, K, 0, wp)
    _pack(ws, cuda, K, 9 * C1, wp)
    ref = (F.conv2d(h.double(), w2.double(), b.double(), padding=1) + rv.double()[:, :, None, None]
           + F.conv2d(x.double(), ws.double()) + res.double()).float()
    y = _run_conv(cuda, _nhwc(h).to(cuda), wp, Cout, H, H, 9, bias=b.to(cuda), rowvec=rv.to(cuda),
                  res=_nhwc(res).to(cuda), x2=_nhwc(x).to(cuda), Cin2=C2, tile=tile, split='fp16x2', ksplit=4)
    assert torch.equal(y.cpu(), _nhwc(ref))


@pytest.mark.parametrize('B,Cin,Cout,H', [(16, 256, 256, 4), (8, 512, 256, 4)])
def test_k32_splitk_fp32_accuracy(cuda, B, Cin, Cout, H):
    xd, wp, b, pro, ref = _rand_case(cuda, B, Cin, Cout, H, 0, seed=92)
    errs = {}
    for name, split, tile in (('fp32', False, 0), ('k32s', 'fp16x2', 12), ('k32s128', 'fp16x2', 13)):
        y = _run_conv(cuda, xd, wp, Cout, H, H, 9, 1, 0, b.to(cuda), pro=pro, split=split, tile=tile,
                      ksplit=4 if split else 0)
        errs[name] = (y.cpu().double() - _nhwc(ref)).abs().max().item()
    scale = ref.abs().max().item()
    for k in ('k32s', 'k32s128'):
        assert errs[k] < 2.0 * errs['fp32'] + 1e-7 * scale, errs
        assert errs[k] < 4e-6 * scale, (errs, scale)


@pytest.mark.parametrize('tile', TILES)
@pytest.mark.parametrize('B,Cin,Cout,H', [(3, 64, 64, 16), (2, 256, 128, 8), (1, 96, 96, 16), (4, 64, 128, 8)])
def test_k32_subpixel_exact(cuda, B, Cin, Cout, H, tile):
    """sub-pixel form of nearest-2x + 3x3 (4 parity convs of 4 taps), output pixels scattered by parity."""
    x = _ints((B, Cin, H, H), -2, 3, seed=70)
    w = _ints((Cout, Cin, 3, 3), -1, 2, seed=71)  # summed sub-pixel weights stay exact in fp16
    b = _ints((Cout, ), seed=72)
    ref = F.conv2d(F.interpolate(x, scale_factor=2, mode='nearest').double(), w.double(), b.double(),
                   padding=1).float()
    y = _run_conv(cuda, _nhwc(x).to(cuda), _pack_subpix(w, cuda), Cout, 2 * H, 2 * H, 9, 1, 2, b.to(cuda),
                  tile=tile, split='fp16x2')
    assert torch.equal(y.cpu(), _nhwc(ref))


@pytest.mark.parametrize('B,Cin,Cout,H', [(4, 256, 128, 16), (16, 256, 256, 8)])
def test_k32_subpixel_fp32_accuracy(cuda, B, Cin, Cout, H):
    xd, wp, b, pro, ref = _rand_case(cuda, B, Cin, Cout, H, 1, seed=93)
    errs = {}
    for name, split, tile in (('fp32', False, 0), ('k32', 'fp16x2', 10), ('k32_64', 'fp16x2', 11)):
        y = _run_conv(cuda, xd, wp, Cout, 2 * H, 2 * H, 9, 1, 2, b.to(cuda), pro=pro, split=split, tile=tile)
        errs[name] = (y.cpu().double() - _nhwc(ref)).abs().max().item()
    scale = ref.abs().max().item()
    for k in ('k32', 'k32_64'):
        assert errs[k] < 2.0 * errs['fp32'] + 1e-7 * scale, errs
        assert errs[k] < 4e-6 * scale, (errs, scale)


@pytest.mark.parametrize('tile', [14, 16, 0])
@pytest.mark.parametrize('B,Cin,Cout,H', [(2, 64, 128, 64), (1, 32, 64, 128), (1, 64, 64, 256), (3, 96, 160, 64)])
def test_k32_row_segments_exact(cuda, B, Cin, Cout, H, tile):
    """64 x 128 tiles over one 64-pixel row or a 64-pixel segment of a wider row (ADM's 64^2 .. 256^2 maps)."""
    x = _ints((B, Cin, H, H), -2, 3, seed=50)
    w = _ints((Cout, Cin, 3, 3), -2, 3, seed=51)
    b = _ints((Cout, ), seed=52)
    ref = F.conv2d(x.double(), w.double(), b.double(), padding=1).float()
    y = _run_conv(cuda, _nhwc(x).to(cuda), _pack(w, cuda), Cout, H, H, 9, 1, 0, b.to(cuda), tile=tile,
                  split='fp16x2')
    assert torch.equal(y.cpu(), _nhwc(ref))


@pytest.mark.parametrize('tile', [14, 16, 0])
def test_k32_row_segments_segments_rowvec_residual(cuda, tile):
    B, C1, C2, Cout, H = 2, 64, 32, 64, 128
    h = _ints((B, C1, H, H), seed=60)
    x = _ints((B, C2, H, H), seed=61)
    w2 = _ints((Cout, C1, 3, 3), -2, 3, seed=62)
    ws = _ints((Cout, C2, 1, 1), seed=63)
    b = _ints((Cout, ), seed=64)
    rv = _ints((B, Cout), seed=65)
    res = _ints((B, Cout, H, H), seed=66)
    K = 9 * C1 + C2
    wp = torch.zeros((Cout, K), device=cuda)
    _pack(w2, cuda, K, 0, wp)
    _pack(ws, cuda, K, 9 * C1, wp)
    ref = (F.conv2d(h.double(), w2.double(), b.double(), padding=1) + rv.double()[:, :, None, None]
           + F.conv2d(x.double(), ws.double()) + res.double()).float()
    y = _run_conv(cuda, _nhwc(h).to(cuda), wp, Cout, H, H, 9, bias=b.to(cuda), rowvec=rv.to(cuda),
                  res=_nhwc(res).to(cuda), x2=_nhwc(x).to(cuda), Cin2=C2, y_pitch=96, tile=tile, split='fp16x2')
    assert torch.equal(y[..., :Cout].cpu(), _nhwc(ref))
    assert torch.isnan(y[..., Cout:]).all()


@pytest.mark.parametrize('tile', [14, 16, 0])
@pytest.mark.parametrize('B,Cin,Cout,H', [(1, 64, 64, 64), (1, 32, 64, 128)])
def test_k32_row_segments_subpixel_exact(cuda, B, Cin, Cout, H, tile):
    x = _ints((B, Cin, H, H), -2, 3, seed=80)
    w = _ints((Cout, Cin, 3, 3), -1, 2, seed=81)
    b = _ints((Cout, ), seed=82)
    ref = F.conv2d(F.interpolate(x, scale_factor=2, mode='nearest').double(), w.double(), b.double(),
                   padding=1).float()
    y = _run_conv(cuda, _nhwc(x).to(cuda), _pack_subpix(w, cuda), Cout, 2 * H, 2 * H, 9, 1, 2, b.to(cuda),
                  tile=tile, split='fp16x2')
    assert torch.equal(y.cpu(), _nhwc(ref))


@pytest.mark.parametrize('tile', [14, 16])
@pytest.mark.parametrize('B,Cin,Cout,H', [(2, 256, 256, 64), (1, 256, 128, 128), (1, 128, 128, 256)])
def test_k32_row_segments_fp32_accuracy(cuda, B, Cin, Cout, H, tile):
    """(the fp32 kernels have no fused-GroupNorm shape this wide: the bound alone, as for the other tiles;
    tile 16 = the 512-thread 128-pixel row segments / two-row tiles)"""
    xd, wp, b, pro, ref = _rand_case(cuda, B, Cin, Cout, H, 0, seed=94)
    y = _run_conv(cuda, xd, wp, Cout, H, H, 9, 1, 0, b.to(cuda), pro=pro, split='fp16x2', tile=tile)
    err = (y.cpu().double() - _nhwc(ref)).abs().max().item()
    scale = ref.abs().max().item()
    assert err < 4e-6 * scale, (err, scale)


# ---- the small-map kernel (conv_k32s_kernel, tile 15 forced / 0 automatic with ksplit = 2): 64 x 64 tiles of
# four 4 x 4 images, the K reduction split in two inside the block
@pytest.mark.parametrize('tile', [15, 0])
@pytest.mark.parametrize('B,Cin,Cout,H', [(5, 256, 256, 4), (3, 128, 64, 4), (8, 512, 256, 4), (1, 64, 128, 4),
                                          (4, 256, 192, 4)])
def test_k32_small_exact(cuda, B, Cin, Cout, H, tile):
    x = _ints((B, Cin, H, H), -2, 3, seed=130)
    w = _ints((Cout, Cin, 3, 3), -2, 3, seed=131)
    b = _ints((Cout, ), seed=132)
    ref = F.conv2d(x.double(), w.double(), b.double(), padding=1).float()
    y = _run_conv(cuda, _nhwc(x).to(cuda), _pack(w, cuda), Cout, H, H, 9, 1, 0, b.to(cuda), tile=tile,
                  split='fp16x2', ksplit=2)
    assert torch.equal(y.cpu(), _nhwc(ref))


@pytest.mark.parametrize('C1,C2', [(256, 512), (256, 64), (128, 32), (64, 0)])
def test_k32_small_segments_rowvec_residual(cuda, C1, C2):
    """ResBlock conv2 at 4 x 4 (the up path's 512-channel shortcut split over the block's two K groups),
    temb row vector, residual, pitched output (untouched beyond Cout); B = 6 leaves a partial last tile."""
    B, Cout, H = 6, 128, 4
    h = _ints((B, C1, H, H), seed=140)
    x = _ints((B, max(C2, 32), H, H), seed=141)
    w2 = _ints((Cout, C1, 3, 3), -2, 3, seed=142)
    ws = _ints((Cout, max(C2, 32), 1, 1), seed=143)
    b = _ints((Cout, ), seed=144)
    rv = _ints((B, Cout), seed=145)
    res = _ints((B, Cout, H, H), seed=146)
    K = 9 * C1 + C2
    wp = torch.zeros((Cout, K), device=cuda)
    _pack(w2, cuda, K, 0, wp)
    ref = F.conv2d(h.double(), w2.double(), b.double(), padding=1) + rv.double()[:, :, None, None] + res.double()
    if C2:
        _pack(ws, cuda, K, 9 * C1, wp)
        ref = ref + F.conv2d(x.double(), ws.double())
    y = _run_conv(cuda, _nhwc(h).to(cuda), wp, Cout, H, H, 9, bias=b.to(cuda), rowvec=rv.to(cuda),
                  res=_nhwc(res).to(cuda), x2=_nhwc(x).to(cuda) if C2 else None, Cin2=C2, y_pitch=160, tile=15,
                  split='fp16x2', ksplit=2)
    assert torch.equal(y[..., :Cout].cpu(), _nhwc(ref.float()))
    assert torch.isnan(y[..., Cout:]).all()


@pytest.mark.parametrize('B,Cin,Cout', [(16, 256, 256), (8, 512, 256)])
def test_k32_small_fp32_accuracy(cuda, B, Cin, Cout):
    """fused GroupNorm + SiLU, random data: within 2x of the fp32 MFMA kernel's error vs fp64 (as the split-K
    tiles it replaces)."""
    xd, wp, b, pro, ref = _rand_case(cuda, B, Cin, Cout, 4, 0, seed=95)
    errs = {}
    for name, split, tile, ks in (('fp32', False, 0, 0), ('k32s', 'fp16x2', 15, 2), ('splitk', 'fp16x2', 13, 2)):
        y = _run_conv(cuda, xd, wp, Cout, 4, 4, 9, 1, 0, b.to(cuda), pro=pro, split=split, tile=tile, ksplit=ks)
        errs[name] = (y.cpu().double() - _nhwc(ref)).abs().max().item()
    scale = ref.abs().max().item()
    assert errs['k32s'] < 2.0 * errs['fp32'] + 1e-7 * scale, errs
    assert errs['k32s'] < 4e-6 * scale, (errs, scale)


# ---- big-table 128 x 128 tiles (tile 17; automatic where the GroupNorm tables of two images exceed the
# 8 KB table: ADM's 8^2 / 16^2 levels with 1024-2048 input channels, formerly on conv_patch3)
@pytest.mark.parametrize('B,Cin,Cout,H,up', [(4, 256, 128, 8, 0), (3, 128, 64, 16, 0), (2, 128, 64, 8, 2)])
def test_k32_bigtab_equals_v1(cuda, B, Cin, Cout, H, up):
    """Same kernel, larger LDS table: bit-identical to the 128 x 128 tiles where those fit."""
    xd, wp, b, pro, ref = _rand_case(cuda, B, Cin, Cout, H, up, seed=97)
    Ho = ref.shape[-1]
    y17 = _run_conv(cuda, xd, wp, Cout, Ho, Ho, 9, 1, up, b.to(cuda), pro=pro, split='fp16x2', tile=17)
    y10 = _run_conv(cuda, xd, wp, Cout, Ho, Ho, 9, 1, up, b.to(cuda), pro=pro, split='fp16x2', tile=10)
    assert torch.equal(y17.cpu(), y10.cpu())


@pytest.mark.parametrize('B,Cin,Cout,H,up', [(4, 1024, 128, 8, 0), (2, 2048, 128, 8, 0), (2, 1536, 256, 16, 0),
                                             (2, 1024, 128, 8, 2)])
def test_k32_bigtab_fp32_accuracy(cuda, B, Cin, Cout, H, up):
    """fused GroupNorm + SiLU with up to 2048 input channels, random data: within 2x of the fp32 MFMA kernel's
    error vs fp64 (the plans pick tile 17 for these shapes at their nominal batch)."""
    xd, wp, b, pro, ref = _rand_case(cuda, B, Cin, Cout, H, up, seed=98)
    Ho = ref.shape[-1]
    errs = {}
    for name, split, tile in (('fp32', False, 0), ('big', 'fp16x2', 17)):
        y = _run_conv(cuda, xd, wp, Cout, Ho, Ho, 9, 1, up, b.to(cuda), pro=pro, split=split, tile=tile)
        errs[name] = (y.cpu().double() - _nhwc(ref)).abs().max().item()
    scale = ref.abs().max().item()
    assert errs['big'] < 2.0 * errs['fp32'] + 1e-7 * scale, errs
