"""Operator-level parity of the HIP kernels (called through the C ABI) against
torch CPU references. Integer-valued operands make contractions exact in fp32,
so the MFMA layout / indexing tests compare bit-for-bit."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import dmhip

pytestmark = pytest.mark.gpu


def _ints(shape, lo=-3, hi=4, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(lo, hi, shape, generator=g).float()


def _gemm_desc(**kw):
    d = dmhip.GemmDesc()
    d.Z1 = d.Z2 = 1
    d.alpha = 1.0
    for k, v in kw.items():
        setattr(d, k, v)
    return d


SPLITS = [dict(), dict(split=2, split_ea=3, split_eb=-2)]  # fp32 MFMA; fp16x2 with power-of-two scales


@pytest.mark.parametrize('sp', SPLITS)
@pytest.mark.parametrize('M,N,K', [(64, 64, 32), (200, 136, 72), (256, 768, 256), (1024, 512, 128), (33, 40, 4)])
def test_gemm_bt_exact(cuda, M, N, K, sp):
    A = _ints((M, K), seed=1)
    B = _ints((N, K), seed=2)
    bias = _ints((N, ), seed=3)
    C = torch.empty((M, N), device=cuda)
    Ad, Bd, bd = A.to(cuda), B.to(cuda), bias.to(cuda)
    d = _gemm_desc(M=M, N=N, K=K, A=Ad.data_ptr(), lda=K, B=Bd.data_ptr(), ldb=K, C=C.data_ptr(), ldc=N,
                   bias=bd.data_ptr(), **sp)
    dmhip.gemm(d, cuda)
    ref = (A.double() @ B.double().T + bias.double()).float()
    assert torch.equal(C.cpu(), ref)


@pytest.mark.parametrize('sp', SPLITS)
@pytest.mark.parametrize('M,N,K,Z1,Z2', [(256, 128, 256, 3, 2), (16, 64, 16, 4, 1), (100, 72, 100, 2, 3)])
def test_gemm_batched_kn_alpha(cuda, M, N, K, Z1, Z2, sp):
    A = _ints((Z1, Z2, M, K), seed=4)
    B = _ints((Z1, Z2, K, N), seed=5)
    C = torch.empty((Z1, Z2, M, N), device=cuda)
    Ad, Bd = A.to(cuda), B.to(cuda)
    d = _gemm_desc(M=M, N=N, K=K, Z1=Z1, Z2=Z2,
                   A=Ad.data_ptr(), a_s1=Z2 * M * K, a_s2=M * K, lda=K,
                   B=Bd.data_ptr(), b_s1=Z2 * K * N, b_s2=K * N, ldb=N, b_kn=1,
                   C=C.data_ptr(), c_s1=Z2 * M * N, c_s2=M * N, ldc=N, alpha=0.5, **sp)
    dmhip.gemm(d, cuda)
    ref = ((A.double() * 0.5) @ B.double()).float()
    assert torch.equal(C.cpu(), ref)


@pytest.mark.parametrize('case', ['qk', 'pv', 'xw'])
def test_gemm_split_fp32_accuracy(cuda, case):
    """fp16x2 GEMM with the plan's exponents (unet_exec.hip split_gemm) on the attention operand
    distributions: error vs fp64 within 2x the fp32 MFMA kernel's (+ 1e-7 relative)."""
    g = torch.Generator().manual_seed(7)
    Z, M, N, K = 4, 256, 256, 256
    if case == 'qk':  # S = (q * d^-1/2) k^T
        A, B, kn, ea, eb, alpha = torch.randn((Z, M, K), generator=g), torch.randn((Z, N, K), generator=g), 0, 6, 6, K ** -0.5
    elif case == 'pv':  # O = softmax(S) v, v stored [k][n]
        A = torch.softmax(torch.randn((Z, M, K), generator=g) * 3, -1)
        B, kn, ea, eb, alpha = torch.randn((Z, K, N), generator=g), 1, 14, 6, 1.0
    else:  # x W^T with a U(+-1/sqrt(K)) weight
        A = torch.randn((Z, M, K), generator=g)
        B = (torch.rand((Z, N, K), generator=g) * 2 - 1) * K ** -0.5
        kn, ea, alpha = 0, 6, 1.0
        eb = 14 - int(torch.frexp(B.abs().max()).exponent)
    ref = (A.double() * alpha) @ (B.double() if kn else B.double().transpose(1, 2))
    errs = []
    for sp in (dict(), dict(split=2, split_ea=ea, split_eb=eb)):
        C = torch.empty((Z, M, N), device=cuda)
        Ad, Bd = A.contiguous().to(cuda), B.contiguous().to(cuda)
        d = _gemm_desc(M=M, N=N, K=K, Z1=Z, A=Ad.data_ptr(), a_s1=M * K, lda=K, B=Bd.data_ptr(), b_s1=K * N,
                       ldb=N if kn else K, b_kn=kn, C=C.data_ptr(), c_s1=M * N, ldc=N, alpha=alpha, **sp)
        dmhip.gemm(d, cuda)
        errs.append((C.cpu().double() - ref).abs().max().item())
    assert errs[1] < 2.0 * errs[0] + 1e-7 * ref.abs().max().item(), errs


def test_gemm_split_range_flag(cuda):
    """a scaled operand beyond 65504 raises the range flag; within range it stays clear."""
    for big, flagged in ((1000.0, False), (1100.0, True)):  # x 2^6 -> 64000 / 70400
        A = torch.randn((64, 32))
        A[5, 7] = big
        B = torch.randn((64, 32))
        C = torch.empty((64, 64), device=cuda)
        flag = torch.zeros(1, dtype=torch.int32, device=cuda)
        Ad, Bd = A.to(cuda), B.to(cuda)
        d = _gemm_desc(M=64, N=64, K=32, A=Ad.data_ptr(), lda=32, B=Bd.data_ptr(), ldb=32, C=C.data_ptr(), ldc=64,
                       split=2, split_ea=6, split_eb=0, range_flag=flag.data_ptr())
        dmhip.gemm(d, cuda)
        assert bool(flag.item()) == flagged


def test_gemm_silu_residual(cuda):
    M, N, K = 130, 96, 64
    g = torch.Generator().manual_seed(9)
    A, B = torch.randn((M, K), generator=g), torch.randn((N, K), generator=g)
    bias, res = torch.randn(N, generator=g), torch.randn((M, N), generator=g)
    C = torch.empty((M, N), device=cuda)
    Ad, Bd, bd, rd = A.to(cuda), B.to(cuda), bias.to(cuda), res.to(cuda)
    d = _gemm_desc(M=M, N=N, K=K, A=Ad.data_ptr(), lda=K, B=Bd.data_ptr(), ldb=K, C=C.data_ptr(), ldc=N,
                   bias=bd.data_ptr(), res=rd.data_ptr(), ld_res=N, act=1)
    dmhip.gemm(d, cuda)
    ref = F.silu((A.double() @ B.double().T + bias.double()) + res.double())
    assert (C.cpu().double() - ref).abs().max().item() < 1e-5


def _pack(w, cuda, K=None, col0=0, out=None):
    Cout, Cin, kh, kw = w.shape
    K = K or kh * kw * Cin
    if out is None:
        out = torch.zeros((Cout, K), device=cuda)
    dmhip.pack_conv_weight(w.to(cuda).contiguous(), out, K, col0)
    return out


def _run_conv(cuda, x_nhwc, w_packed, Cout, Hout, Wout, taps, stride=1, upsample=0, bias=None, rowvec=None,
              res=None, x2=None, Cin2=0, y_pitch=None, x_pitch=None, tile=0, pro=None, split=False,
              range_flag=None, pro_nosilu=0, ksplit=0, wino=False):
    B, Hin, Win, Cin = x_nhwc.shape[0], x_nhwc.shape[1], x_nhwc.shape[2], x_nhwc.shape[3]
    x_pitch = x_pitch or Cin
    y_pitch = y_pitch or Cout
    y = torch.full((B, Hout, Wout, y_pitch), float('nan'), device=cuda)
    d = dmhip.ConvDesc()
    d.x, d.x_pitch, d.Cin, d.Hin, d.Win = x_nhwc.data_ptr(), x_pitch, Cin, Hin, Win
    d.taps, d.stride, d.upsample = taps, stride, upsample
    d.x2, d.x2_pitch, d.Cin2 = (x2.data_ptr() if x2 is not None else None), (x2.shape[-1] if x2 is not None else 0), Cin2
    d.w, d.K = w_packed.data_ptr(), w_packed.shape[1]
    d.y, d.y_pitch, d.Cout, d.B, d.Hout, d.Wout = y.data_ptr(), y_pitch, Cout, B, Hout, Wout
    d.bias = bias.data_ptr() if bias is not None else None
    d.rowvec = rowvec.data_ptr() if rowvec is not None else None
    d.rowvec_pitch = rowvec.shape[1] if rowvec is not None else 0
    d.res = res.data_ptr() if res is not None else None
    d.res_pitch = res.shape[-1] if res is not None else 0
    d.tile = tile
    if pro is not None:
        d.pro_scale, d.pro_shift = pro[0].data_ptr(), pro[1].data_ptr()
        d.pro_nosilu = pro_nosilu
    if split:  # split weights (True = 'bf16x3', or 'fp16x2'): halo-patch shapes run conv_patch3_kernel
        kind = dmhip.SPLIT_FP16X2 if split == 'fp16x2' else dmhip.SPLIT_BF16X3
        nmat, ntap = (4, 4) if upsample == 2 else (1, taps)
        ws = dmhip.pack_conv_weight_split(w_packed, nmat, Cin, ntap, kind)
        d.w_split, d.w_split_kind = ws.data_ptr(), kind
        if range_flag is not None:
            d.range_flag = range_flag.data_ptr()
    if wino:  # Winograd F(2,3) weights (conv_wino.hip; with fp16x2 split weights)
        fold = pro is not None and not pro_nosilu
        ww = dmhip.pack_conv_weight_wino(w_packed, Cin, Cin2, fold)
        d.w_wino, d.w_wino_fold = ww.data_ptr(), int(fold)
    if ksplit > 1:  # split-K partial sums [ksplit][B * Hout * Wout][Cout]
        kpart = torch.empty((ksplit, B * Hout * Wout, Cout), device=cuda)
        d.ksplit, d.kpart = ksplit, kpart.data_ptr()
    dmhip.conv2d_nhwc(d, cuda)
    if wino:
        torch.cuda.synchronize(cuda)  # ww is freed on return
    return y


def _nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


@pytest.mark.parametrize('tile', [0, 1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize('B,Cin,Cout,H,stride,up', [
    (2, 32, 64, 8, 1, 0), (3, 64, 32, 16, 2, 0), (2, 32, 32, 4, 1, 1), (1, 128, 256, 16, 1, 0),
    (5, 64, 64, 4, 1, 0), (2, 96, 160, 8, 2, 0), (3, 32, 96, 5, 1, 0), (2, 64, 64, 7, 2, 0),
    (4, 64, 128, 32, 1, 0), (3, 64, 64, 16, 1, 1), (2, 32, 64, 8, 1, 1), (3, 32, 32, 2, 1, 1),
])
def test_conv3x3_exact(cuda, B, Cin, Cout, H, stride, up, tile):
    x = _ints((B, Cin, H, H), -2, 3, seed=10)
    w = _ints((Cout, Cin, 3, 3), -2, 3, seed=11)
    b = _ints((Cout, ), seed=12)
    xin = F.interpolate(x, scale_factor=2, mode='nearest') if up else x
    ref = F.conv2d(xin.double(), w.double(), b.double(), stride=stride, padding=1).float()
    Hout = ref.shape[-1]
    y = _run_conv(cuda, _nhwc(x).to(cuda), _pack(w, cuda), Cout, Hout, Hout, 9, stride, up, b.to(cuda), tile=tile)
    assert torch.equal(y.cpu(), _nhwc(ref))


@pytest.mark.parametrize('tile', [0, 1, 2, 3, 4, 5, 6])
def test_conv_segments_rowvec_residual_pitch(cuda, tile):
    # ResBlock second conv with the shortcut folded in as a 1x1 K segment, temb rowvec, pitched output
    B, C1, C2, Cout, H = 3, 64, 32, 64, 8
    h = _ints((B, C1, H, H), seed=20)
    x = _ints((B, C2, H, H), seed=21)
    w2 = _ints((Cout, C1, 3, 3), -2, 3, seed=22)
    ws = _ints((Cout, C2, 1, 1), seed=23)
    b = _ints((Cout, ), seed=24)
    rv = _ints((B, Cout), seed=25)
    K = 9 * C1 + C2
    wp = torch.zeros((Cout, K), device=cuda)
    _pack(w2, cuda, K, 0, wp)
    _pack(ws, cuda, K, 9 * C1, wp)
    ref = (F.conv2d(h.double(), w2.double(), b.double(), padding=1) + rv.double()[:, :, None, None]
           + F.conv2d(x.double(), ws.double())).float()
    y = _run_conv(cuda, _nhwc(h).to(cuda), wp, Cout, H, H, 9, bias=b.to(cuda), rowvec=rv.to(cuda),
                  x2=_nhwc(x).to(cuda), Cin2=C2, y_pitch=96, tile=tile)
    assert torch.equal(y[..., :Cout].cpu(), _nhwc(ref))
    assert torch.isnan(y[..., Cout:]).all()  # channels outside the view untouched


def test_conv1x1_residual(cuda):
    B, C, H = 2, 64, 8
    x = _ints((B, C, H, H), seed=30)
    w = _ints((C, C, 1, 1), seed=31)
    r = _ints((B, C, H, H), seed=32)
    ref = (F.conv2d(x.double(), w.double()) + r.double()).float()
    y = _run_conv(cuda, _nhwc(x).to(cuda), _pack(w, cuda), C, H, H, 1, res=_nhwc(r).to(cuda))
    assert torch.equal(y.cpu(), _nhwc(ref))


@pytest.mark.parametrize('B,C,HW,silu,mod', [(2, 128, 1024, True, False), (3, 384, 256, True, False),
                                              (2, 256, 16, False, False), (2, 64, 64, True, True),
                                              (1, 192, 100, True, False)])
def test_groupnorm(cuda, B, C, HW, silu, mod):
    g = torch.Generator().manual_seed(40)
    x = torch.randn((B, C, HW), generator=g) * 3 + 0.5
    gamma, beta = torch.randn(C, generator=g), torch.randn(C, generator=g)
    ms, mb = torch.randn((B, C), generator=g), torch.randn((B, C), generator=g)
    ref = F.group_norm(x.double(), 32, gamma.double(), beta.double(), 1e-5)
    if mod:
        ref = ref * (1 + ms.double()[:, :, None]) + mb.double()[:, :, None]
    if silu:
        ref = F.silu(ref)
    xn = x.permute(0, 2, 1).contiguous().to(cuda)
    y = torch.empty_like(xn)
    dmhip.groupnorm_nhwc(xn, y, B, HW, C, 32, 1e-5, gamma.to(cuda), beta.to(cuda),
                         ms.to(cuda) if mod else None, mb.to(cuda) if mod else None, C if mod else 0, silu)
    err = (y.cpu().double() - ref.permute(0, 2, 1)).abs().max().item()
    assert err < 2e-5, err


def test_softmax_rows(cuda):
    g = torch.Generator().manual_seed(50)
    for L in (16, 256, 500, 512, 1024, 1000):
        x = torch.randn((37, L), generator=g) * 5
        xd = x.to(cuda)
        dmhip.softmax_rows(xd, 37, L, L)
        assert (xd.cpu() - x.softmax(-1)).abs().max().item() < 1e-6


def test_timestep_embedding(cuda):
    import math
    import oracle.unet as ou
    t = torch.tensor([0, 1, 17, 500, 999])
    ref = ou.sinusoidal(t, 128)
    out = torch.empty((5, 128), device=cuda)
    # host-provided frequency table (as the UNet installs it): only sin/cos ulps differ
    freqs = torch.exp(torch.arange(64) * -(math.log(10000) / 63)).to(cuda)
    dmhip.timestep_embedding(t.to(cuda), 128, 0, out, freqs)
    assert (out.cpu() - ref).abs().max().item() < 1e-6
    # on-device frequencies: expf ulps are amplified by t up to 999 (args ~1e3 rad)
    dmhip.timestep_embedding(t.to(cuda), 128, 0, out)
    assert (out.cpu() - ref).abs().max().item() < 1e-4


@pytest.mark.parametrize('tile', [0, 4, 5, 6])
@pytest.mark.parametrize('B,Cin,Cout,H,up', [(2, 64, 64, 8, 0), (2, 96, 64, 16, 0), (3, 64, 32, 4, 0),
                                             (2, 64, 64, 8, 1)])
def test_conv_fused_groupnorm_silu(cuda, B, Cin, Cout, H, up, tile):
    """GroupNorm(32) + SiLU folded into the conv's patch load == group_norm -> silu -> conv (padding after SiLU)."""
    g = torch.Generator().manual_seed(60)
    x = torch.randn((B, Cin, H, H), generator=g) * 2 + 0.3
    gamma, beta = torch.randn(Cin, generator=g), torch.randn(Cin, generator=g)
    w = torch.randn((Cout, Cin, 3, 3), generator=g) * 0.05
    b = torch.randn(Cout, generator=g)
    a = F.silu(F.group_norm(x.double(), 32, gamma.double(), beta.double(), 1e-5))
    if up:
        a = F.interpolate(a, scale_factor=2, mode='nearest')
    ref = F.conv2d(a, w.double(), b.double(), padding=1)
    xd = _nhwc(x).to(cuda)
    pro = dmhip.groupnorm_affine(xd, B, H * H, Cin, 32, 1e-5, gamma.to(cuda), beta.to(cuda))
    Ho = ref.shape[-1]
    y = _run_conv(cuda, xd, _pack(w, cuda), Cout, Ho, Ho, 9, 1, up, b.to(cuda), tile=tile, pro=pro)
    err = (y.cpu().double() - _nhwc(ref)).abs().max().item()
    assert err < 1e-4, err


def _pack_subpix(w, cuda):
    Cout, Cin = w.shape[:2]
    out = torch.zeros((4, Cout, 4 * Cin), device=cuda)
    dmhip.pack_conv_weight_subpixel(w.to(cuda).contiguous(), out)
    return out.view(4 * Cout, 4 * Cin)


@pytest.mark.parametrize('tile', [0, 4, 5, 6])
@pytest.mark.parametrize('B,Cin,Cout,H', [(2, 32, 32, 4), (3, 64, 64, 16), (2, 32, 64, 8), (3, 32, 32, 2),
                                          (4, 64, 128, 8), (2, 96, 64, 4)])
def test_conv_subpixel_upsample_exact(cuda, B, Cin, Cout, H, tile):
    """nearest-2x + 3x3 conv as four 4-tap sub-pixel convs (upsample = 2): integer operands keep the
    summed weights and every product exact, so the result equals the upsampled conv bit for bit."""
    x = _ints((B, Cin, H, H), -2, 3, seed=70)
    w = _ints((Cout, Cin, 3, 3), -2, 3, seed=71)
    b = _ints((Cout, ), seed=72)
    ref = F.conv2d(F.interpolate(x, scale_factor=2, mode='nearest').double(), w.double(), b.double(),
                   padding=1).float()
    wp = _pack_subpix(w, cuda)
    try:
        y = _run_conv(cuda, _nhwc(x).to(cuda), wp, Cout, 2 * H, 2 * H, 9, 1, 2, b.to(cuda), tile=tile)
    except ValueError as e:  # low-res shape without a whole-row tiling (the UNet plan then keeps the
        assert tile != 0 or H < 4, e  # nearest-2x conv); every shape >= 4x4 tiles automatically
        pytest.skip(str(e))
    assert torch.equal(y.cpu(), _nhwc(ref))


@pytest.mark.parametrize('B,Cin,Cout,H', [(2, 64, 64, 8), (3, 32, 64, 16), (2, 64, 32, 4)])
def test_conv_subpixel_fused_groupnorm_silu(cuda, B, Cin, Cout, H):
    g = torch.Generator().manual_seed(73)
    x = torch.randn((B, Cin, H, H), generator=g) * 2 + 0.3
    gamma, beta = torch.randn(Cin, generator=g), torch.randn(Cin, generator=g)
    w = torch.randn((Cout, Cin, 3, 3), generator=g) * 0.05
    b = torch.randn(Cout, generator=g)
    a = F.interpolate(F.silu(F.group_norm(x.double(), 32, gamma.double(), beta.double(), 1e-5)), scale_factor=2,
                      mode='nearest')
    ref = F.conv2d(a, w.double(), b.double(), padding=1)
    xd = _nhwc(x).to(cuda)
    pro = dmhip.groupnorm_affine(xd, B, H * H, Cin, 32, 1e-5, gamma.to(cuda), beta.to(cuda))
    y = _run_conv(cuda, xd, _pack_subpix(w, cuda), Cout, 2 * H, 2 * H, 9, 1, 2, b.to(cuda), pro=pro)
    err = (y.cpu().double() - _nhwc(ref)).abs().max().item()
    assert err < 1e-4, err
