"""Round-5 GPU tests.

* the Winograd F(2,3)-along-x 3x3 conv (conv_wino.hip; models/unet.py:13-27, the ResBlock convs): integer operands
  bit for bit against float64 (transforms, padding, tap rows, epilogue), random operands at fp32-class accuracy,
  the range flag; whole CIFAR / CFG-CIFAR / ADM forwards against the direct conv (DM_CONV_WINO=0) and the
  reference fixtures, with the launch log showing which kernels ran;
* the plan-resolved small-map variants: the 4- and 8-wave forms (conv_k32s_kernel) are both launched (launch log)
  and give the same bits.
"""
import pytest
import torch
import torch.nn.functional as F

import dmhip
from tests.test_gpu_conv_split import _rand_case
from tests.test_gpu_ops import _ints, _nhwc, _pack, _run_conv
from tests.test_gpu_parity import TOL, _model

pytestmark = pytest.mark.gpu

WINO = 21  # ConvDesc.tile: force the Winograd kernel


@pytest.mark.parametrize('B,Cin,Cout,H', [(1, 128, 128, 32), (2, 32, 128, 32), (3, 64, 256, 16), (2, 256, 128, 16),
                                          (1, 96, 384, 32), (5, 160, 128, 16), (1, 128, 128, 8), (3, 64, 256, 8),
                                          (4, 512, 256, 8)])
def test_wino_conv3x3_exact(cuda, B, Cin, Cout, H):
    """Integer operands: V = B^T d, U = G g (half-integers), their fp16 pieces and the fp32 sums are exact, so the
    Winograd conv equals the float64 conv bit for bit (zero padding at every map edge, all tap rows)."""
    x = _ints((B, Cin, H, H), -2, 3, seed=50)
    w = _ints((Cout, Cin, 3, 3), -2, 3, seed=51)
    b = _ints((Cout, ), seed=52)
    ref = F.conv2d(x.double(), w.double(), b.double(), padding=1).float()
    dmhip.launch_log(True)
    y = _run_conv(cuda, _nhwc(x).to(cuda), _pack(w, cuda), Cout, H, H, 9, 1, 0, b.to(cuda), tile=WINO,
                  split='fp16x2', wino=True)
    log = dmhip.launch_log_read()
    dmhip.launch_log(False)
    assert log == [f'conv_wino_kernel<{H},0,false>'], log
    assert torch.equal(y.cpu(), _nhwc(ref))


@pytest.mark.parametrize('H', [32, 16, 8])
def test_wino_rowvec_residual_pitch(cuda, H):
    """temb row vector, residual, pitched input and output (untouched beyond Cout), integer-exact."""
    B, Cin, Cout = 3, 64, 128
    x = _ints((B, Cin, H, H), seed=60)
    w = _ints((Cout, Cin, 3, 3), -2, 3, seed=61)
    b = _ints((Cout, ), seed=62)
    rv = _ints((B, Cout), seed=63)
    res = _ints((B, Cout, H, H), seed=64)
    ref = (F.conv2d(x.double(), w.double(), b.double(), padding=1) + rv.double()[:, :, None, None]
           + res.double()).float()
    xp = torch.full((B, H, H, 96), float('nan'), device=cuda)
    xp[..., :Cin] = _nhwc(x).to(cuda)
    y = _run_conv(cuda, xp[..., :Cin], _pack(w, cuda), Cout, H, H, 9, bias=b.to(cuda), rowvec=rv.to(cuda),
                  res=_nhwc(res).to(cuda), y_pitch=160, x_pitch=96, tile=WINO, split='fp16x2', wino=True)
    assert torch.equal(y[..., :Cout].cpu(), _nhwc(ref))
    assert torch.isnan(y[..., Cout:]).all()


@pytest.mark.parametrize('C1,C2,H,Cout,pro', [(64, 64, 32, 128, False), (128, 384, 32, 128, False), (96, 128, 16, 256, False),
                                              (32, 192, 16, 128, False), (64, 128, 32, 128, True), (256, 256, 8, 256, False),
                                              (128, 128, 8, 256, True)])
def test_wino_shortcut_segment_exact(cuda, C1, C2, H, Cout, pro):
    """ResBlock conv2: 3x3 over h plus the 1x1 shortcut of x as a second K segment (nu 0 / 3: the pair's pixels,
    nu 1 / 2: their sum and difference against half the weights), temb row vector, residual -- integer-exact (with the
    GroupNorm affine prologue of integer tables and no SiLU: exact too)."""
    B = 2
    h = _ints((B, C1, H, H), seed=70)
    x = _ints((B, C2, H, H), seed=71)
    w2 = _ints((Cout, C1, 3, 3), -2, 3, seed=72)
    ws = _ints((Cout, C2, 1, 1), seed=73)
    b = _ints((Cout, ), seed=74)
    rv = _ints((B, Cout), seed=75)
    res = _ints((B, Cout, H, H), seed=76)
    K = 9 * C1 + C2
    wp = torch.zeros((Cout, K), device=cuda)
    _pack(w2, cuda, K, 0, wp)
    _pack(ws, cuda, K, 9 * C1, wp)
    hin = h
    prot = None
    if pro:  # integer GroupNorm-affine tables (scale 2, shift -1), no SiLU: exact
        sc = torch.full((B, C1), 2.0)
        sh = torch.full((B, C1), -1.0)
        hin = h * 2 - 1
        prot = (sc.to(cuda), sh.to(cuda))
    ref = (F.conv2d(hin.double(), w2.double(), b.double(), padding=1) + rv.double()[:, :, None, None]
           + F.conv2d(x.double(), ws.double()) + res.double()).float()
    dmhip.launch_log(True)
    y = _run_conv(cuda, _nhwc(h).to(cuda), wp, Cout, H, H, 9, bias=b.to(cuda), rowvec=rv.to(cuda),
                  res=_nhwc(res).to(cuda), x2=_nhwc(x).to(cuda), Cin2=C2, tile=WINO, split='fp16x2', wino=True,
                  pro=prot, pro_nosilu=1 if pro else 0)
    log = dmhip.launch_log_read()
    dmhip.launch_log(False)
    assert log == [f'conv_wino_kernel<{H},{1 if pro else 0},true>'], log
    assert torch.equal(y.cpu(), _nhwc(ref))


@pytest.mark.parametrize('B,C1,C2,Cout,H', [(4, 128, 384, 128, 32), (8, 256, 128, 256, 16)])
def test_wino_shortcut_fp32_accuracy(cuda, report, B, C1, C2, Cout, H):
    """GroupNorm + SiLU conv2 with the shortcut segment (the SiLU fold in its weights) on random data: within 3x the
    fp32 MFMA kernel's error vs float64."""
    xd, wp3, b, pro, ref3 = _rand_case(cuda, B, C1, Cout, H, 0, seed=93)
    g = torch.Generator().manual_seed(94)
    x2 = torch.randn((B, C2, H, H), generator=g)
    ws = torch.randn((Cout, C2, 1, 1), generator=g) * (1.0 / C2 ** 0.5)
    K = 9 * C1 + C2
    wp = torch.zeros((Cout, K), device=cuda)
    wp[:, :9 * C1] = wp3
    _pack(ws, cuda, K, 9 * C1, wp)
    ref = ref3 + F.conv2d(x2.double(), ws.double())
    errs = {}
    for name, split, tile, wino in (('fp32', False, 0, False), ('wino', 'fp16x2', WINO, True)):
        y = _run_conv(cuda, xd, wp, Cout, H, H, 9, 1, 0, b.to(cuda), pro=pro, split=split, tile=tile, wino=wino,
                      x2=_nhwc(x2).to(cuda), Cin2=C2)
        errs[name] = (y.cpu().double() - _nhwc(ref)).abs().max().item()
    scale = ref.abs().max().item()
    report(f'wino_shortcut_accuracy_{B}_{C1}_{C2}_{H}_max_rel', errs['wino'] / scale)
    assert errs['wino'] < 3.0 * errs['fp32'] + 1e-7 * scale, errs


@pytest.mark.parametrize('B,Cin,Cout,H', [(4, 128, 128, 32), (8, 256, 256, 16), (2, 384, 128, 32), (4, 512, 256, 16),
                                          (8, 256, 256, 8), (5, 512, 256, 8)])
def test_wino_fp32_accuracy(cuda, report, B, Cin, Cout, H):
    """Fused GroupNorm + SiLU conv on random data: the Winograd kernel's error vs float64 is at most the fp32 MFMA
    kernel's (measured 0.28-0.47x max, 0.44-0.47x rms over these shapes) and its rms at most the direct fp16x2
    kernel's (measured 0.65-0.76x): U and V are exact or one rounding, so fewer products means less error (VERDICT r5:
    the earlier 3x bound would have let a tripled error pass)."""
    xd, wp, b, pro, ref = _rand_case(cuda, B, Cin, Cout, H, 0, seed=91)
    errs, rms = {}, {}
    for name, split, tile, wino in (('fp32', False, 0, False), ('k32', 'fp16x2', 10, False),
                                    ('wino', 'fp16x2', WINO, True)):
        y = _run_conv(cuda, xd, wp, Cout, H, H, 9, 1, 0, b.to(cuda), pro=pro, split=split, tile=tile, wino=wino)
        d = y.cpu().double() - _nhwc(ref)
        errs[name] = d.abs().max().item()
        rms[name] = d.pow(2).mean().sqrt().item()
    scale = ref.abs().max().item()
    for k in errs:
        report(f'wino_accuracy_{B}_{Cin}_{Cout}_{H}_{k}_max_rel', errs[k] / scale)
        report(f'wino_accuracy_{B}_{Cin}_{Cout}_{H}_{k}_rms_rel', rms[k] / scale)
    assert errs['wino'] <= 1.0 * errs['fp32'], errs
    assert rms['wino'] <= 1.0 * rms['fp32'], rms
    assert rms['wino'] <= 1.0 * rms['k32'], rms
    assert errs['wino'] < 6e-6 * scale, (errs, scale)


def test_wino_range_flag(cuda):
    """A transformed activation beyond 65504 (no fp16 image) raises the range flag; in range it stays clear."""
    B, C, H = 2, 64, 16
    g = torch.Generator().manual_seed(7)
    x = torch.randn((B, C, H, H), generator=g)
    w = torch.randn((128, C, 3, 3), generator=g) * 0.05
    for big, expect in ((1.0, 0), (1e5, 1)):
        flag = torch.zeros(1, dtype=torch.int32, device=cuda)
        _run_conv(cuda, _nhwc(x * big).to(cuda), _pack(w, cuda), 128, H, H, 9, tile=WINO, split='fp16x2',
                  wino=True, range_flag=flag)
        assert int(flag.item()) == expect


def _forward_logged(meta, name, cuda, x, t, y=None):
    dmhip.launch_log(True)
    model, _ = _model(meta, name, cuda)
    out = model(x, t) if y is None else model(x, t, y)
    log = dmhip.launch_log_read()
    dmhip.launch_log(False)
    return model, out, log


@pytest.mark.parametrize('B', [2, 5])
def test_wino_cifar_forward(cuda, golden, monkeypatch, report, B):
    """The CIFAR-10 UNet with its 32^2 / 16^2 / 8^2 ResBlock convs (no shortcut segment) on the Winograd kernel: within
    1e-5 of the direct-conv forward (DM_CONV_WINO=0) and within TOL of the reference fixture; the launch log holds
    the Winograd launches and the direct forward none."""
    g, meta = golden('forward')
    xg = torch.Generator().manual_seed(41)
    x = torch.randn((B, 3, 32, 32), generator=xg).to(cuda)
    t = torch.randint(0, 1000, (B, ), generator=xg).to(cuda)
    model_w, out_w, log_w = _forward_logged(meta, 'cifar10', cuda, x, t)
    # no range fallback (a non-finite Winograd output raises the flag and the forward re-runs in bf16x3, which would
    # hide it from the comparison below)
    assert dmhip.range_stats(model_w.native_handle(cuda))[0] == 0
    monkeypatch.setenv('DM_CONV_WINO', '0')
    _, out_d, log_d = _forward_logged(meta, 'cifar10', cuda, x, t)
    n32 = sum(log_w.count(f'conv_wino_kernel<32,2,{sc}>') for sc in ('false', 'true'))
    n16 = sum(log_w.count(f'conv_wino_kernel<16,2,{sc}>') for sc in ('false', 'true'))
    n8 = sum(log_w.count(f'conv_wino_kernel<8,2,{sc}>') for sc in ('false', 'true'))
    n4 = sum(log_w.count(f'conv_wino_kernel<4,2,{sc}>') for sc in ('false', 'true'))
    # every 3x3 ResBlock conv of the 32^2 / 16^2 / 8^2 levels, shortcuts included; at 4^2 the up path's three
    # 512-channel conv1s (split-K, round 6: >= 12 K steps per split), the other eleven on conv_k32s
    assert n32 == 10 and n16 == 10 and n8 == 10 and n4 == 3, log_w
    assert sum(s.startswith('conv_k32s_kernel') for s in log_w) == 11, log_w
    assert not any(s.startswith('conv_wino') for s in log_d), log_d
    err = (out_w - out_d).abs().max().item()
    report(f'wino_cifar_forward_B{B}_vs_direct', err)
    assert err <= 1e-5, err
    monkeypatch.delenv('DM_CONV_WINO')
    model, _ = _model(meta, 'cifar10', cuda)
    xr = torch.from_numpy(g['cifar10_x']).to(cuda)
    tr = torch.from_numpy(g['cifar10_t']).to(cuda)
    err_ref = (model(xr, tr).cpu() - torch.from_numpy(g['cifar10_y'])).abs().max().item()
    report('wino_cifar_vs_reference', err_ref)
    assert err_ref <= TOL, err_ref


def test_small_map_variants_both_launched_bit_identical(cuda, golden, monkeypatch):
    """The 4x4-level convs on the direct kernels (DM_CONV_WINO=0; the default takes the split-K Winograd kernel since
    round 6): DM_K32S_W4=1 resolves the 4-wave conv_k32s_kernel at plan build (variant 12) and the default the 8-wave
    one (variant 6) -- the launch log proves each ran -- with the same bits."""
    _, meta = golden('forward')
    monkeypatch.setenv('DM_CONV_WINO', '0')
    xg = torch.Generator().manual_seed(33)
    x = torch.randn((5, 3, 32, 32), generator=xg).to(cuda)
    t = torch.randint(0, 1000, (5, ), generator=xg).to(cuda)
    outs, logs = {}, {}
    for w4 in ('0', '1'):
        monkeypatch.setenv('DM_K32S_W4', w4)
        _, outs[w4], logs[w4] = _forward_logged(meta, 'cifar10', cuda, x, t)
    k8 = [s for s in logs['0'] if s.startswith('conv_k32s_kernel<')]
    k4 = [s for s in logs['1'] if s.startswith('conv_k32s_kernel<')]
    assert k8 and all(s.endswith(',8>') for s in k8), logs['0']
    assert k4 and all(s.endswith(',4>') for s in k4), logs['1']
    assert len(k4) == len(k8)
    assert torch.equal(outs['0'], outs['1'])


def test_linear_split_k_tail(cuda, monkeypatch, report):
    """linear_k32's split-K tail (DiT-S/2 at B = 16: the N = 384 proj / fc2 GEMMs have 96 tiles, a tail of less
    than half a round on 512 resident blocks, split 2 ways over K, one block per CU): the launch log shows it with the default and
    not with DM_LIN_SK=0; two forwards are bit-identical (the slabs are summed in slice order whichever block
    arrives last); the re-associated sums stay within 1e-5 (relative to the output's max) of the whole-K tiles."""
    from models.dit.model import DiT_models
    from utils.synthetic import init_synthetic_
    ref = DiT_models['DiT-S/2'](input_size=32, num_classes=1000, learn_sigma=True).eval()
    init_synthetic_(ref)
    sd = ref.state_dict()
    g = torch.Generator().manual_seed(17)
    B = 16
    x = torch.randn((B, 4, 32, 32), generator=g).to(cuda)
    t = torch.randint(0, 1000, (B, ), generator=g).to(cuda)
    y = torch.randint(0, 1000, (B, ), generator=g).to(cuda)

    def run(sk):
        monkeypatch.setenv('DM_LIN_SK', sk)
        dmhip.launch_log(True)
        m = DiT_models['DiT-S/2'](input_size=32, num_classes=1000, learn_sigma=True).eval()
        m.load_state_dict(sd)
        m = m.to(cuda)
        with torch.no_grad():
            a = m(x, t, y).cpu()
            b = m(x, t, y).cpu()
        log = dmhip.launch_log_read()
        dmhip.launch_log(False)
        return a, b, log

    on_a, on_b, log_on = run('1')
    off_a, off_b, log_off = run('0')
    assert 'linear_k32_sk' in log_on, log_on
    assert 'linear_k32_sk' not in log_off, log_off
    assert torch.isfinite(on_a).all()
    assert torch.equal(on_a, on_b)
    assert torch.equal(off_a, off_b)
    rel = ((on_a - off_a).abs().max() / off_a.abs().max()).item()
    report('linear_split_k_tail_dit_s2_rel_vs_whole_k', rel)
    assert rel <= 1e-5, rel


def _linear_k32(A, W, bias=None, res=None, sc=None, sh=None, rows=0, ea=0, presplit=0, sk=1):
    """dm_debug_linear_k32: one linear_k32 launch (weights split in the hook), with or without the split-K tail's
    workspace."""
    import ctypes
    from dmhip import _lib
    L = _lib.load()
    f = L.dm_debug_linear_k32
    f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                  ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    M, K = A.shape
    N = W.shape[0]
    C = torch.full((M, N), float('nan'), device=A.device)
    p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    _lib.check(f(p(A), K, p(W), p(bias), p(res), N, p(sc), p(sh), rows, p(C), N, M, N, K, ea, presplit, sk,
                 torch.cuda.current_stream().cuda_stream), 'dm_debug_linear_k32')
    return C


def _sk_split(M, N, K):
    """dm_debug_linear_k32_split: the split-K ways linear_k32 picks for this shape on this device (its CU count and
    resident blocks decide the tail), with the device's slots and CUs."""
    import ctypes
    from dmhip import _lib
    S, P, cus = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    _lib.check(_lib.load().dm_debug_linear_k32_split(M, N, K, ctypes.byref(S), ctypes.byref(P), ctypes.byref(cus)),
               'dm_debug_linear_k32_split')
    return S.value, P.value, cus.value


# (M, N, K) on MI355X (256 CUs, 512 resident blocks): tile counts 64 (tail 64: 4 slices; partial M and N tiles, 9 K
# stages split 3/2/2/2), 1152 (the DiT-XL/2 proj shape: tail 128, 2 slices), 96 (K = 128: 2 stages, 2 slices), 600
# (tail 88: 2 slices of 9); on another CU count the tails differ and the test takes the device's own decision
SK_SHAPES = [(1000, 996, 576), (16384, 1152, 1152), (4096, 384, 128), (7680, 1280, 1152)]


@pytest.mark.parametrize('M,N,K', SK_SHAPES)
@pytest.mark.parametrize('form', ['fp32', 'presplit', 'groupnorm'])
def test_linear_k32_split_k_tail_vs_fp64(cuda, report, M, N, K, form):
    """linear_k32 with the split-K tail (write-through slabs, arrival ticket, slice-order reduce) against the whole-K
    tiles and a float64 reference, across the A forms (in-GEMM split, pre-split A, GroupNorm prologue), with bias and
    residual epilogues and partial tiles: the split launch agrees with the whole-K one to fp32 re-association
    (<= 2e-6 of the output's max) and both meet the fp16x2 bound against float64; two split launches are
    bit-identical (the reducer sums in slice order whichever block arrives last)."""
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn((M, K), generator=g).to(cuda)
    W = (torch.randn((N, K), generator=g) / K ** 0.5).to(cuda)
    bias = torch.randn((N, ), generator=g).to(cuda)
    res = torch.randn((M, N), generator=g).to(cuda)
    kw = dict(bias=bias, res=res, ea=4)
    Ar = A.double()
    if form == 'presplit':
        kw['presplit'] = 1
    if form == 'groupnorm':
        rows = 128 if M % 128 == 0 else M
        imgs = (M + rows - 1) // rows
        sc = (torch.rand((imgs, K), generator=g) + 0.5).to(cuda)
        sh = (torch.rand((imgs, K), generator=g) - 0.5).to(cuda)
        kw.update(sc=sc, sh=sh, rows=rows)
        idx = torch.arange(M, device=cuda) // rows
        Ar = (A * sc[idx] + sh[idx]).double()  # (the kernel's fp32 mul + add, then the split)
    ref = Ar @ W.double().t() + bias.double() + res.double()
    dmhip.launch_log(True)
    whole = _linear_k32(A, W, sk=0, **kw)
    assert 'linear_k32_sk' not in dmhip.launch_log_read()
    split1 = _linear_k32(A, W, sk=1, **kw)
    S, slots, cus = _sk_split(M, N, K)
    if cus == 256 and slots == 512:  # MI355X: every one of these shapes has a tail to split
        assert S > 1, (M, N, K, S)
    assert dmhip.launch_log_read().count('linear_k32_sk') == int(S > 1), (S, slots, cus)
    dmhip.launch_log(False)
    split2 = _linear_k32(A, W, sk=1, **kw)
    assert torch.isfinite(split1).all()
    assert torch.equal(split1, split2)
    scale = ref.abs().max().item()
    rel_sk = (split1.double() - whole.double()).abs().max().item() / scale
    rel_ref = max((split1.double() - ref).abs().max().item(), (whole.double() - ref).abs().max().item()) / scale
    report(f'linear_k32_sk_{form}_{M}x{N}x{K}_rel_vs_whole_k', rel_sk)
    report(f'linear_k32_sk_{form}_{M}x{N}x{K}_rel_vs_fp64', rel_ref)
    assert rel_sk <= 2e-6, rel_sk
    assert rel_ref <= 2e-6, rel_ref


def test_linear_split_k_tail_plan_cache(cuda):
    """The split-K tail's arrival counters are shared by a DiT model's cached plans (one workspace per model, the
    reducing block resets its tile's counter): alternating batch sizes (plans built, captured and replayed in turn)
    gives the same bits for the same batch every time."""
    from models.dit.model import DiT_models
    from utils.synthetic import init_synthetic_
    m = DiT_models['DiT-S/2'](input_size=32, num_classes=1000, learn_sigma=True).eval()
    init_synthetic_(m)
    m = m.to(cuda)
    g = torch.Generator().manual_seed(23)
    xs = {B: (torch.randn((B, 4, 32, 32), generator=g).to(cuda), torch.randint(0, 1000, (B, ), generator=g).to(cuda),
              torch.randint(0, 1000, (B, ), generator=g).to(cuda)) for B in (16, 3, 24)}
    first = {}
    with torch.no_grad():
        for B in (16, 3, 24, 16, 24, 3, 16):
            out = m(*xs[B]).cpu()
            assert torch.isfinite(out).all()
            if B in first:
                assert torch.equal(out, first[B]), B
            else:
                first[B] = out
