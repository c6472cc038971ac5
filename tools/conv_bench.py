"""Microbenchmark of the dominant conv shapes of the CIFAR-10 UNet at B=256 through the C ABI.

    python tools/conv_bench.py [--iters 20] [--shape NAME]

Times each shape with HIP events over `iters` launches on one stream and prints
TFLOP/s against the 157.3 TF fp32 MFMA peak. Used for kernel tuning and as the
target of rocprofv3 PMC passes (tools/gpu_conv_pmc.sh).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'diffusion-models-pytorch_amd')]

import torch  # noqa: E402

import dmhip  # noqa: E402

# name: (B, Cin, Cout, H, pro, upsample)
SHAPES = {
    'res32_256': (256, 256, 256, 32, True, 0),     # up-path ResBlock conv2 at 32x32 (K = 2304)
    'res32_128': (256, 128, 128, 32, True, 0),     # down-path ResBlock at 32x32
    'res32_384': (256, 384, 128, 32, True, 0),     # up-path conv1 with concat input
    'res16_256': (256, 256, 256, 16, True, 0),
    'res8_256': (256, 256, 256, 8, True, 0),
    'res8_512': (256, 512, 256, 8, True, 0),       # up-path conv1 at 8x8 with concat input
    'adm8_1024': (64, 1024, 1024, 8, True, 0),    # ADM-256 8x8 level ResBlock conv (C4, B = 64)
    'adm8_2048': (64, 2048, 1024, 8, True, 0),    # ADM-256 8x8 up-path conv1 with concat input
    'adm16_2048': (64, 2048, 1024, 16, True, 0),  # ADM-256 16x16 up-path conv1 with concat input
    'res4_256': (256, 256, 256, 4, True, 0),
    'res4_512': (256, 512, 256, 4, True, 0),      # up-path conv1 at 4x4 with concat input
    'up16_256': (256, 256, 256, 16, False, 2),     # sub-pixel upsample 16 -> 32
    'up8_256': (256, 256, 256, 8, False, 2),       # sub-pixel upsample 8 -> 16
    'up4_256': (256, 256, 256, 4, False, 2),       # sub-pixel upsample 4 -> 8 (conv_patch3 MODE 2)
    'down8_256': (256, 256, 256, 8, True, -2),     # stride-2 downsample 8 -> 4 (conv_patch3 MODE 4)
    'qkv16': (256, 256, 768, 16, True, -1),        # attention qkv: 1x1 conv (GroupNorm prologue, no SiLU)
    'proj16': (256, 256, 256, 16, False, -1),      # attention proj: 1x1 conv
}


def run(name, iters, split, tile=0, ksplit=0):
    B, Cin, Cout, H, pro, up = SHAPES[name]
    dev = torch.device('cuda', 0)
    g = torch.Generator(device='cpu').manual_seed(0)
    x = torch.randn((B, H, H, Cin), generator=g).to(dev)
    stride = 1
    if up == -2:  # stride-2 downsample
        up, stride = 0, 2
    taps = 1 if up < 0 else 9
    w = (torch.randn((Cout, Cin, 3, 3) if taps == 9 else (Cout, Cin, 1, 1), generator=g) * 0.02).to(dev)
    if up < 0:  # 1x1 (only the split path runs it with the prologue)
        if not split:
            return
        wp = torch.zeros((Cout, Cin), device=dev)
        dmhip.pack_conv_weight(w, wp, Cin, 0)
        Ho, up = H, 0
    elif up == 2:
        wp = torch.zeros((4, Cout, 4 * Cin), device=dev)
        dmhip.pack_conv_weight_subpixel(w, wp)
        wp = wp.view(4 * Cout, 4 * Cin)
        Ho = 2 * H
    else:
        wp = torch.zeros((Cout, 9 * Cin), device=dev)
        dmhip.pack_conv_weight(w, wp, 9 * Cin, 0)
        Ho = H // stride
    b = torch.zeros(Cout, device=dev)
    y = torch.empty((B, Ho, Ho, Cout), device=dev)
    sc = torch.rand((B, Cin), device=dev) + 0.5
    sh = torch.rand((B, Cin), device=dev) - 0.5
    d = dmhip.ConvDesc()
    d.x, d.x_pitch, d.Cin, d.Hin, d.Win = x.data_ptr(), Cin, Cin, H, H
    d.taps, d.stride, d.upsample = taps, stride, up
    d.pro_nosilu = int(taps == 1)
    d.w, d.K = wp.data_ptr(), wp.shape[1]
    d.y, d.y_pitch, d.Cout, d.B, d.Hout, d.Wout = y.data_ptr(), Cout, Cout, B, Ho, Ho
    d.bias = b.data_ptr()
    d.tile = tile
    if pro:
        d.pro_scale, d.pro_shift = sc.data_ptr(), sh.data_ptr()
    if split:
        kind = dmhip.SPLIT_FP16X2 if split == 'fp16x2' else dmhip.SPLIT_BF16X3
        ws = dmhip.pack_conv_weight_split(wp, 4 if up == 2 else 1, Cin, 4 if up == 2 else taps, kind)
        d.w_split, d.w_split_kind = ws.data_ptr(), kind
    if tile == 21:  # the Winograd F(2,3) kernel (conv_wino.hip)
        ww = dmhip.pack_conv_weight_wino(wp, Cin)
        d.w_wino = ww.data_ptr()  # (no shortcut segment here: the fold does not apply)
    if ksplit > 1:
        kpart = torch.empty((ksplit, B * Ho * Ho, Cout), device=dev)
        d.ksplit, d.kpart = ksplit, kpart.data_ptr()
    try:
        for _ in range(3):
            dmhip.conv2d_nhwc(d, dev)
    except ValueError as e:  # a forced tile that does not take this shape
        print(f'{name:12s} t{tile}: n/a ({e})', flush=True)
        return
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        dmhip.conv2d_nhwc(d, dev)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    flops = 2.0 * B * Ho * Ho * Cout * wp.shape[1] * (1 if up != 2 else 1)
    if up == 2:
        flops = 2.0 * B * H * H * 4 * Cout * 4 * Cin  # executed sub-pixel work
    tf = flops / ms / 1e9
    tag = split or 'fp32'
    tag = f'{tag}/t{tile}' if tile else tag
    tag = f'{tag}/k{ksplit}' if ksplit > 1 else tag
    print(f'{name:12s} {tag:7s} {ms:8.4f} ms  {tf:6.1f} TF/s  {tf / 157.3 * 100:5.1f} % of fp32 peak', flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--shape', default=None)
    ap.add_argument('--math', choices=['fp32', 'bf16x3', 'fp16x2', 'all'], default='all')
    ap.add_argument('--tiles', default='0', help='comma-separated ConvDesc.tile values (0 = auto)')
    ap.add_argument('--ksplit', type=int, default=0, help='split-K (ConvDesc.ksplit; with a workspace)')
    args = ap.parse_args()
    dmhip.load()
    for name in ([args.shape] if args.shape else SHAPES):
        kinds = (False, 'bf16x3', 'fp16x2') if args.math == 'all' else ({'fp32': False}.get(args.math, args.math), )
        for split in kinds:
            for tile in [int(v) for v in args.tiles.split(',')]:
                run(name, args.iters, split, tile, args.ksplit)


if __name__ == '__main__':
    main()
