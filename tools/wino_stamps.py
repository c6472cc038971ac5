"""Phase timing of conv_wino_kernel from a diagnostic build (-DDM_K32_STAMPS): per block, wave 0's s_memtime at the
start, after the prologue, after the main loop and at the end, plus s_memrealtime start / end.

    make -C diffusion-models-pytorch_amd/csrc OUT=../../tools/bin/libdm_stamps.so BUILD=build_stamps \
        EXTRA=-DDM_K32_STAMPS
    DM_HIP_LIB=tools/bin/libdm_stamps.so python tools/wino_stamps.py --shape res32_128
"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import conv_bench  # noqa: E402

import dmhip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--shape', default='res32_128')
    args = ap.parse_args()
    dmhip.load()
    conv_bench.run(args.shape, 5, 'fp16x2', 21)
    B, Cin, Cout, H, pro, up = conv_bench.SHAPES[args.shape]
    imgs = 2 if H == 8 else 8 if H == 4 else 1  # images per 128-pixel tile (8 x 8 / 4 x 4 maps)
    groups = -(-B // imgs)
    tpi = (imgs * H * H // 128) * (Cout // 128)  # tiles per image group
    parts = next((p for p in range(1, tpi + 1) if tpi % p == 0 and groups * p >= 256), tpi)
    nblk = groups * parts
    buf = np.zeros((nblk, 16), dtype=np.uint64)
    L = dmhip.load()
    L.dm_debug_wino_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert L.dm_debug_wino_stamps(buf.ctypes.data, nblk) == 0
    s = buf.astype(np.int64)
    ntile = np.maximum(s[:, 4], 1)
    pro = s[:, 1] - s[:, 0]
    loop = s[:, 2]
    tot = s[:, 3] - s[:, 0]
    rest = tot - pro - loop
    rt0, rt1 = s[:, 5], s[:, 6]
    wall_us = (rt1.max() - rt0.min()) / 100.0
    clk = tot / np.maximum(rt1 - rt0, 1) * 100e6 / 1e9
    print(f'{args.shape} wino: {nblk} persistent blocks x {ntile.mean():.1f} tiles, Cin {Cin} ({Cin // 32} chunks), '
          f'kernel wall (stamps) {wall_us:.1f} us')
    for name, v in (('first prologue', pro), ('main loops', loop), ('epilogues + next prologues', rest),
                    ('  E writes + barrier', s[:, 8]), ('  outputs + GroupNorm', s[:, 9]), ('  next prologues', s[:, 10]),
                    ('block total', tot)):
        print(f'  {name:28s} cycles mean {v.mean():10.0f}  per tile {(v / ntile).mean():9.0f}  '
              f'share {v.mean() / tot.mean():.3f}')
    print(f'  main loop cycles per chunk {(loop / ntile).mean() / (Cin // 32):.0f} '
          f'(MFMA floor 4608 per SIMD: 2 waves x 144 x 16)')
    nck = ntile * (Cin // 32)
    for role, (a, b, c) in (('early (wave 0): finish | MFMAs | barrier', (11, 12, 13)),
                            ('late  (wave 4): MFMAs | finish | barrier', (14, 15, 7))):
        print(f'  {role}: per chunk {(s[:, a] / nck).mean():6.0f} | {(s[:, b] / nck).mean():6.0f} | '
              f'{(s[:, c] / nck).mean():6.0f}')
    print(f'  block wall us mean {((rt1 - rt0) / 100.0).mean():.2f}, clock GHz mean {clk.mean():.3f}')


if __name__ == '__main__':
    main()
