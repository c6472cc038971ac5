"""Phase timing of conv_k32_kernel from a diagnostic build (-DDM_K32_STAMPS): per block, wave 0's
s_memtime after the prologue, the main loop, segment 2 and the epilogue, plus s_memrealtime start/end.

    make -C diffusion-models-pytorch_amd/csrc OUT=../../tools/bin/libdm_stamps.so BUILD=build_stamps \
        EXTRA=-DDM_K32_STAMPS
    DM_HIP_LIB=tools/bin/libdm_stamps.so python tools/k32_stamps.py --shape res32_256 --tile 10
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
    ap.add_argument('--shape', default='res32_256')
    ap.add_argument('--tile', type=int, default=10)
    args = ap.parse_args()
    dmhip.load()
    conv_bench.run(args.shape, 5, 'fp16x2', args.tile, 2 if args.tile == 15 else 0)
    B, Cin, Cout, H, pro, up = conv_bench.SHAPES[args.shape]
    bm, bn = (64, 64) if args.tile == 15 else (128, 128 if args.tile == 10 else 64)
    nblk = (B * H * H // bm) * ((Cout + bn - 1) // bn)
    buf = np.zeros((nblk, 8), dtype=np.uint64)
    L = dmhip.load()
    L.dm_debug_k32_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert L.dm_debug_k32_stamps(buf.ctypes.data, nblk) == 0
    s = buf.astype(np.int64)
    pro_c = s[:, 1] - s[:, 0]
    loop_c = s[:, 2] - s[:, 1]
    seg2_c = s[:, 3] - s[:, 2]
    epi_c = s[:, 4] - s[:, 3]
    tot_c = s[:, 4] - s[:, 0]
    rt0, rt1 = s[:, 5], s[:, 6]
    wall_us = (rt1.max() - rt0.min()) / 100.0
    blk_us = (rt1 - rt0) / 100.0
    clk = tot_c / np.maximum(rt1 - rt0, 1) * 100e6 / 1e9
    print(f'{args.shape} tile {args.tile}: {nblk} blocks, kernel wall (stamps) {wall_us:.1f} us')
    for name, v in (('prologue', pro_c), ('main loop', loop_c), ('segment 2', seg2_c), ('epilogue', epi_c),
                    ('block total', tot_c)):
        print(f'  {name:12s} cycles mean {v.mean():10.0f}  p10 {np.percentile(v, 10):10.0f}  '
              f'p90 {np.percentile(v, 90):10.0f}  share {v.mean() / tot_c.mean():.3f}')
    print(f'  block wall us mean {blk_us.mean():.2f}, clock GHz mean {clk.mean():.3f}')
    order = np.argsort(rt0)
    starts = (rt0[order] - rt0.min()) / 100.0
    q = np.percentile(starts, [0, 12.5, 25, 37.5, 50, 62.5, 75, 87.5, 100])
    print('  block start times (us) at octiles:', ' '.join(f'{v:.1f}' for v in q))
    busy = np.zeros(int(wall_us) + 1)
    for a0, a1 in zip((rt0 - rt0.min()) / 100.0, (rt1 - rt0.min()) / 100.0):
        busy[int(a0):int(a1) + 1] += 1
    print('  resident blocks per us (every 10 us):', ' '.join(str(int(v)) for v in busy[::10]))


if __name__ == '__main__':
    main()
