"""Phase timing of attn_block_kernel (the folded CIFAR attention block) from the diagnostic build
(-DDM_K32_STAMPS): CIFAR-10 UNet forwards at B=256, then the last attention launch's per-work-group stamps.
Caveat: variants 3-5 sit at the register limit, and the stamps' scheduling barriers make their diagnostic builds
spill (556-968 B per lane, -Rpass-analysis=kernel-resource-usage): their phase shares (the "O finalize" above
all) describe the spilled build, not the product kernel; variant 2 does not spill.

    make -C diffusion-models-pytorch_amd/csrc BUILD=build_stamps OUT=../../tools/lib/libdm_stamps.so EXTRA=-DDM_K32_STAMPS
    DM_HIP_LIB=tools/lib/libdm_stamps.so [DM_ATTN=3] python tools/ab_stamps.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'diffusion-models-pytorch_amd')]

import dmhip  # noqa: E402
from models.unet import UNet  # noqa: E402
from utils.synthetic import init_synthetic_  # noqa: E402


def main():
    dmhip.load()
    dev = torch.device('cuda', 0)
    model = UNet().eval()
    init_synthetic_(model)
    model = model.to(dev)
    B = 256
    x = torch.randn((B, 3, 32, 32), device=dev)
    t = torch.full((B, ), 500, dtype=torch.long, device=dev)
    for _ in range(4):
        model(x, t)
    torch.cuda.synchronize()
    nblk = B * 2
    buf = np.zeros((nblk, 10), dtype=np.uint64)
    L = dmhip.load()
    L.dm_debug_ab_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert L.dm_debug_ab_stamps(buf.ctypes.data, nblk) == 0
    s = buf.astype(np.int64)
    names = ['T (At xn^T)', 'T finalize + split', 'keys: S + softmax + P xn', 'O finalize', 'Y = Wg O', 'epilogue']
    tot = s[:, 6] - s[:, 0]
    wall = s[:, 9] - s[:, 8]
    print(f'attn_block kernel (variant {os.environ.get("DM_ATTN", "4")}): {nblk} work-groups, wall (stamps) {(s[:, 9].max() - s[:, 8].min()) / 100.0:.1f} us, '
          f'work-group cycles mean {tot.mean():.0f}, clock {np.mean(tot / np.maximum(wall, 1)) / 100:.3f} GHz')
    for i, n in enumerate(names):
        v = s[:, i + 1] - s[:, i]
        print(f'  {n:20s} cycles mean {v.mean():9.0f} p10 {np.percentile(v, 10):9.0f} p90 {np.percentile(v, 90):9.0f}'
              f'  share {v.mean() / tot.mean():.3f}')
    ids = s[:, 7]
    u, cnt = np.unique(ids, return_counts=True)
    print(f'  distinct CU ids {len(u)}, work-groups per id: min {cnt.min()} max {cnt.max()} mean {cnt.mean():.2f}')
    dur = (s[:, 9] - s[:, 8]) / 100.0
    print(f'  work-group wall us: min {dur.min():.1f} p50 {np.median(dur):.1f} max {dur.max():.1f}')
    start = (s[:, 8] - s[:, 8].min()) / 100.0
    print(f'  start times (us): p0 {np.min(start):.1f} p25 {np.percentile(start, 25):.1f} p50 {np.median(start):.1f} '
          f'p75 {np.percentile(start, 75):.1f} max {np.max(start):.1f}')


if __name__ == '__main__':
    main()
