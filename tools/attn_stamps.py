"""Phase timing of attn_presplit_kernel (the fused CIFAR attention) from the diagnostic build
(-DDM_K32_STAMPS): CIFAR-10 UNet forwards at B=256, then the last attention launch's per-block stamps.

    DM_HIP_LIB=tools/bin/libdm_stamps.so python tools/attn_stamps.py
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
    nblk = B * 4
    buf = np.zeros((nblk, 10), dtype=np.uint64)
    L = dmhip.load()
    L.dm_debug_attn_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert L.dm_debug_attn_stamps(buf.ctypes.data, nblk) == 0
    s = buf.astype(np.int64)
    names = ['S (QK^T)', 'S -> LDS? softmax', 'PV', 'proj split', 'proj MFMA', 'proj epilogue']
    bounds = [(0, 1), (1, 2), (2, 3), (3, 4), (4, 5), (5, 8)]
    tot = s[:, 8] - s[:, 0]
    print(f'attn_presplit_kernel: {nblk} blocks, wall (stamps) {(s[:, 7].max() - s[:, 6].min()) / 100.0:.1f} us, '
          f'block cycles mean {tot.mean():.0f}, clock {np.mean(tot / np.maximum(s[:, 7] - s[:, 6], 1)) / 10:.3f} GHz')
    for n, (i, j) in zip(names, bounds):
        v = s[:, j] - s[:, i]
        print(f'  {n:18s} cycles mean {v.mean():9.0f} p10 {np.percentile(v, 10):9.0f} p90 {np.percentile(v, 90):9.0f}'
              f'  share {v.mean() / tot.mean():.3f}')
    # the qkv 1x1 conv (conv_patch3 MODE 3, attention-plane epilogue) of the same forward
    nq = (B * 256 // 128) * (768 // 128)
    buf = np.zeros((nq, 8), dtype=np.uint64)
    L.dm_debug_pw_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert L.dm_debug_pw_stamps(buf.ctypes.data, nq) == 0
    s = buf.astype(np.int64)
    tot = s[:, 3] - s[:, 0]
    print(f'qkv conv_patch3 MODE 3: {nq} blocks, wall (stamps) {(s[:, 6].max() - s[:, 5].min()) / 100.0:.1f} us, '
          f'block cycles mean {tot.mean():.0f}')
    for n, (i, j) in zip(['prologue', 'main loop', 'plane epilogue'], [(0, 1), (1, 2), (2, 3)]):
        v = s[:, j] - s[:, i]
        print(f'  {n:18s} cycles mean {v.mean():9.0f} p10 {np.percentile(v, 10):9.0f} p90 {np.percentile(v, 90):9.0f}'
              f'  share {v.mean() / tot.mean():.3f}')


if __name__ == '__main__':
    main()
