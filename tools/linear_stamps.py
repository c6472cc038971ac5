"""Phase timing of linear_k32_kernel (diagnostic build -DDM_K32_STAMPS) on DiT-XL/2's GEMMs: the blocks of
the last launch with the given K (1152: qkv / proj / fc1 / final, the last of which is recorded; 4608: fc2),
or (--unet) on the CIFAR-10 UNet's attention qkv projection at B=256 (K 256, N 768, attention-plane epilogue).

    DM_HIP_LIB=tools/bin/libdm_stamps.so python tools/linear_stamps.py --k 4608
    DM_HIP_LIB=tools/bin/libdm_stamps.so python tools/linear_stamps.py --unet
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'diffusion-models-pytorch_amd')]

import dmhip  # noqa: E402
from models.dit.model import DiT_models  # noqa: E402
from utils.synthetic import init_synthetic_  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--k', type=int, default=4608)
    ap.add_argument('--n', type=int, default=1152, help='N of the recorded launch (blocks = 128 x N / 128)')
    ap.add_argument('--unet', action='store_true')
    args = ap.parse_args()
    if args.unet:
        args.k, args.n = 256, 768
    L = dmhip.load()
    L.dm_debug_lin_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    assert L.dm_debug_lin_stamps(None, 0, args.k) == 0
    dev = torch.device('cuda', 0)
    if args.unet:
        from models.unet import UNet
        model = UNet().eval()
        init_synthetic_(model)
        model = model.to(dev)
        B, L_tok = 256, 256
        x = torch.randn((B, 3, 32, 32), device=dev)
        t = torch.full((B, ), 500, dtype=torch.long, device=dev)
        for _ in range(4):
            model(x, t)
    else:
        model = DiT_models['DiT-XL/2'](input_size=32, num_classes=1000, learn_sigma=True).eval()
        init_synthetic_(model)
        model = model.to(dev)
        B, L_tok = 64, 256
        x = torch.randn((B, 4, 32, 32), device=dev)
        t = torch.randint(0, 1000, (B, ), device=dev)
        y = torch.randint(0, 1000, (B, ), device=dev)
        for _ in range(3):
            model(x, t, y)
    torch.cuda.synchronize()
    nblk = (B * L_tok // 128) * (args.n // 128)
    buf = np.zeros((nblk, 8), dtype=np.uint64)
    assert L.dm_debug_lin_stamps(buf.ctypes.data, nblk, args.k) == 0
    s = buf.astype(np.int64)
    tot = s[:, 3] - s[:, 0]
    print(f'linear_k32 K={args.k} N={args.n}: {nblk} blocks, wall (stamps) {(s[:, 6].max() - s[:, 5].min()) / 100.0:.1f} us,'
          f' block cycles mean {tot.mean():.0f}')
    for name, (i, j) in zip(['prologue', 'K loop', 'epilogue'], [(0, 1), (1, 2), (2, 3)]):
        v = s[:, j] - s[:, i]
        print(f'  {name:10s} cycles mean {v.mean():9.0f} p10 {np.percentile(v, 10):9.0f} p90 {np.percentile(v, 90):9.0f}'
              f'  share {v.mean() / tot.mean():.3f}')


if __name__ == '__main__':
    main()
