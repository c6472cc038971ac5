"""DiT-XL/2 forward timing (BASELINE config C5 geometry: 4x32x32 latents, CFG batch 2 x 32) per GEMM math.

    python tools/dit_bench.py [--batch 64] [--iters 5]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'diffusion-models-pytorch_amd')]

import torch  # noqa: E402

import dmhip  # noqa: E402
from models.dit.model import DiT_models  # noqa: E402
from utils.synthetic import init_synthetic_  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=64)
    ap.add_argument('--iters', type=int, default=5)
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    model = DiT_models['DiT-XL/2'](input_size=32, num_classes=1000, learn_sigma=True).eval()
    init_synthetic_(model)
    model = model.to(dev)
    B = args.batch
    x = torch.randn((B, 4, 32, 32), device=dev)
    t = torch.randint(0, 1000, (B, ), device=dev)
    y = torch.randint(0, 1000, (B, ), device=dev)
    h = model.native_handle(dev)
    gflop = 237.2  # per image per forward (analytic)
    for math in ('fp32', 'fp16x2'):
        dmhip.dit_math(h, math)
        for _ in range(2):
            model(x, t, y)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            model(x, t, y)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.iters
        print(f'DiT-XL/2 B={B} {math:7s} {ms:8.2f} ms/forward  {B * gflop / ms:7.1f} TFLOP/s  '
              f'{B / ms * 1e3:8.1f} img-forwards/s', flush=True)


if __name__ == '__main__':
    main()
