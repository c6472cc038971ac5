"""Per-GEMM-shape times of the DiT-XL/2 C5 forward (2B = 64 rows of 32x32 latents) from the plan's per-op
HIP events: the token GEMMs told apart by their FLOP count (qkv, proj, fc1, fc2, final layer).
    python tools/dit_gemms.py [--batch 64] [--iters 3]"""
import argparse
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'diffusion-models-pytorch_amd')]

import torch  # noqa: E402

import dmhip  # noqa: E402
from models.dit.model import DiT_models  # noqa: E402
from utils.synthetic import init_synthetic_  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=64)
    ap.add_argument('--iters', type=int, default=3)
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    m = DiT_models['DiT-XL/2'](input_size=32, num_classes=1000, learn_sigma=True).eval()
    init_synthetic_(m)
    m = m.to(dev)
    B = args.batch
    g = torch.Generator().manual_seed(0)
    x = torch.randn((B, 4, 32, 32), generator=g).to(dev)
    t = torch.randint(0, 1000, (B, ), generator=g).to(dev)
    y = torch.randint(0, 1000, (B, ), generator=g).to(dev)
    for _ in range(2):
        m(x, t, y)
    torch.cuda.synchronize()
    h = m.native_handle(dev)
    dmhip.unet_profile_enable(h, 1, m._abi)
    for _ in range(args.iters):
        m(x, t, y)
    torch.cuda.synchronize()
    fam = defaultdict(lambda: [0.0, 0])
    for op in dmhip.unet_profile_read(h, m._abi):
        f = fam[(op['label'], op['flops'] / max(op['launches'], 1))]
        f[0] += op['ms_total']
        f[1] += op['launches']
    dmhip.unet_profile_enable(h, 0, m._abi)
    tot = sum(v[0] for v in fam.values())
    for (lab, fl), (ms, n) in sorted(fam.items(), key=lambda kv: -kv[1][0]):
        us = ms / n * 1e3
        tf = fl / (us * 1e-6) / 1e12 if fl > 0 else 0.0
        print(f'{100 * ms / tot:6.2f} %  {n:4d} x {us:8.1f} us  {fl / 1e9:8.2f} GF  {tf:7.1f} TF ({tf / 833.3:.3f})  {lab}',
              flush=True)


if __name__ == '__main__':
    main()
