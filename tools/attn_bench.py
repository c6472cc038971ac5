"""Attention paths on the BASELINE geometries, flash vs unfused, with per-op-family times of one forward
(HIP events on every launch, dm_*_profile): DiT-XL/2 at the C5 CFG batch (2B = 64, 32x32 latents) and the
guided-diffusion 256x256 UNet (C4 arch, L = 1024 / 256 / 64 attention) at B = 4.

    python tools/attn_bench.py [--which dit|adm|both] [--iters 3]
"""
import argparse
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'diffusion-models-pytorch_amd')]

import torch  # noqa: E402

import dmhip  # noqa: E402
from utils.synthetic import init_synthetic_  # noqa: E402


def build(which):
    if which == 'dit':
        from models.dit.model import DiT_models
        m = DiT_models['DiT-XL/2'](input_size=32, num_classes=1000, learn_sigma=True).eval()
        B, shape = 64, (4, 32, 32)
    else:
        import json
        from models.adm.unet import UNetModel
        arch = json.load(open(os.path.join(ROOT, 'tests', 'golden', 'adm.json')))['archs']['adm256_combined']
        m = UNetModel(**arch).eval()
        B, shape = 4, (3, 256, 256)
    init_synthetic_(m)
    return m, B, shape


def run(which, mode, iters):
    if mode == 'unfused':
        os.environ['DM_ATTN'] = 'unfused'
    else:
        os.environ.pop('DM_ATTN', None)
    dev = torch.device('cuda', 0)
    m, B, shape = build(which)
    m = m.to(dev)
    g = torch.Generator().manual_seed(0)
    x = torch.randn((B, ) + shape, generator=g).to(dev)
    t = torch.randint(0, 1000, (B, ), generator=g).to(dev)
    y = torch.randint(0, 1000, (B, ), generator=g).to(dev)
    for _ in range(2):
        m(x, t, y)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        m(x, t, y)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    h = m.native_handle(dev)
    dmhip.unet_profile_enable(h, 1, m._abi)
    m(x, t, y)
    torch.cuda.synchronize()
    fam = defaultdict(lambda: [0.0, 0, 0.0])
    for op in dmhip.unet_profile_read(h, m._abi):
        f = fam[op['label']]
        f[0] += op['ms_total']
        f[1] += op['launches']
        f[2] += op['flops']
    dmhip.unet_profile_enable(h, 0, m._abi)
    print(f'{which} {mode}: {ms:.2f} ms / forward (B = {B})', flush=True)
    for lab, (t_ms, n, fl) in sorted(fam.items(), key=lambda kv: -kv[1][0])[:12]:
        tf = fl / (t_ms * 1e-3) / 1e12 if t_ms > 0 and fl > 0 else 0.0
        print(f'   {t_ms:8.3f} ms  {n:4d} x  {tf:7.1f} TF  {lab}', flush=True)
    del m
    torch.cuda.empty_cache()


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('--which', default='both')
    ap.add_argument('--iters', type=int, default=3)
    ap.add_argument('--modes', default='flash,unfused')
    a = ap.parse_args()
    for w in (['dit', 'adm'] if a.which == 'both' else [a.which]):
        for mode in a.modes.split(','):
            run(w, mode, a.iters)
