"""Diagnostic: is the ADM forward batch-invariant (row r of a B batch == the same row at B=1)?"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'diffusion-models-pytorch_amd')]
import torch  # noqa: E402

import dmhip  # noqa: E402
from models.adm.unet import UNetModel  # noqa: E402
from tests.conftest import load_golden  # noqa: E402
from utils.synthetic import init_synthetic_  # noqa: E402

dev = torch.device('cuda:0')
_, meta = load_golden('adm')
for name, res, batches in (('adm_tiny', 16, (1, 2, 8, 64)), ('adm256_combined', 256, (1, 2, 8))):
    arch = dict(meta['archs'][name])
    for math in ('fp16x2', 'bf16x3', 'fp32'):
        net = UNetModel(**arch).eval()
        init_synthetic_(net)
        net = net.to(dev)
        dmhip.unet_conv_math(net.native_handle(dev), math)
        g = torch.Generator().manual_seed(1)
        Bm = max(batches)
        x = torch.randn((Bm, arch['in_channels'], res, res), generator=g).to(dev)
        t = torch.randint(0, 1000, (Bm, ), generator=g).to(dev)
        y = torch.randint(0, arch.get('num_classes') or 1, (Bm, ), generator=g).to(dev) if arch.get('num_classes') else None
        ref = None
        for B in batches:
            out = net(x[:B].contiguous(), t[:B].contiguous(), None if y is None else y[:B].contiguous())
            if ref is None:
                ref = out[:1].clone()
            print(name, math, 'B', B, 'row0 maxdiff vs B=1', (out[:1] - ref).abs().max().item(),
                  'math now', dmhip.unet_conv_math(net.native_handle(dev)), flush=True)
        del net
        torch.cuda.empty_cache()
