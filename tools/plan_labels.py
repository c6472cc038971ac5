"""Diagnostic: kernel labels of an ADM-256 plan at two batch sizes (which launches change with B)."""
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
arch = dict(meta['archs']['adm256_combined'])
net = UNetModel(**arch).eval()
init_synthetic_(net)
net = net.to(dev)
labels = {}
for B in (1, 2):
    x = torch.zeros((B, 3, 256, 256), device=dev)
    t = torch.zeros((B, ), dtype=torch.long, device=dev)
    y = torch.zeros((B, ), dtype=torch.long, device=dev)
    net(x, t, y)
    h = net.native_handle(dev)
    dmhip.unet_profile_enable(h, 1)
    net(x, t, y)
    labels[B] = [op['label'] for op in dmhip.unet_profile_read(h)]
    dmhip.unet_profile_enable(h, 0)
print(len(labels[1]), len(labels[2]))
for i, (a, b) in enumerate(zip(labels[1], labels[2])):
    if a != b:
        print(i, a, '|', b)
