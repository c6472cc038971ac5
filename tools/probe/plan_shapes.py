"""Diagnostics: the conv shapes and kernels of an ADM-256 plan at B = 64 (DM_PLAN_DEBUG output on stderr).
    DM_PLAN_DEBUG=1 python tools/probe/plan_shapes.py 2> gpurun_out/plan_shapes.txt"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'diffusion-models-pytorch_amd')]
import torch  # noqa: E402

from models.adm.unet import UNetModel  # noqa: E402
from tests.conftest import load_golden  # noqa: E402
from utils.synthetic import init_synthetic_  # noqa: E402

dev = torch.device('cuda:0')
_, meta = load_golden('adm')
net = UNetModel(**dict(meta['archs']['adm256_combined'])).eval()
init_synthetic_(net)
net = net.to(dev)
B = int(os.environ.get('B', '64'))
x = torch.zeros((B, 3, 256, 256), device=dev)
t = torch.zeros((B, ), dtype=torch.long, device=dev)
y = torch.zeros((B, ), dtype=torch.long, device=dev)
net(x, t, y)
torch.cuda.synchronize()
print('done')
