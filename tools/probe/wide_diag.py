"""Where the wide-map Winograd conv differs from float64 on integer operands (diagnostic)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'diffusion-models-pytorch_amd')]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
import dmhip  # noqa: E402
from tests.test_gpu_ops import _ints, _nhwc, _pack, _run_conv  # noqa: E402

dmhip.load()
cuda = torch.device('cuda', 0)
for (B, Cin, Cout, H, W) in [(1, 64, 128, 8, 64), (1, 32, 128, 4, 64)]:
    x = _ints((B, Cin, H, W), -2, 3, seed=150)
    w = _ints((Cout, Cin, 3, 3), -2, 3, seed=151)
    b = _ints((Cout, ), seed=152)
    ref = _nhwc(F.conv2d(x.double(), w.double(), b.double(), padding=1).float())
    y = _run_conv(cuda, _nhwc(x).to(cuda), _pack(w, cuda), Cout, H, W, 9, 1, 0, b.to(cuda), tile=21,
                  split='fp16x2', wino=True).cpu()
    d = (y - ref).abs()
    bad = d.amax(dim=(0, 3))  # [H][W]
    print(B, Cin, Cout, H, W, 'max', d.max().item(), 'bad pixels', int((bad > 0).sum()))
    for hh in range(H):
        print(' '.join('X' if bad[hh, ww] > 0 else '.' for ww in range(W)))
    badc = d.amax(dim=(0, 1, 2))
    print('bad channels', (badc > 0).nonzero().flatten().tolist()[:40])
