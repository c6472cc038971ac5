import sys, os
sys.path[:0] = ['/root/repo', '/root/repo/diffusion-models-pytorch_amd']
import torch, torch.nn.functional as F
import dmhip
from tests.test_gpu_ops import _nhwc, _pack, _pack_subpix, _run_conv
cuda = torch.device('cuda', 0)
def case(B, Cin, Cout, H, up, tiles, pro=True):
    g = torch.Generator().manual_seed(5)
    x = torch.randn((B, Cin, H, H), generator=g)
    w = torch.randn((Cout, Cin, 3, 3), generator=g) * 0.05
    b = torch.randn(Cout, generator=g)
    xd = _nhwc(x).to(cuda)
    sc = (torch.rand((B, Cin), generator=g) + 0.5).to(cuda); sh = (torch.rand((B, Cin), generator=g) - 0.5).to(cuda)
    wp = _pack_subpix(w, cuda) if up == 2 else _pack(w, cuda)
    Ho = 2 * H if up else H
    outs = {}
    for split in (False, True):
        for tile in tiles:
            try:
                y = _run_conv(cuda, xd, wp, Cout, Ho, Ho, 9, 1, up, b.to(cuda), tile=tile, pro=(sc, sh) if pro else None, split=split)
            except Exception as e:
                print('  skip', tile, split, e); continue
            outs[(split, tile)] = y.cpu()
            # B=2 subset
            y2 = _run_conv(cuda, xd[[0, B - 1]].contiguous(), wp, Cout, Ho, Ho, 9, 1, up, b.to(cuda), tile=tile,
                           pro=(sc[[0, B - 1]].contiguous(), sh[[0, B - 1]].contiguous()) if pro else None, split=split)
            outs[(split, tile, 'b2')] = y2.cpu()
    base = outs.get((True, tiles[0]))
    for k, v in outs.items():
        ref = outs[(k[0], tiles[0])]
        if len(k) == 3:
            d = (v - ref[[0, B - 1]]).abs().max().item()
        else:
            d = (v - ref).abs().max().item()
        print(f'  B={B} Cin={Cin} H={H} up={up} split={k[0]} tile={k[1:]} maxdiff vs tile{tiles[0]}: {d:.3e}')
for args in [(256, 128, 128, 32, 0), (256, 256, 256, 16, 0), (256, 256, 256, 8, 0), (256, 256, 256, 4, 0), (256, 256, 256, 8, 2), (64, 256, 256, 16, 2)]:
    case(*args, tiles=[4, 5, 6])
