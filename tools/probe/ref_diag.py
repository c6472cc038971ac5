"""Diagnostics: the CIFAR reference-fixture forward (tests/golden/forward.npz) under plan toggles, twice each.
    python tools/probe/ref_diag.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'diffusion-models-pytorch_amd')]
import dmhip  # noqa: E402
from tests.test_gpu_parity import _model  # noqa: E402


def main():
    import json
    cuda = torch.device('cuda', 0)
    z = np.load(os.path.join(ROOT, 'tests/golden/forward.npz'), allow_pickle=False)
    meta = json.load(open(os.path.join(ROOT, 'tests/golden/forward.json')))
    x = torch.from_numpy(z['cifar10_x']).to(cuda)
    t = torch.from_numpy(z['cifar10_t']).to(cuda)
    ref = torch.from_numpy(z['cifar10_y'])
    print('x absmax', float(x.abs().max()), 't', t.tolist(), flush=True)
    for env in ([], [('DM_CONV_K32S2', '0')], [('DM_ATTN', '3')], [('DM_ATTN', '0')],
                [('DM_ATTN', '4')], [('DM_CONV_K32S2', '0'), ('DM_ATTN', '0')]):
        for k in ('DM_CONV_K32S2', 'DM_ATTN'):
            os.environ.pop(k, None)
        for k, v in env:
            os.environ[k] = v
        m, _ = _model(meta, 'cifar10', cuda)
        errs = []
        for _ in range(2):
            y = m(x, t).cpu()
            errs.append((y - ref).abs().max().item())
        h = m.native_handle(cuda)
        try:
            st = dmhip.range_stats(h)
        except Exception as e:  # noqa: BLE001
            st = repr(e)
        print(env, 'err', errs, 'range', st, flush=True)
        del m
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
