"""Plan-level rewrites that must not change the result, checked by building the same model twice with the
rewrite switched off by its environment toggle (read at plan build):

* linear_k32 with the A operand pre-split once per GEMM (`linear_presplit_a`, `row_stats_split`, fc1's
  epilogue writing fc2's pre-split A) against the split inside the GEMM: the same fp32 expressions, so
  the outputs are bit-identical (DiT: DM_DIT_PRESPLIT=0);
* GroupNorm partials emitted by producers instead of a `gn_partial` pass over the tensor (DM_GN_FUSION=0 turns
  all of them off): a concat's combined from its slices' partials (`gn_concat_stats`), the 4-channel units the
  h slice of a 384 = 256 + 128 concat emits, the first conv's epilogue, the sub-pixel upsample's epilogue: the
  same sums in another fp64 order, so equal to within a few fp32 ulps of the output.
"""
import os

import pytest
import torch

from models.dit.model import DiT_models
from models.unet import UNet
from utils.synthetic import init_synthetic_

pytestmark = pytest.mark.gpu


def _with_env(var, val, fn):
    old = os.environ.get(var)
    if val is None:
        os.environ.pop(var, None)
    else:
        os.environ[var] = val
    try:
        return fn()
    finally:
        if old is None:
            os.environ.pop(var, None)
        else:
            os.environ[var] = old


def _dit_out(cuda, sd, x, t, y):
    m = DiT_models['DiT-S/2'](input_size=32, num_classes=1000, learn_sigma=True).eval()
    m.load_state_dict(sd)
    m = m.to(cuda)
    with torch.no_grad():
        return m(x, t, y).cpu()


def test_dit_presplit_bit_identical(cuda):
    ref = DiT_models['DiT-S/2'](input_size=32, num_classes=1000, learn_sigma=True).eval()
    init_synthetic_(ref)
    sd = ref.state_dict()
    g = torch.Generator().manual_seed(7)
    B = 16  # B * T = 4096 token rows: the pre-split path's threshold
    x = torch.randn((B, 4, 32, 32), generator=g).to(cuda)
    t = torch.randint(0, 1000, (B, ), generator=g).to(cuda)
    y = torch.randint(0, 1000, (B, ), generator=g).to(cuda)
    on = _with_env('DM_DIT_PRESPLIT', None, lambda: _dit_out(cuda, sd, x, t, y))
    off = _with_env('DM_DIT_PRESPLIT', '0', lambda: _dit_out(cuda, sd, x, t, y))
    assert torch.isfinite(on).all()
    assert torch.equal(on, off), (on - off).abs().max().item()


def _unet_out(cuda, sd, x, t):
    m = UNet().eval()
    m.load_state_dict(sd)
    m = m.to(cuda)
    with torch.no_grad():
        return m(x, t).cpu()


@pytest.fixture(scope='module')
def unet_case(cuda):
    ref = UNet().eval()
    init_synthetic_(ref)
    g = torch.Generator().manual_seed(11)
    B = 8
    x = torch.randn((B, 3, 32, 32), generator=g).to(cuda)
    t = torch.randint(0, 1000, (B, ), generator=g).to(cuda)
    return ref.state_dict(), x, t


def test_unet_emitted_gn_stats(cuda, unet_case):
    sd, x, t = unet_case
    on = _with_env('DM_GN_FUSION', None, lambda: _unet_out(cuda, sd, x, t))
    off = _with_env('DM_GN_FUSION', '0', lambda: _unet_out(cuda, sd, x, t))
    scale = off.abs().max().item()
    assert (on - off).abs().max().item() <= 1e-6 * scale
