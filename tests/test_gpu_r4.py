"""Round-4 GPU tests: the folded single-head attention block (attn_block.hip) against the unfolded path
(q / k / v / proj as the reference computes them, DM_ATTN_FOLD=0) and the reference fixtures.

Reference: models/modules.py:77-102 (SelfAttentionBlock), models/unet.py:121-152.
"""
import numpy as np
import pytest
import torch

import dmhip
from tests.test_gpu_parity import TOL, _model
from utils.synthetic import init_synthetic_

pytestmark = pytest.mark.gpu


def _profile_labels(model, cuda):
    h = model.native_handle(torch.device(cuda))
    dmhip.unet_profile_enable(h, 1)
    return h


def _labels(h):
    return [op['label'] for op in dmhip.unet_profile_read(h)]


@pytest.mark.parametrize('B', [2, 7])
def test_folded_attention_vs_unfolded(cuda, golden, monkeypatch, B):
    """The CIFAR-10 UNet's five 16 x 16 attention blocks run folded (g GEMM + attn_block_kernel, no q / k / v
    planes): whole forwards within 1e-5 of the unfolded path (same weights, same inputs), and the folded
    kernels are the ones in the plan."""
    _, meta = golden('forward')
    g = torch.Generator().manual_seed(31)
    x = torch.randn((B, 3, 32, 32), generator=g).to(cuda)
    t = torch.randint(0, 1000, (B, ), generator=g).to(cuda)
    folded, _ = _model(meta, 'cifar10', cuda)
    out_f = folded(x, t)
    h = folded.native_handle(torch.device(cuda))
    dmhip.unet_profile_enable(h, 1)
    folded(x, t)
    labels = _labels(h)
    dmhip.unet_profile_enable(h, 0)
    assert labels.count('attn_block_kernel') == 5, labels
    assert not any(lb.startswith('attn_presplit_kernel') for lb in labels)
    monkeypatch.setenv('DM_ATTN_FOLD', '0')
    unfolded, _ = _model(meta, 'cifar10', cuda)
    out_u = unfolded(x, t)
    err = (out_f - out_u).abs().max().item()
    assert err <= 1e-5, err
    assert torch.isfinite(out_f).all()


def test_folded_attention_vs_reference(cuda, golden, report):
    """Reference fixture (tests/golden/forward.npz, the reference UNet itself at B = 2): the folded forward
    within 1e-4 (north_star tolerance)."""
    arrays, meta = golden('forward')
    model, _ = _model(meta, 'cifar10', cuda)
    y = model(torch.from_numpy(arrays['cifar10_x']).to(cuda), torch.from_numpy(arrays['cifar10_t']).to(cuda))
    err = (y.cpu() - torch.from_numpy(arrays['cifar10_y'])).abs().max().item()
    report('forward_cifar10_folded_attention_maxabs_vs_reference', err)
    assert err <= TOL, err


def test_folded_attention_batch_invariance(cuda, golden):
    """B = 256 (the benchmark batch) rows equal the B = 3 forward's rows bit for bit: every work-group is one
    (image, query half) and reads only its image."""
    _, meta = golden('forward')
    model, _ = _model(meta, 'cifar10', cuda)
    g = torch.Generator().manual_seed(32)
    x = torch.randn((256, 3, 32, 32), generator=g).to(cuda)
    t = torch.randint(0, 1000, (256, ), generator=g).to(cuda)
    big = model(x, t)
    idx = [0, 129, 255]
    small = model(x[idx].contiguous(), t[idx].contiguous())
    assert torch.equal(big[idx], small)
