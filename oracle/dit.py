"""DiT forward oracle (TEST INFRASTRUCTURE ONLY) — torch CPU functional ops.

Restates models/dit/model.py:19-252 together with the timm~=0.9.12 blocks the
reference imports at model.py:16 (timm is not installed in this image, so the
reference module cannot run here):
  * PatchEmbed  — Conv2d(C, D, kernel = stride = p) -> flatten(2).transpose(1, 2)
  * Attention   — qkv Linear -> reshape(B, N, 3, heads, d).permute(2, 0, 3, 1, 4)
                  -> softmax((q * d^-1/2) k^T) v -> transpose(1, 2).reshape(B, N, D) -> proj
                  (timm's non-fused path; its fused path, F.scaled_dot_product_attention,
                  is the same function)
  * Mlp         — fc1 -> GELU(approximate='tanh') -> fc2
PARITY UNPINNED: the reference ships no DiT tests or outputs, and timm is
absent, so this restatement (and the fixtures generated from it,
tests/golden/dit.*) is checked only against the published algorithm above.
"""
import math
from typing import Dict, Optional

import torch
import torch.nn.functional as F
from torch import Tensor


def _lin(sd, name, x):
    return F.linear(x, sd[name + '.weight'], sd[name + '.bias'])


def modulate(x, shift, scale):
    """model.py:19-20"""
    return x * (1 + scale.unsqueeze(1)) + shift.unsqueeze(1)


def timestep_embedding(t: Tensor, dim: int, max_period=10000) -> Tensor:
    """model.py:40-59 ([cos, sin])"""
    half = dim // 2
    freqs = torch.exp(-math.log(max_period) * torch.arange(start=0, end=half, dtype=torch.float32) / half)
    args = t[:, None].float() * freqs[None]
    emb = torch.cat([torch.cos(args), torch.sin(args)], dim=-1)
    if dim % 2:
        emb = torch.cat([emb, torch.zeros_like(emb[:, :1])], dim=-1)
    return emb


def attention(sd, p, x, heads):
    B, N, C = x.shape
    d = C // heads
    qkv = _lin(sd, p + '.qkv', x).reshape(B, N, 3, heads, d).permute(2, 0, 3, 1, 4)
    q, k, v = qkv.unbind(0)
    a = ((q * d ** -0.5) @ k.transpose(-2, -1)).softmax(dim=-1)
    x = (a @ v).transpose(1, 2).reshape(B, N, C)
    return _lin(sd, p + '.proj', x)


def mlp(sd, p, x):
    return _lin(sd, p + '.fc2', F.gelu(_lin(sd, p + '.fc1', x), approximate='tanh'))


def dit_forward(sd: Dict[str, Tensor], x: Tensor, t: Tensor, y: Optional[Tensor], patch_size: int, num_heads: int,
                depth: int, num_classes: int, out_channels: int, **_unused) -> Tensor:
    """model.py:234-252"""
    if y is None:
        y = torch.full((x.shape[0], ), fill_value=num_classes, dtype=torch.long)
    p = patch_size
    w = sd['x_embedder.proj.weight']
    h = F.conv2d(x, w, sd['x_embedder.proj.bias'], stride=p).flatten(2).transpose(1, 2)
    h = h + sd['pos_embed']
    te = _lin(sd, 't_embedder.mlp.2', F.silu(_lin(sd, 't_embedder.mlp.0', timestep_embedding(t, 256).to(h.dtype))))
    c = te + F.embedding(y, sd['y_embedder.embedding_table.weight'])
    D = h.shape[-1]
    for b in range(depth):
        pre = f'blocks.{b}'
        mods = _lin(sd, pre + '.adaLN_modulation.1', F.silu(c)).chunk(6, dim=1)
        shift_msa, scale_msa, gate_msa, shift_mlp, scale_mlp, gate_mlp = mods
        n1 = F.layer_norm(h, (D, ), eps=1e-6)
        h = h + gate_msa.unsqueeze(1) * attention(sd, pre + '.attn', modulate(n1, shift_msa, scale_msa), num_heads)
        n2 = F.layer_norm(h, (D, ), eps=1e-6)
        h = h + gate_mlp.unsqueeze(1) * mlp(sd, pre + '.mlp', modulate(n2, shift_mlp, scale_mlp))
    shift, scale = _lin(sd, 'final_layer.adaLN_modulation.1', F.silu(c)).chunk(2, dim=1)
    h = _lin(sd, 'final_layer.linear', modulate(F.layer_norm(h, (D, ), eps=1e-6), shift, scale))
    # unpatchify (model.py:219-232)
    n, T, _ = h.shape
    s = int(T ** 0.5)
    h = h.reshape(n, s, s, p, p, out_channels)
    h = torch.einsum('nhwpqc->nchpwq', h)
    return h.reshape(n, out_channels, s * p, s * p)


class OracleDiT:
    """Callable model(x, t, y=None) over a DiT state_dict."""

    def __init__(self, sd: Dict[str, Tensor], dtype=torch.float32, **arch):
        # dtype float64: the same restatement in double precision (the drift bound of the trajectory tests)
        self.sd = {k: v.detach().to('cpu', dtype) for k, v in sd.items()}
        self.dtype = dtype
        self.arch = arch

    @torch.no_grad()
    def __call__(self, x: Tensor, t: Tensor, y: Optional[Tensor] = None) -> Tensor:
        return dit_forward(self.sd, x.to(self.dtype), t, y, **self.arch)
