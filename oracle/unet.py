"""UNet forward oracle (TEST INFRASTRUCTURE ONLY) — torch CPU functional ops.

Restates models/unet.py:121-152 + models/modules.py:45-102 (and
models/unet_categorial_adagn.py:12-208 + modules.py:105-123) from a reference
state_dict, in the reference's op order (F.conv2d / F.group_norm / F.silu /
F.linear / bmm / softmax are the ops nn.Module.forward dispatches to), so it
is bit-identical to the reference module at the same torch thread count.
"""
import math
from typing import Dict, Optional, Sequence

import torch
import torch.nn.functional as F
from torch import Tensor


def _conv(sd, name, x, stride=1):
    w = sd[name + '.weight']
    return F.conv2d(x, w, sd[name + '.bias'], stride=stride, padding=w.shape[-1] // 2)


def _gn(sd, name, x, groups=32):
    return F.group_norm(x, groups, sd[name + '.weight'], sd[name + '.bias'], 1e-5)


def _lin(sd, name, x):
    return F.linear(x, sd[name + '.weight'], sd[name + '.bias'])


def sinusoidal(t: Tensor, dim: int) -> Tensor:
    """models/modules.py:45-57"""
    half = dim // 2
    f = torch.exp(torch.arange(half, device=t.device) * -(math.log(10000) / (half - 1)))
    e = t[:, None] * f[None, :]
    return torch.cat((e.sin(), e.cos()), dim=-1)


def resblock(sd, p, x, temb):
    """models/unet.py:30-43 (eval mode: Dropout is identity)"""
    sc = _conv(sd, p + '.shortcut', x) if (p + '.shortcut.weight') in sd else x
    h = _conv(sd, p + '.blk1.2', F.silu(_gn(sd, p + '.blk1.0', x)))
    h = h + _lin(sd, p + '.proj.1', F.silu(temb))[:, :, None, None]
    h = _conv(sd, p + '.blk2.3', F.silu(_gn(sd, p + '.blk2.0', h)))
    return h + sc


def attention(sd, p, x, heads):
    """models/modules.py:89-102"""
    bs, C, H, W = x.shape
    nx = _gn(sd, p + '.norm', x)
    q = _conv(sd, p + '.q', nx).view(bs * heads, -1, H * W)
    k = _conv(sd, p + '.k', nx).view(bs * heads, -1, H * W)
    v = _conv(sd, p + '.v', nx).view(bs * heads, -1, H * W)
    q = q * ((C // heads) ** -0.5)
    a = torch.bmm(q.permute(0, 2, 1), k).softmax(dim=-1)
    o = torch.bmm(v, a.permute(0, 2, 1)).view(bs, -1, H, W)
    return _conv(sd, p + '.proj', o) + x


def unet_forward(sd: Dict[str, Tensor], x: Tensor, t: Tensor, dim=128, dim_mults: Sequence[int] = (1, 2, 2, 2),
                 use_attn: Sequence[bool] = (False, True, False, False), num_res_blocks=2, n_heads=1) -> Tensor:
    """models/unet.py:121-152"""
    temb = _lin(sd, 'time_embed.3', F.silu(_lin(sd, 'time_embed.1', sinusoidal(t, dim))))
    h = _conv(sd, 'first_conv', x)
    skips = [h]
    n = len(dim_mults)
    for i in range(n):
        j = 0
        for _ in range(num_res_blocks):
            h = resblock(sd, f'down_blocks.{i}.{j}', h, temb)
            skips.append(h)
            j += 1
            if use_attn[i]:
                h = attention(sd, f'down_blocks.{i}.{j}', h, n_heads)
                skips[-1] = h
                j += 1
        if i < n - 1:
            h = _conv(sd, f'down_blocks.{i}.{j}', h, stride=2)
            skips.append(h)
    h = resblock(sd, 'bottleneck_block.0', h, temb)
    h = attention(sd, 'bottleneck_block.1', h, 1)
    h = resblock(sd, 'bottleneck_block.2', h, temb)
    for s, i in enumerate(reversed(range(n))):
        j = 0
        for _ in range(num_res_blocks + 1):
            h = resblock(sd, f'up_blocks.{s}.{j}', torch.cat((h, skips.pop()), dim=1), temb)
            j += 1
            if use_attn[i]:
                h = attention(sd, f'up_blocks.{s}.{j}', h, n_heads)
                j += 1
        if i > 0:
            h = _conv(sd, f'up_blocks.{s}.{j}.1', F.interpolate(h, scale_factor=2, mode='nearest'))
    h = _conv(sd, 'last_conv.2', F.silu(_gn(sd, 'last_conv.0', h)))
    return h


def adagn_resblock(sd, p, x, temb, updown=None):
    """models/unet_categorial_adagn.py:44-62 + AdaGN models/modules.py:114-123 (eval mode)"""
    if updown is None:
        h = _conv(sd, p + '.blk1.2', F.silu(_gn(sd, p + '.blk1.0', x)))
    else:
        h = updown(F.silu(_gn(sd, p + '.blk1.0', x)))
        x = updown(x)
        h = _conv(sd, p + '.blk1.2', h)
    ys, yb = torch.chunk(_lin(sd, p + '.adagn.proj.1', F.silu(temb)), 2, dim=-1)
    h = _gn(sd, p + '.adagn.gn', h) * (1 + ys[:, :, None, None]) + yb[:, :, None, None]
    h = _conv(sd, p + '.blk2.2', F.silu(h))
    sc = _conv(sd, p + '.shortcut', x) if (p + '.shortcut.weight') in sd else x
    return h + sc


def _up(h):
    return F.interpolate(h, scale_factor=2, mode='nearest')


def _down(h):
    return F.avg_pool2d(h, kernel_size=2, stride=2)


def unet_categorial_forward(sd: Dict[str, Tensor], x: Tensor, t: Tensor, y: Optional[Tensor] = None, dim=128,
                            dim_mults: Sequence[int] = (1, 2, 2, 2),
                            use_attn: Sequence[bool] = (False, True, True, False), num_res_blocks=2,
                            attn_head_dims=64, resblock_updown=True) -> Tensor:
    """models/unet_categorial_adagn.py:165-208"""
    temb = _lin(sd, 'time_embed.3', F.silu(_lin(sd, 'time_embed.1', sinusoidal(t, dim))))
    if 'class_embed.weight' in sd and y is not None:
        temb = temb + F.embedding(y, sd['class_embed.weight'])
    h = _conv(sd, 'first_conv', x)
    skips = [h]
    n = len(dim_mults)
    for i in range(n):
        j = 0
        heads = dim * dim_mults[i] // attn_head_dims
        for _ in range(num_res_blocks):
            h = adagn_resblock(sd, f'down_blocks.{i}.{j}', h, temb)
            skips.append(h)
            j += 1
            if use_attn[i]:
                h = attention(sd, f'down_blocks.{i}.{j}', h, heads)
                skips[-1] = h
                j += 1
        if i < n - 1:
            if resblock_updown:
                h = adagn_resblock(sd, f'down_blocks.{i}.{j}', h, temb, _down)
            else:
                h = _conv(sd, f'down_blocks.{i}.{j}', h, stride=2)
            skips.append(h)
    h = adagn_resblock(sd, 'bottleneck_block.0', h, temb)
    h = attention(sd, 'bottleneck_block.1', h, 1)
    h = adagn_resblock(sd, 'bottleneck_block.2', h, temb)
    for s, i in enumerate(reversed(range(n))):
        j = 0
        heads = dim * dim_mults[i] // attn_head_dims
        for _ in range(num_res_blocks + 1):
            h = adagn_resblock(sd, f'up_blocks.{s}.{j}', torch.cat((h, skips.pop()), dim=1), temb)
            j += 1
            if use_attn[i]:
                h = attention(sd, f'up_blocks.{s}.{j}', h, heads)
                j += 1
        if i > 0:
            if resblock_updown:
                h = adagn_resblock(sd, f'up_blocks.{s}.{j}', h, temb, _up)
            else:
                h = _conv(sd, f'up_blocks.{s}.{j}.1', _up(h))
    h = _conv(sd, 'last_conv.2', F.silu(_gn(sd, 'last_conv.0', h)))
    return h


class OracleUNetCategorialAdaGN:
    """Callable model(x, t, y=None) over a state_dict, matching UNetCategorialAdaGN.forward."""

    def __init__(self, sd: Dict[str, Tensor], **arch):
        self.sd = {k: v.detach().to('cpu', torch.float32) for k, v in sd.items()}
        keep = ('dim', 'dim_mults', 'use_attn', 'num_res_blocks', 'attn_head_dims', 'resblock_updown')
        self.arch = {k: v for k, v in arch.items() if k in keep}

    @torch.no_grad()
    def __call__(self, x: Tensor, t: Tensor, y: Optional[Tensor] = None) -> Tensor:
        return unet_categorial_forward(self.sd, x, t, y, **self.arch)


class OracleUNet:
    """Callable model(x, t) over a state_dict, matching the reference UNet's forward."""

    def __init__(self, sd: Dict[str, Tensor], **arch):
        self.sd = {k: v.detach().to('cpu', torch.float32) for k, v in sd.items()}
        self.arch = {k: v for k, v in arch.items() if k in ('dim', 'dim_mults', 'use_attn', 'num_res_blocks', 'n_heads')}

    @torch.no_grad()
    def __call__(self, x: Tensor, t: Tensor, y: Optional[Tensor] = None) -> Tensor:
        return unet_forward(self.sd, x, t, **self.arch)
