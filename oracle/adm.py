"""ADM UNetModel forward oracle (TEST INFRASTRUCTURE ONLY) — torch CPU functional ops.

Restates models/adm/unet.py:162-682 and models/adm/nn.py:93-121 (the OpenAI
guided-diffusion UNet as vendored by the reference) from a state_dict, in the
reference's op order, plus the UNetCombined routing (adm/unet_combined.py:23-25).
Pinned against tests/golden/adm.npz (outputs of the reference module itself).
"""
import math
from typing import Dict, Optional, Sequence

import torch
import torch.nn.functional as F
from torch import Tensor


def _gn(sd, name, x):
    return F.group_norm(x.float(), 32, sd[name + '.weight'], sd[name + '.bias'], 1e-5)


def _conv(sd, name, x, stride=1):
    w = sd[name + '.weight']
    if w.ndim == 3:  # Conv1d
        return F.conv1d(x, w, sd[name + '.bias'])
    return F.conv2d(x, w, sd[name + '.bias'], stride=stride, padding=w.shape[-1] // 2)


def _lin(sd, name, x):
    return F.linear(x, sd[name + '.weight'], sd[name + '.bias'])


def timestep_embedding(t: Tensor, dim: int, max_period=10000) -> Tensor:
    """adm/nn.py:103-121 ([cos, sin])"""
    half = dim // 2
    freqs = torch.exp(-math.log(max_period) * torch.arange(start=0, end=half, dtype=torch.float32) / half)
    args = t[:, None].float() * freqs[None]
    emb = torch.cat([torch.cos(args), torch.sin(args)], dim=-1)
    if dim % 2:
        emb = torch.cat([emb, torch.zeros_like(emb[:, :1])], dim=-1)
    return emb


def resblock(sd, p, x, emb, scale_shift, updown=None):
    """adm/unet.py:255-275 (eval mode)"""
    if updown is not None:
        h = F.silu(_gn(sd, p + '.in_layers.0', x))
        h = updown(h)
        x = updown(x)
        h = _conv(sd, p + '.in_layers.2', h)
    else:
        h = _conv(sd, p + '.in_layers.2', F.silu(_gn(sd, p + '.in_layers.0', x)))
    e = _lin(sd, p + '.emb_layers.1', F.silu(emb))[:, :, None, None]
    if scale_shift:
        scale, shift = torch.chunk(e, 2, dim=1)
        h = _gn(sd, p + '.out_layers.0', h) * (1 + scale) + shift
        h = _conv(sd, p + '.out_layers.3', F.silu(h))
    else:
        h = h + e
        h = _conv(sd, p + '.out_layers.3', F.silu(_gn(sd, p + '.out_layers.0', h)))
    skip = _conv(sd, p + '.skip_connection', x) if (p + '.skip_connection.weight') in sd else x
    return skip + h


def attention(sd, p, x, heads, legacy):
    """adm/unet.py:318-324 + QKVAttentionLegacy :356-373 / QKVAttention :389-408"""
    b, c, *spatial = x.shape
    x = x.reshape(b, c, -1)
    qkv = _conv(sd, p + '.qkv', _gn(sd, p + '.norm', x))
    bs, width, length = qkv.shape
    ch = width // (3 * heads)
    scale = 1 / math.sqrt(math.sqrt(ch))
    if legacy:
        q, k, v = qkv.reshape(bs * heads, ch * 3, length).split(ch, dim=1)
        w = torch.einsum('bct,bcs->bts', q * scale, k * scale)
    else:
        q, k, v = qkv.chunk(3, dim=1)
        w = torch.einsum('bct,bcs->bts', (q * scale).view(bs * heads, ch, length),
                         (k * scale).view(bs * heads, ch, length))
        v = v.reshape(bs * heads, ch, length)
    w = torch.softmax(w.float(), dim=-1)
    a = torch.einsum('bts,bcs->bct', w, v).reshape(bs, -1, length)
    h = _conv(sd, p + '.proj_out', a)
    return (x + h).reshape(b, c, *spatial)


def _heads(C, num_heads, num_head_channels):
    return num_heads if num_head_channels == -1 else C // num_head_channels


def unet_model_forward(sd: Dict[str, Tensor], x: Tensor, t: Tensor, y: Optional[Tensor], model_channels: int,
                       num_res_blocks: int, attention_resolutions: Sequence[int], channel_mult=(1, 2, 4, 8),
                       conv_resample=True, num_classes=None, num_heads=1, num_head_channels=-1,
                       num_heads_upsample=-1, use_scale_shift_norm=False, resblock_updown=False,
                       use_new_attention_order=False, **_unused) -> Tensor:
    """adm/unet.py:653-682 with the block layout of :489-635"""
    assert (y is not None) == (num_classes is not None)
    if num_heads_upsample == -1:
        num_heads_upsample = num_heads
    legacy = not use_new_attention_order
    ss = use_scale_shift_norm
    emb = _lin(sd, 'time_embed.2', F.silu(_lin(sd, 'time_embed.0', timestep_embedding(t, model_channels))))
    if num_classes is not None:
        emb = emb + F.embedding(y, sd['label_emb.weight'])
    pool = lambda h: F.avg_pool2d(h, kernel_size=2, stride=2)  # noqa: E731
    near = lambda h: F.interpolate(h, scale_factor=2, mode='nearest')  # noqa: E731
    hs = []
    h = _conv(sd, 'input_blocks.0.0', x)
    hs.append(h)
    ch = int(channel_mult[0] * model_channels)
    ds, blk = 1, 1
    for level, mult in enumerate(channel_mult):
        for _ in range(num_res_blocks):
            h = resblock(sd, f'input_blocks.{blk}.0', h, emb, ss)
            ch = int(mult * model_channels)
            if ds in attention_resolutions:
                h = attention(sd, f'input_blocks.{blk}.1', h, _heads(ch, num_heads, num_head_channels), legacy)
            hs.append(h)
            blk += 1
        if level != len(channel_mult) - 1:
            p = f'input_blocks.{blk}.0'
            if resblock_updown:
                h = resblock(sd, p, h, emb, ss, pool)
            elif conv_resample:
                h = _conv(sd, p + '.op', h, stride=2)
            else:
                h = pool(h)
            hs.append(h)
            blk += 1
            ds *= 2
    h = resblock(sd, 'middle_block.0', h, emb, ss)
    h = attention(sd, 'middle_block.1', h, _heads(ch, num_heads, num_head_channels), legacy)
    h = resblock(sd, 'middle_block.2', h, emb, ss)
    blk = 0
    for level, mult in list(enumerate(channel_mult))[::-1]:
        for i in range(num_res_blocks + 1):
            h = torch.cat([h, hs.pop()], dim=1)
            p = f'output_blocks.{blk}'
            h = resblock(sd, p + '.0', h, emb, ss)
            ch = int(model_channels * mult)
            j = 1
            if ds in attention_resolutions:
                h = attention(sd, f'{p}.1', h, _heads(ch, num_heads_upsample, num_head_channels), legacy)
                j = 2
            if level and i == num_res_blocks:
                if resblock_updown:
                    h = resblock(sd, f'{p}.{j}', h, emb, ss, near)
                elif conv_resample:
                    h = _conv(sd, f'{p}.{j}.conv', near(h))
                else:
                    h = near(h)
                ds //= 2
            blk += 1
    return _conv(sd, 'out.2', F.silu(_gn(sd, 'out.0', h)))


class OracleADM:
    """Callable model(x, t, y=None) over a UNetModel state_dict."""

    def __init__(self, sd: Dict[str, Tensor], **arch):
        self.sd = {k: v.detach().to('cpu', torch.float32) for k, v in sd.items()}
        self.arch = arch

    @torch.no_grad()
    def __call__(self, x: Tensor, t: Tensor, y: Optional[Tensor] = None) -> Tensor:
        return unet_model_forward(self.sd, x, t, y, **self.arch)


class OracleADMCombined:
    """adm/unet_combined.py:23-25: y None -> unet_uncond, else unet_cond."""

    def __init__(self, sd: Dict[str, Tensor], **arch):
        cond = {k[len('unet_cond.'):]: v for k, v in sd.items() if k.startswith('unet_cond.')}
        unc = {k[len('unet_uncond.'):]: v for k, v in sd.items() if k.startswith('unet_uncond.')}
        self.cond = OracleADM(cond, **arch)
        self.uncond = OracleADM(unc, **dict(arch, num_classes=None))

    def __call__(self, x: Tensor, t: Tensor, y: Optional[Tensor] = None) -> Tensor:
        return (self.uncond if y is None else self.cond)(x, t, y)
