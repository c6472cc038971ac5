"""ADM UNetModel (OpenAI guided-diffusion) on the MI355X engine.

Drop-in for the reference models/adm/unet.py:415-682 (UNetModel): same
constructor arguments and the same state_dict names/shapes
(``input_blocks.1.0.in_layers.0.weight``, ``...emb_layers.1.weight``,
``...qkv.weight [3C, C, 1]``, ``out.2.weight`` ...), so guided-diffusion /
RePaint / ILVR checkpoints and the reference YAML configs load unchanged.
``forward(x, timesteps, y=None)`` with y required iff ``num_classes`` is set
(adm/unet.py:662-664).

The modules below are parameter containers; the forward pass runs as one
dm_unet_forward call (variant 2 of dm_unet_arch): [cos, sin] timestep
embedding (adm/nn.py:103-121), scale-shift-norm ResBlocks folded into the
conv2 GroupNorm prologue, ResBlock up/down (avg-pool / nearest), fused qkv
1x1 conv with q and k each scaled by ch^-1/4 (QKVAttentionLegacy or
QKVAttention head layout), learned-sigma outputs (out_channels = 2C).
fp32 only (``use_fp16=True`` is refused); gradient checkpointing is a
training option and has no effect here.
"""
import torch
import torch.nn as nn
from torch import Tensor

from ..unet import NativeDenoiser


def _gn(C: int) -> nn.GroupNorm:
    return nn.GroupNorm(32, C)   # GroupNorm32 (adm/nn.py:17-19, 93-100)


class ResBlock(nn.Module):
    """Parameter container of adm/unet.py:162-275."""

    def __init__(self, channels, emb_channels, dropout, out_channels=None, use_conv=False,
                 use_scale_shift_norm=False, dims=2, use_checkpoint=False, up=False, down=False):
        super().__init__()
        out = out_channels or channels
        if out != channels and use_conv:
            raise NotImplementedError('3x3 skip_connection (use_conv=True) is not used by UNetModel')
        self.in_layers = nn.Sequential(_gn(channels), nn.SiLU(), nn.Conv2d(channels, out, 3, padding=1))
        self.updown = up or down
        self.emb_layers = nn.Sequential(nn.SiLU(), nn.Linear(emb_channels, 2 * out if use_scale_shift_norm else out))
        self.out_layers = nn.Sequential(_gn(out), nn.SiLU(), nn.Dropout(p=dropout), nn.Conv2d(out, out, 3, padding=1))
        self.skip_connection = nn.Identity() if out == channels else nn.Conv2d(channels, out, 1)


class AttentionBlock(nn.Module):
    """Parameter container of adm/unet.py:278-324 (norm, qkv Conv1d, proj_out Conv1d)."""

    def __init__(self, channels, num_heads=1, num_head_channels=-1, use_checkpoint=False,
                 use_new_attention_order=False):
        super().__init__()
        if num_head_channels == -1:
            self.num_heads = num_heads
        else:
            assert channels % num_head_channels == 0, \
                f'q,k,v channels {channels} is not divisible by num_head_channels {num_head_channels}'
            self.num_heads = channels // num_head_channels
        self.norm = _gn(channels)
        self.qkv = nn.Conv1d(channels, channels * 3, 1)
        self.proj_out = nn.Conv1d(channels, channels, 1)


class Downsample(nn.Module):
    """adm/unet.py:132-159: stride-2 conv (`op`) or 2x2 average pool."""

    def __init__(self, channels, use_conv, dims=2, out_channels=None):
        super().__init__()
        out = out_channels or channels
        self.op = nn.Conv2d(channels, out, 3, stride=2, padding=1) if use_conv else nn.AvgPool2d(2, 2)


class Upsample(nn.Module):
    """adm/unet.py:100-129: nearest 2x, then an optional conv (`conv`)."""

    def __init__(self, channels, use_conv, dims=2, out_channels=None):
        super().__init__()
        if use_conv:
            self.conv = nn.Conv2d(channels, out_channels or channels, 3, padding=1)


class UNetModel(NativeDenoiser):
    """The full ADM UNet with attention and timestep embedding (adm/unet.py:415-682)."""

    def __init__(self, image_size, in_channels, model_channels, out_channels, num_res_blocks,
                 attention_resolutions, dropout=0, channel_mult=(1, 2, 4, 8), conv_resample=True, dims=2,
                 num_classes=None, use_checkpoint=False, use_fp16=False, num_heads=1, num_head_channels=-1,
                 num_heads_upsample=-1, use_scale_shift_norm=False, resblock_updown=False,
                 use_new_attention_order=False):
        super().__init__()
        if dims != 2:
            raise NotImplementedError('only 2-D ADM models are supported')
        if use_fp16:
            raise NotImplementedError('use_fp16: the engine computes in fp32 (the reference CPU path precision)')
        if num_heads_upsample == -1:
            num_heads_upsample = num_heads
        self.image_size = image_size
        self.in_channels = in_channels
        self.model_channels = model_channels
        self.out_channels = out_channels
        self.num_res_blocks = num_res_blocks
        self.attention_resolutions = attention_resolutions
        self.channel_mult = channel_mult
        self.num_classes = num_classes
        self.num_heads = num_heads
        self.num_head_channels = num_head_channels
        self.num_heads_upsample = num_heads_upsample
        self.dtype = torch.float32
        n = len(channel_mult)
        use_attn = [(2 ** lvl) in attention_resolutions for lvl in range(n)]
        self.arch = dict(in_channels=in_channels, out_channels=out_channels, dim=model_channels,
                         dim_mults=list(channel_mult), use_attn=use_attn, num_res_blocks=num_res_blocks,
                         n_heads=num_heads, variant=2, num_classes=num_classes or 0,
                         attn_head_dims=num_head_channels if num_head_channels != -1 else 0,
                         resblock_updown=bool(resblock_updown), n_heads_up=num_heads_upsample,
                         scale_shift_norm=bool(use_scale_shift_norm), pool_resample=not conv_resample,
                         attn_legacy=not use_new_attention_order)

        ted = model_channels * 4
        self.time_embed = nn.Sequential(nn.Linear(model_channels, ted), nn.SiLU(), nn.Linear(ted, ted))
        if num_classes is not None:
            self.label_emb = nn.Embedding(num_classes, ted)
        rb = dict(emb_channels=ted, dropout=dropout, use_scale_shift_norm=use_scale_shift_norm)
        at = dict(num_head_channels=num_head_channels, use_new_attention_order=use_new_attention_order)

        ch = input_ch = int(channel_mult[0] * model_channels)
        self.input_blocks = nn.ModuleList([nn.Sequential(nn.Conv2d(in_channels, ch, 3, padding=1))])
        chans = [ch]
        ds = 1
        for level, mult in enumerate(channel_mult):
            for _ in range(num_res_blocks):
                layers = [ResBlock(ch, out_channels=int(mult * model_channels), **rb)]
                ch = int(mult * model_channels)
                if ds in attention_resolutions:
                    layers.append(AttentionBlock(ch, num_heads=num_heads, **at))
                self.input_blocks.append(nn.Sequential(*layers))
                chans.append(ch)
            if level != n - 1:
                self.input_blocks.append(nn.Sequential(
                    ResBlock(ch, out_channels=ch, down=True, **rb) if resblock_updown
                    else Downsample(ch, conv_resample, out_channels=ch)))
                chans.append(ch)
                ds *= 2
        self.middle_block = nn.Sequential(
            ResBlock(ch, **rb), AttentionBlock(ch, num_heads=num_heads, **at), ResBlock(ch, **rb))
        self.output_blocks = nn.ModuleList()
        for level, mult in list(enumerate(channel_mult))[::-1]:
            for i in range(num_res_blocks + 1):
                ich = chans.pop()
                layers = [ResBlock(ch + ich, out_channels=int(model_channels * mult), **rb)]
                ch = int(model_channels * mult)
                if ds in attention_resolutions:
                    layers.append(AttentionBlock(ch, num_heads=num_heads_upsample, **at))
                if level and i == num_res_blocks:
                    layers.append(ResBlock(ch, out_channels=ch, up=True, **rb) if resblock_updown
                                  else Upsample(ch, conv_resample, out_channels=ch))
                    ds //= 2
                self.output_blocks.append(nn.Sequential(*layers))
        self.out = nn.Sequential(_gn(ch), nn.SiLU(), nn.Conv2d(input_ch, out_channels, 3, padding=1))

    def forward(self, x: Tensor, timesteps: Tensor, y: Tensor = None):
        """adm/unet.py:653-682."""
        assert (y is not None) == (self.num_classes is not None), \
            'must specify y if and only if the model is class-conditional'
        if y is not None and y.shape != (x.shape[0], ):
            raise AssertionError(f'expected y of shape ({x.shape[0]},), got {tuple(y.shape)}')
        return self._run(x, timesteps, y)
