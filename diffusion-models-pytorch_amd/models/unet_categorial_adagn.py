"""Class-conditional UNet with AdaGN (UNetCategorialAdaGN) on the MI355X engine.

Drop-in for the reference models/unet_categorial_adagn.py:75-208:
  * same constructor (in_channels, out_channels, dim, dim_mults, use_attn,
    num_res_blocks, num_classes, attn_head_dims, resblock_updown, dropout) and
    the same parameter names/shapes (``class_embed.weight``,
    ``down_blocks.0.0.adagn.proj.1.weight`` ...), so reference configs and
    checkpoints load unchanged;
  * ``forward(X, T, y=None)``: y [B] int64 class labels or None. Inside
    ``dmhip.null_label_scope()`` (opened only by the CFG samplers) a label -1
    marks a row as unconditional, which lets classifier-free guidance run both
    branches as one 2B batch (the reference runs two calls, one with y and one
    with y=None; the per-row result is identical). Outside it a negative label
    raises IndexError, as nn.Embedding does upstream.

Executor differences from models/unet.py (variant 1 of dm_unet_arch):
  * AdaGN (modules.py:105-123) before conv2: gn(h) * (1 + ys) + yb with
    [ys | yb] = Linear(SiLU(temb)) is folded into the GroupNorm affine table
    that conv2's fused GN+SiLU prologue reads;
  * ResBlockDownsample / ResBlockUpsample (resblock_updown): avg-pool / nearest
    resampling of both the normalised branch and the residual, the upsample
    folded into conv1's halo-patch load;
  * stage attention uses C / attn_head_dims heads (bottleneck: 1 head).
"""
from typing import List

import torch.nn as nn
from torch import Tensor

from .unet import NativeDenoiser, SelfAttentionBlock, _TimeEmbedding, _conv, _gn


class AdaGN(nn.Module):
    """Parameter container of models/modules.py:105-123 (gn, proj = SiLU -> Linear(embed, 2C))."""

    def __init__(self, num_groups: int, num_channels: int, embed_dim: int):
        super().__init__()
        self.gn = nn.GroupNorm(num_groups, num_channels)
        self.proj = nn.Sequential(nn.SiLU(), nn.Linear(embed_dim, num_channels * 2))


class ResBlock(nn.Module):
    """Parameter container of models/unet_categorial_adagn.py:12-62."""

    def __init__(self, in_channels: int, out_channels: int, embed_dim: int, dropout: float = 0.1,
                 up: bool = False, down: bool = False):
        super().__init__()
        if up and down:
            raise ValueError('up and down cannot both be True')
        self.up, self.down = up, down
        self.blk1 = nn.Sequential(_gn(in_channels), nn.SiLU(), _conv(in_channels, out_channels, 3))
        self.adagn = AdaGN(32, out_channels, embed_dim)
        self.blk2 = nn.Sequential(nn.SiLU(), nn.Dropout(dropout), _conv(out_channels, out_channels, 3))
        self.shortcut = _conv(in_channels, out_channels, 1) if in_channels != out_channels else nn.Identity()


class ResBlockUpsample(ResBlock):
    def __init__(self, in_channels: int, out_channels: int, embed_dim: int, dropout: float = 0.1):
        super().__init__(in_channels, out_channels, embed_dim, dropout, up=True)


class ResBlockDownsample(ResBlock):
    def __init__(self, in_channels: int, out_channels: int, embed_dim: int, dropout: float = 0.1):
        super().__init__(in_channels, out_channels, embed_dim, dropout, down=True)


class UNetCategorialAdaGN(NativeDenoiser):
    """UNet conditioned on categorial labels with AdaGN (unet_categorial_adagn.py:75-208)."""

    supports_null_label = True  # y[b] = -1 = no label for row b (batched CFG, dmhip.null_label_scope)

    def __init__(
            self,
            in_channels: int = 3,
            out_channels: int = 3,
            dim: int = 128,
            dim_mults: List[int] = (1, 2, 2, 2),
            use_attn: List[int] = (False, True, True, False),
            num_res_blocks: int = 2,
            num_classes: int = None,
            attn_head_dims: int = 64,
            resblock_updown: bool = True,
            dropout: float = 0.1,
    ):
        super().__init__()
        if len(dim_mults) != len(use_attn):
            raise ValueError('dim_mults and use_attn must have the same length')
        self.arch = dict(in_channels=in_channels, out_channels=out_channels, dim=dim,
                         dim_mults=list(dim_mults), use_attn=[bool(a) for a in use_attn],
                         num_res_blocks=num_res_blocks, n_heads=1, variant=1,
                         num_classes=num_classes or 0, attn_head_dims=attn_head_dims,
                         resblock_updown=bool(resblock_updown))
        self.num_classes = num_classes
        embed_dim = 4 * dim
        self.time_embed = _TimeEmbedding(dim)
        self.class_embed = nn.Embedding(num_classes, embed_dim) if num_classes is not None else None
        self.first_conv = _conv(in_channels, dim, 3)

        chans = [dim]
        cur = dim
        self.down_blocks = nn.ModuleList()
        for i, mult in enumerate(dim_mults):
            out = dim * mult
            stage = nn.ModuleList()
            for _ in range(num_res_blocks):
                stage.append(ResBlock(cur, out, embed_dim, dropout))
                if use_attn[i]:
                    if out % attn_head_dims:
                        raise ValueError(f'{out} channels not divisible by attn_head_dims={attn_head_dims}')
                    stage.append(SelfAttentionBlock(out, n_heads=out // attn_head_dims))
                chans.append(out)
                cur = out
            if i < len(dim_mults) - 1:
                if resblock_updown:
                    stage.append(ResBlockDownsample(out, out, embed_dim, dropout))
                else:
                    stage.append(_conv(out, out, 3, stride=2))   # Downsample (modules.py:70-72)
                chans.append(out)
            self.down_blocks.append(stage)

        self.bottleneck_block = nn.ModuleList([
            ResBlock(cur, cur, embed_dim, dropout), SelfAttentionBlock(cur), ResBlock(cur, cur, embed_dim, dropout),
        ])

        self.up_blocks = nn.ModuleList()
        for i in reversed(range(len(dim_mults))):
            out = dim * dim_mults[i]
            stage = nn.ModuleList()
            for _ in range(num_res_blocks + 1):
                stage.append(ResBlock(chans.pop() + cur, out, embed_dim, dropout))
                if use_attn[i]:
                    stage.append(SelfAttentionBlock(out, n_heads=out // attn_head_dims))
                cur = out
            if i > 0:
                if resblock_updown:
                    stage.append(ResBlockUpsample(out, out, embed_dim, dropout))
                else:
                    stage.append(nn.Sequential(nn.Upsample(scale_factor=2, mode='nearest'), _conv(out, out, 3)))
            self.up_blocks.append(stage)

        self.last_conv = nn.Sequential(_gn(cur), nn.SiLU(), _conv(cur, out_channels, 3))

    def forward(self, X: Tensor, T: Tensor, y: Tensor = None):
        """unet_categorial_adagn.py:165-208. With ``class_embed`` None, y is ignored (as in the reference)."""
        return self._run(X, T, y if self.class_embed is not None else None)
