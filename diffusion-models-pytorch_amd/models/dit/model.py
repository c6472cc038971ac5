"""DiT (Scalable Diffusion Models with Transformers) on the MI355X engine.

Drop-in for the reference models/dit/model.py:145-385: same constructor
(input_size, patch_size, in_channels, hidden_size, depth, num_heads,
mlp_ratio, class_dropout_prob, num_classes, learn_sigma), the DiT_models
table, and the same state_dict names/shapes, including the timm~=0.9.12
submodule names the reference builds on (``x_embedder.proj``,
``blocks.N.attn.qkv``, ``blocks.N.mlp.fc1`` ...), so DiT checkpoints load
unchanged. ``forward(x, t, y=None)``: y None (or, inside the CFG samplers'
``dmhip.null_label_scope()``, y[b] = -1) selects the null
class ``num_classes`` (model.py:241-242); ``forward_with_cfg`` as upstream.

The modules are parameter containers; the forward pass is one dm_dit_forward
call (csrc/dit_exec.hip): patch-embed GEMM + pos_embed, one GEMM for every
block's adaLN modulation, LayerNorm + modulate fused into the QKV / fc1 /
final GEMM prologues, gated residuals in the proj / fc2 epilogues,
GELU(tanh) epilogue, MFMA attention. Inference only (dropout / label dropout
off, as in the reference's eval path).

Parity note: timm is not installed here, so the reference module cannot be
executed; parity of this path is against oracle/dit.py (a restatement of
model.py + timm 0.9.12 PatchEmbed / Attention / Mlp), i.e. UNPINNED.
"""
import math

import numpy as np
import torch
import torch.nn as nn
from torch import Tensor

from dmhip._lib import DiTArch, check, load, stream_handle
from ..unet import NativeDenoiser


def get_2d_sincos_pos_embed(embed_dim: int, grid_size: int) -> np.ndarray:
    """Fixed 2-D sin-cos position table (model.py:278-325; MAE pos_embed): [grid^2, embed_dim] float64."""
    assert embed_dim % 2 == 0

    def one_d(dim, pos):
        omega = np.arange(dim // 2, dtype=np.float64)
        omega /= dim / 2.
        omega = 1. / 10000 ** omega
        out = np.einsum('m,d->md', pos.reshape(-1), omega)
        return np.concatenate([np.sin(out), np.cos(out)], axis=1)

    gh = np.arange(grid_size, dtype=np.float32)
    gw = np.arange(grid_size, dtype=np.float32)
    grid = np.stack(np.meshgrid(gw, gh), axis=0).reshape([2, 1, grid_size, grid_size])
    return np.concatenate([one_d(embed_dim // 2, grid[0]), one_d(embed_dim // 2, grid[1])], axis=1)


class PatchEmbed(nn.Module):
    """timm PatchEmbed parameters: proj = Conv2d(C, D, k = s = p)."""

    def __init__(self, img_size, patch_size, in_chans, embed_dim, bias=True):
        super().__init__()
        self.img_size = (img_size, img_size)
        self.patch_size = (patch_size, patch_size)
        self.num_patches = (img_size // patch_size) ** 2
        self.proj = nn.Conv2d(in_chans, embed_dim, kernel_size=patch_size, stride=patch_size, bias=bias)


class Attention(nn.Module):
    """timm Attention parameters: qkv Linear(D, 3D), proj Linear(D, D)."""

    def __init__(self, dim, num_heads=8, qkv_bias=True):
        super().__init__()
        self.num_heads = num_heads
        self.head_dim = dim // num_heads
        self.scale = self.head_dim ** -0.5
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.proj = nn.Linear(dim, dim)


class Mlp(nn.Module):
    """timm Mlp parameters: fc1 Linear(D, H), fc2 Linear(H, D)."""

    def __init__(self, in_features, hidden_features):
        super().__init__()
        self.fc1 = nn.Linear(in_features, hidden_features)
        self.fc2 = nn.Linear(hidden_features, in_features)


class TimestepEmbedder(nn.Module):
    """model.py:27-64 parameters (mlp = Linear(256, D), SiLU, Linear(D, D))."""

    def __init__(self, hidden_size, frequency_embedding_size=256):
        super().__init__()
        self.mlp = nn.Sequential(nn.Linear(frequency_embedding_size, hidden_size, bias=True), nn.SiLU(),
                                 nn.Linear(hidden_size, hidden_size, bias=True))
        self.frequency_embedding_size = frequency_embedding_size


class LabelEmbedder(nn.Module):
    """model.py:67-94 parameters: table of num_classes (+1 CFG null row when dropout_prob > 0)."""

    def __init__(self, num_classes, hidden_size, dropout_prob):
        super().__init__()
        self.embedding_table = nn.Embedding(num_classes + int(dropout_prob > 0), hidden_size)
        self.num_classes = num_classes
        self.dropout_prob = dropout_prob


class DiTBlock(nn.Module):
    """model.py:101-122 parameters (norm1/norm2 have none)."""

    def __init__(self, hidden_size, num_heads, mlp_ratio=4.0):
        super().__init__()
        self.attn = Attention(hidden_size, num_heads=num_heads, qkv_bias=True)
        self.mlp = Mlp(hidden_size, int(hidden_size * mlp_ratio))
        self.adaLN_modulation = nn.Sequential(nn.SiLU(), nn.Linear(hidden_size, 6 * hidden_size, bias=True))


class FinalLayer(nn.Module):
    """model.py:125-142 parameters."""

    def __init__(self, hidden_size, patch_size, out_channels):
        super().__init__()
        self.linear = nn.Linear(hidden_size, patch_size * patch_size * out_channels, bias=True)
        self.adaLN_modulation = nn.Sequential(nn.SiLU(), nn.Linear(hidden_size, 2 * hidden_size, bias=True))


class DiT(NativeDenoiser):
    """Diffusion model with a Transformer backbone (model.py:145-270)."""

    _abi = 'dm_dit'

    def __init__(self, input_size=32, patch_size=2, in_channels=4, hidden_size=1152, depth=28, num_heads=16,
                 mlp_ratio=4.0, class_dropout_prob=0.1, num_classes=1000, learn_sigma=True):
        super().__init__()
        self.learn_sigma = learn_sigma
        self.in_channels = in_channels
        self.out_channels = in_channels * 2 if learn_sigma else in_channels
        self.patch_size = patch_size
        self.num_heads = num_heads
        self.num_classes = num_classes
        self.supports_null_label = class_dropout_prob > 0
        self.arch = dict(in_channels=in_channels, out_channels=self.out_channels, input_size=input_size,
                         patch_size=patch_size, hidden_size=hidden_size, depth=depth, num_heads=num_heads,
                         mlp_hidden=int(hidden_size * mlp_ratio), num_classes=num_classes,
                         null_class=class_dropout_prob > 0, learn_sigma=learn_sigma,
                         label_rows=num_classes + int(class_dropout_prob > 0))

        self.x_embedder = PatchEmbed(input_size, patch_size, in_channels, hidden_size, bias=True)
        self.t_embedder = TimestepEmbedder(hidden_size)
        self.y_embedder = LabelEmbedder(num_classes, hidden_size, class_dropout_prob)
        num_patches = self.x_embedder.num_patches
        self.pos_embed = nn.Parameter(torch.zeros(1, num_patches, hidden_size), requires_grad=False)
        self.blocks = nn.ModuleList([DiTBlock(hidden_size, num_heads, mlp_ratio=mlp_ratio) for _ in range(depth)])
        self.final_layer = FinalLayer(hidden_size, patch_size, self.out_channels)
        pos = get_2d_sincos_pos_embed(hidden_size, int(num_patches ** 0.5))
        self.pos_embed.data.copy_(torch.from_numpy(pos).float().unsqueeze(0))

    # ----------------------------------------------------------- native side
    def _arch_struct(self) -> DiTArch:
        a = DiTArch()
        for k in ('input_size', 'patch_size', 'in_channels', 'hidden_size', 'depth', 'num_heads', 'mlp_hidden',
                  'num_classes'):
            setattr(a, k, int(self.arch[k]))
        a.null_class = int(self.arch['null_class'])
        a.learn_sigma = int(self.arch['learn_sigma'])
        return a

    def _time_freqs(self) -> Tensor:
        # model.py:51-54 (frequency_embedding_size 256, max_period 10000)
        half = 128
        return torch.exp(-math.log(10000) * torch.arange(start=0, end=half, dtype=torch.float32) / half)

    def _launch(self, handle, X: Tensor, T: Tensor, y_ptr, out: Tensor):
        if X.shape[2] != self.arch['input_size'] or X.shape[3] != self.arch['input_size']:
            raise ValueError(f'expected {self.arch["input_size"]}x{self.arch["input_size"]} latents, '
                             f'got {tuple(X.shape)}')
        check(load().dm_dit_forward(handle, X.data_ptr(), T.data_ptr(), y_ptr, X.shape[0], out.data_ptr(),
                                    stream_handle(X.device)), 'dm_dit_forward')

    # --------------------------------------------------------------- forward
    def forward(self, x: Tensor, t: Tensor, y: Tensor = None):
        """model.py:234-252. y None -> the null class (requires class_dropout_prob > 0, as upstream)."""
        if y is None and not self.arch['null_class']:
            raise IndexError('index out of range in self')  # nn.Embedding on label num_classes
        return self._run(x, t, y)

    def forward_with_cfg(self, x: Tensor, t: Tensor, y: Tensor, cfg_scale: float):
        """model.py:254-270: CFG on the first 3 channels, both halves from one batched forward."""
        half = x[: len(x) // 2]
        combined = torch.cat([half, half], dim=0)
        model_out = self.forward(combined, t, y)
        eps, rest = model_out[:, :3], model_out[:, 3:]
        cond_eps, uncond_eps = torch.split(eps, len(eps) // 2, dim=0)
        half_eps = uncond_eps + cfg_scale * (cond_eps - uncond_eps)
        eps = torch.cat([half_eps, half_eps], dim=0)
        return torch.cat([eps, rest], dim=1)


def DiT_XL_2(**kwargs):
    return DiT(depth=28, hidden_size=1152, patch_size=2, num_heads=16, **kwargs)


def DiT_XL_4(**kwargs):
    return DiT(depth=28, hidden_size=1152, patch_size=4, num_heads=16, **kwargs)


def DiT_XL_8(**kwargs):
    return DiT(depth=28, hidden_size=1152, patch_size=8, num_heads=16, **kwargs)


def DiT_L_2(**kwargs):
    return DiT(depth=24, hidden_size=1024, patch_size=2, num_heads=16, **kwargs)


def DiT_L_4(**kwargs):
    return DiT(depth=24, hidden_size=1024, patch_size=4, num_heads=16, **kwargs)


def DiT_L_8(**kwargs):
    return DiT(depth=24, hidden_size=1024, patch_size=8, num_heads=16, **kwargs)


def DiT_B_2(**kwargs):
    return DiT(depth=12, hidden_size=768, patch_size=2, num_heads=12, **kwargs)


def DiT_B_4(**kwargs):
    return DiT(depth=12, hidden_size=768, patch_size=4, num_heads=12, **kwargs)


def DiT_B_8(**kwargs):
    return DiT(depth=12, hidden_size=768, patch_size=8, num_heads=12, **kwargs)


def DiT_S_2(**kwargs):
    return DiT(depth=12, hidden_size=384, patch_size=2, num_heads=6, **kwargs)


def DiT_S_4(**kwargs):
    return DiT(depth=12, hidden_size=384, patch_size=4, num_heads=6, **kwargs)


def DiT_S_8(**kwargs):
    return DiT(depth=12, hidden_size=384, patch_size=8, num_heads=6, **kwargs)


DiT_models = {
    'DiT-XL/2': DiT_XL_2, 'DiT-XL/4': DiT_XL_4, 'DiT-XL/8': DiT_XL_8,
    'DiT-L/2': DiT_L_2, 'DiT-L/4': DiT_L_4, 'DiT-L/8': DiT_L_8,
    'DiT-B/2': DiT_B_2, 'DiT-B/4': DiT_B_4, 'DiT-B/8': DiT_B_8,
    'DiT-S/2': DiT_S_2, 'DiT-S/4': DiT_S_4, 'DiT-S/8': DiT_S_8,
}
