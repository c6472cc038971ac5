"""DDPM UNet denoiser (CIFAR-10 / MNIST / CelebA configs) on the MI355X engine.

Drop-in for the reference models/unet.py:46-152:
  * same constructor (in_channels, out_channels, dim, dim_mults, use_attn,
    num_res_blocks, n_heads, dropout) and the same parameter names/shapes, so
    reference YAML configs and checkpoints load unchanged
    (e.g. ``down_blocks.1.1.q.weight [256,256,1,1]``, 328 tensors for CIFAR-10);
  * ``forward(X [B,C,H,W] f32, T [B] int64) -> [B, out_channels, H, W] f32``.

The torch modules below are parameter containers only. ``forward`` hands the
parameters to the native executor (dm_unet_create packs them once into the
library's own layout) and runs the whole network as one C-ABI call
(dm_unet_forward): NHWC activations, implicit-GEMM convolutions on the matrix cores (fp16x2 split
of the fp32 operands by default),
fused GroupNorm+SiLU, zero-copy skip concatenation. Inference only
(Dropout = identity, i.e. the reference in eval mode). No CPU fallback.
"""
import ctypes
import math
from typing import List, Sequence

import torch
import torch.nn as nn
from torch import Tensor

import dmhip
from dmhip._lib import UNetArch, check, load, stream_handle


def _gn(C: int) -> nn.GroupNorm:
    return nn.GroupNorm(32, C)


def _conv(cin: int, cout: int, k: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, k, stride=stride, padding=k // 2)


class ResBlock(nn.Module):
    """Parameter container of models/unet.py:10-43 (GN-SiLU-conv, temb add, GN-SiLU-conv, shortcut)."""

    def __init__(self, in_channels: int, out_channels: int, embed_dim: int, dropout: float = 0.1):
        super().__init__()
        # Sequential indices reproduce the reference state_dict names:
        # blk1.{0: GroupNorm, 2: Conv}, proj.1: Linear, blk2.{0: GroupNorm, 3: Conv}
        self.blk1 = nn.Sequential(_gn(in_channels), nn.SiLU(), _conv(in_channels, out_channels, 3))
        self.proj = nn.Sequential(nn.SiLU(), nn.Linear(embed_dim, out_channels))
        self.blk2 = nn.Sequential(_gn(out_channels), nn.SiLU(), nn.Dropout(dropout),
                                  _conv(out_channels, out_channels, 3))
        self.shortcut = _conv(in_channels, out_channels, 1) if in_channels != out_channels else nn.Identity()


class SelfAttentionBlock(nn.Module):
    """Parameter container of models/modules.py:77-102 (GN, q/k/v/proj 1x1 convs)."""

    def __init__(self, dim: int, n_heads: int = 1, groups: int = 32):
        super().__init__()
        assert dim % n_heads == 0
        self.n_heads = n_heads
        self.norm = nn.GroupNorm(groups, dim)
        self.q = _conv(dim, dim, 1)
        self.k = _conv(dim, dim, 1)
        self.v = _conv(dim, dim, 1)
        self.proj = _conv(dim, dim, 1)
        self.scale = (dim // n_heads) ** -0.5


class _TimeEmbedding(nn.Sequential):
    """Index layout of the reference time MLP: 0 sinusoid (no params), 1 Linear, 2 SiLU, 3 Linear."""

    def __init__(self, dim: int):
        super().__init__(nn.Identity(), nn.Linear(dim, 4 * dim), nn.SiLU(), nn.Linear(4 * dim, 4 * dim))


class NativeDenoiser(nn.Module):
    """Parameter-container base: packs ``state_dict()`` into the native executor and runs
    the whole forward pass as one C-ABI call. Subclasses set ``self.arch``; the UNet family
    binds the dm_unet_* entry points, other executors (DiT) override the ``_abi`` hooks."""

    _native = None
    _native_key = None
    _param_list = None
    _abi = 'dm_unet'

    # ----------------------------------------------------------- native side
    def _arch_struct(self) -> UNetArch:
        a = UNetArch()
        a.in_channels = self.arch['in_channels']
        a.out_channels = self.arch['out_channels']
        a.dim = self.arch['dim']
        a.n_stages = len(self.arch['dim_mults'])
        for i, (m, at) in enumerate(zip(self.arch['dim_mults'], self.arch['use_attn'])):
            a.dim_mults[i] = m
            a.use_attn[i] = int(at)
        a.num_res_blocks = self.arch['num_res_blocks']
        a.n_heads = self.arch.get('n_heads', 1)
        a.variant = self.arch.get('variant', 0)
        a.num_classes = self.arch.get('num_classes', 0) or 0
        a.attn_head_dims = self.arch.get('attn_head_dims', 0)
        a.resblock_updown = int(self.arch.get('resblock_updown', False))
        a.n_heads_up = self.arch.get('n_heads_up', 0)
        a.scale_shift_norm = int(self.arch.get('scale_shift_norm', False))
        a.pool_resample = int(self.arch.get('pool_resample', False))
        a.attn_legacy = int(self.arch.get('attn_legacy', False))
        return a

    @staticmethod
    def _params_key(tensors: Sequence[Tensor]):
        # storage identity + in-place version counters: load_state_dict / optimizer steps /
        # manual edits all bump _version, so the packed copy is refreshed on any change
        return (tuple(t.data_ptr() for t in tensors), sum(t._version for t in tensors))

    def _release_native(self):
        if getattr(self, '_native', None) is not None:
            # an open deferred-range scope polls (and forgets) the handle before it is freed
            dmhip.deferred_range_check.release(self._native)
            getattr(load(), self._abi + '_destroy')(self._native)
            self._native = None
            self._native_key = None
        self._param_list = None

    def native_handle(self, device: torch.device):
        """Create (or reuse) the packed native model. Re-packs when parameters change."""
        tensors = getattr(self, '_param_list', None)
        if tensors is None:
            # the Parameter objects themselves (their version counters see in-place updates)
            tensors = list(self.state_dict(keep_vars=True).values())
            self._param_list = tensors
        if self._native is not None and self._native_key == self._params_key(tensors):
            return self._native
        for p in tensors:
            if p.device != device:
                raise RuntimeError(f'UNet parameters are on {p.device} but the input is on {device}; '
                                   f'move the model with .to(device) first')
            if p.dtype != torch.float32 or not p.is_contiguous():
                raise TypeError('UNet parameters must be contiguous float32')
        key = self._params_key(tensors)
        self._release_native()
        self._param_list = tensors
        L = load()
        n = len(tensors)
        ptrs = (ctypes.c_void_p * n)(*[t.data_ptr() for t in tensors])
        numels = (ctypes.c_int64 * n)(*[t.numel() for t in tensors])
        handle = ctypes.c_void_p()
        arch = self._arch_struct()
        check(getattr(L, self._abi + '_create')(ctypes.byref(arch), ptrs, numels, n, stream_handle(device),
                                                ctypes.byref(handle)), self._abi + '_create')
        # sinusoid frequencies evaluated with the reference's own torch CPU expression
        freqs = self._time_freqs().to(device)
        check(getattr(L, self._abi + '_set_time_freqs')(handle, freqs.data_ptr(), freqs.numel(), stream_handle(device)),
              self._abi + '_set_time_freqs')
        self._share_peer_workspace(handle)
        torch.cuda.current_stream(device).synchronize()
        self._native = handle
        self._native_key = key
        return handle

    def _share_peer_workspace(self, handle):
        """UNetCombined's two networks never need to run at the same time: the second handle to be created
        adopts the first one's plan scratch (dm_unet_share_workspace), one workspace for both. Forwards issued
        on different streams stay correct: the engine makes a forward on a new stream wait for the previous
        forward over the shared scratch (an event wait), so they serialise instead of racing."""
        ref = self.__dict__.get('_ws_peer')
        peer = ref() if ref is not None else None
        if peer is not None and self._abi == 'dm_unet' and getattr(peer, '_abi', None) == 'dm_unet' \
                and getattr(peer, '_native', None) is not None:
            dmhip.share_workspace(peer._native, handle)

    def _time_freqs(self) -> Tensor:
        half = self.arch['dim'] // 2
        if self.arch.get('variant', 0) == 2:
            # adm/nn.py:114-116
            return torch.exp(-math.log(10000) * torch.arange(start=0, end=half, dtype=torch.float32) / half)
        # models/modules.py:52-54
        return torch.exp(torch.arange(half) * -(math.log(10000) / (half - 1)))

    def _launch(self, handle, X: Tensor, T: Tensor, y_ptr, out: Tensor):
        B, _, H, W = X.shape
        check(load().dm_unet_forward(handle, X.data_ptr(), T.data_ptr(), y_ptr, B, H, W, out.data_ptr(),
                                     stream_handle(X.device)), 'dm_unet_forward')

    def _apply(self, fn, *args, **kwargs):
        self._release_native()
        return super()._apply(fn, *args, **kwargs)

    def __del__(self):
        try:
            self._release_native()
        except Exception:
            pass

    # --------------------------------------------------------------- forward
    def _run(self, X: Tensor, T: Tensor, y: Tensor = None) -> Tensor:
        dmhip.require_device_tensor(X, 'X')
        dmhip.require_device_tensor(T, 'T', dtype=torch.long)
        if X.ndim != 4 or X.shape[1] != self.arch['in_channels']:
            raise ValueError(f'expected input [B, {self.arch["in_channels"]}, H, W], got {tuple(X.shape)}')
        B, _, H, W = X.shape
        if T.shape != (B, ):
            raise ValueError(f'expected T of shape ({B},), got {tuple(T.shape)}')
        y_ptr = None
        if y is not None:
            dmhip.require_device_tensor(y, 'y', dtype=torch.long)
            if y.shape != (B, ):
                raise ValueError(f'expected y of shape ({B},), got {tuple(y.shape)}')
            self._check_labels(y)
            y_ptr = y.data_ptr()
        handle = self.native_handle(X.device)
        scope = dmhip.deferred_range_check.active
        if scope is not None:   # inside a sampler's sample(): the range flag is polled once per loop
            scope.register(handle, self._abi, X.device)
        out = torch.empty((B, self.arch['out_channels'], H, W), device=X.device, dtype=torch.float32)
        self._launch(handle, X, T, y_ptr, out)
        return out

    def _check_labels(self, y: Tensor):
        """nn.Embedding raises IndexError on an out-of-range label; so do we. y[b] = -1 ("no label"
        for row b) is accepted only inside dmhip.null_label_scope(), which the CFG samplers open
        around their batched 2B forward. The check syncs once per distinct label tensor (labels are
        fixed across a sampling loop)."""
        null_ok = dmhip.null_labels_allowed()
        key = (y.data_ptr(), y._version, y.numel(), null_ok)
        if getattr(self, '_labels_ok', None) == key:
            return
        n = self.arch.get('label_rows', self.arch.get('num_classes', 0) or 0)
        if y.numel():
            hi, lo = int(y.max()), int(y.min())
            if hi >= n:
                raise IndexError(f'class label {hi} out of range for num_classes={n}')
            if lo < (-1 if null_ok else 0):
                raise IndexError(f'class label {lo} out of range for num_classes={n}')
        self._labels_ok = key


class UNet(NativeDenoiser):
    def __init__(
            self,
            in_channels: int = 3,
            out_channels: int = 3,
            dim: int = 128,
            dim_mults: List[int] = (1, 2, 2, 2),
            use_attn: List[int] = (False, True, False, False),
            num_res_blocks: int = 2,
            n_heads: int = 1,
            dropout: float = 0.1,
    ):
        super().__init__()
        if len(dim_mults) != len(use_attn):
            raise ValueError('dim_mults and use_attn must have the same length')
        self.arch = dict(in_channels=in_channels, out_channels=out_channels, dim=dim,
                         dim_mults=list(dim_mults), use_attn=[bool(a) for a in use_attn],
                         num_res_blocks=num_res_blocks, n_heads=n_heads)
        temb = 4 * dim
        self.time_embed = _TimeEmbedding(dim)
        self.first_conv = _conv(in_channels, dim, 3)

        chans = [dim]       # channels of every skip, in push order
        cur = dim
        self.down_blocks = nn.ModuleList()
        for i, mult in enumerate(dim_mults):
            out = dim * mult
            stage = nn.ModuleList()
            for _ in range(num_res_blocks):
                stage.append(ResBlock(cur, out, temb, dropout))
                if use_attn[i]:
                    stage.append(SelfAttentionBlock(out, n_heads=n_heads))
                chans.append(out)
                cur = out
            if i < len(dim_mults) - 1:
                stage.append(_conv(out, out, 3, stride=2))   # Downsample (modules.py:70-72)
                chans.append(out)
            self.down_blocks.append(stage)

        self.bottleneck_block = nn.ModuleList([
            ResBlock(cur, cur, temb, dropout), SelfAttentionBlock(cur), ResBlock(cur, cur, temb, dropout),
        ])

        self.up_blocks = nn.ModuleList()
        for i in reversed(range(len(dim_mults))):
            out = dim * dim_mults[i]
            stage = nn.ModuleList()
            for _ in range(num_res_blocks + 1):
                stage.append(ResBlock(chans.pop() + cur, out, temb, dropout))
                if use_attn[i]:
                    stage.append(SelfAttentionBlock(out, n_heads=n_heads))
                cur = out
            if i > 0:
                # Upsample = nearest 2x then conv (modules.py:60-65); index 1 holds the conv
                stage.append(nn.Sequential(nn.Upsample(scale_factor=2, mode='nearest'), _conv(out, out, 3)))
            self.up_blocks.append(stage)

        self.last_conv = nn.Sequential(_gn(cur), nn.SiLU(), _conv(cur, out_channels, 3))

    def forward(self, X: Tensor, T: Tensor):
        """models/unet.py:121-152: X [B, C, H, W] f32, T [B] int64 -> [B, out_channels, H, W]."""
        return self._run(X, T)
