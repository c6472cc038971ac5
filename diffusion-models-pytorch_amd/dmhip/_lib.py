"""Loader and thin wrappers for libdm_hip.so.

Tensors cross the boundary as raw device pointers (``tensor.data_ptr()``);
torch-ROCm is used only for allocation and for the current HIP stream.
"""
import ctypes
import os
import re
from typing import Optional

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# DM_HIP_LIB: an alternative build of the same library (kernel-tuning experiments only)
lib_path = os.environ.get('DM_HIP_LIB') or os.path.join(_HERE, 'libdm_hip.so')
_HEADER = os.path.join(os.path.dirname(os.path.dirname(_HERE)), 'include', 'dm_hip.h')

ABI_VERSION = 2   # include/dm_hip.h DM_ABI_VERSION
DM_OK = 0
DM_ERR_ARG = -1
DM_ERR_HIP = -2
DM_ERR_STATE = -3
DM_ERR_UNSUPPORTED = -4
DM_MAX_STAGES = 8


class DMError(RuntimeError):
    """A failure reported by the native library (HIP error, bad state)."""


c_float_p = ctypes.POINTER(ctypes.c_float)
vp = ctypes.c_void_p


class UNetArch(ctypes.Structure):
    _fields_ = [
        ('in_channels', ctypes.c_int),
        ('out_channels', ctypes.c_int),
        ('dim', ctypes.c_int),
        ('n_stages', ctypes.c_int),
        ('dim_mults', ctypes.c_int * DM_MAX_STAGES),
        ('use_attn', ctypes.c_int * DM_MAX_STAGES),
        ('num_res_blocks', ctypes.c_int),
        ('n_heads', ctypes.c_int),
        ('variant', ctypes.c_int),
        ('num_classes', ctypes.c_int),
        ('attn_head_dims', ctypes.c_int),
        ('resblock_updown', ctypes.c_int),
        ('n_heads_up', ctypes.c_int),
        ('scale_shift_norm', ctypes.c_int),
        ('pool_resample', ctypes.c_int),
        ('attn_legacy', ctypes.c_int),
    ]


class DiTArch(ctypes.Structure):
    _fields_ = [
        ('input_size', ctypes.c_int), ('patch_size', ctypes.c_int), ('in_channels', ctypes.c_int),
        ('hidden_size', ctypes.c_int), ('depth', ctypes.c_int), ('num_heads', ctypes.c_int),
        ('mlp_hidden', ctypes.c_int), ('num_classes', ctypes.c_int), ('null_class', ctypes.c_int),
        ('learn_sigma', ctypes.c_int),
    ]


class StepDesc(ctypes.Structure):
    _fields_ = [
        ('B', ctypes.c_int), ('C', ctypes.c_int), ('HW', ctypes.c_int), ('Cm', ctypes.c_int),
        ('xt', vp), ('model_out', vp), ('model_out_uncond', vp),
        ('w_uncond', ctypes.c_float), ('w_cond', ctypes.c_float),
        ('objective', ctypes.c_int), ('clip_denoised', ctypes.c_int),
        ('sqrt_recip_ac', ctypes.c_float), ('sqrt_recipm1_ac', ctypes.c_float),
        ('sqrt_ac', ctypes.c_float), ('sqrt_one_minus_ac', ctypes.c_float),
        ('kind', ctypes.c_int),
        ('coef1', ctypes.c_float), ('coef2', ctypes.c_float),
        ('var_mode', ctypes.c_int), ('std', ctypes.c_float),
        ('min_logvar', ctypes.c_float), ('max_logvar', ctypes.c_float),
        ('add_noise', ctypes.c_int), ('noise', vp),
        ('sample', vp), ('mean', vp), ('pred_x0', vp), ('pred_eps', vp), ('var', vp),
        ('euler', ctypes.c_int), ('e_st1', ctypes.c_float), ('e_sig_t', ctypes.c_float),
        ('e_dsig', ctypes.c_float), ('e_sp1', ctypes.c_float), ('e_sig_p', ctypes.c_float),
        ('e_d1', vp), ('e_x1', vp), ('e_dout', vp),
    ]


class ConvDesc(ctypes.Structure):
    _fields_ = [
        ('x', vp), ('x_pitch', ctypes.c_int), ('Cin', ctypes.c_int), ('Hin', ctypes.c_int), ('Win', ctypes.c_int),
        ('taps', ctypes.c_int), ('stride', ctypes.c_int), ('upsample', ctypes.c_int),
        ('x2', vp), ('x2_pitch', ctypes.c_int), ('Cin2', ctypes.c_int),
        ('w', vp), ('K', ctypes.c_int),
        ('y', vp), ('y_pitch', ctypes.c_int), ('Cout', ctypes.c_int), ('B', ctypes.c_int),
        ('Hout', ctypes.c_int), ('Wout', ctypes.c_int),
        ('bias', vp), ('rowvec', vp), ('rowvec_pitch', ctypes.c_int),
        ('res', vp), ('res_pitch', ctypes.c_int),
        ('tile', ctypes.c_int),
        ('pro_scale', vp), ('pro_shift', vp),
        ('w_split', vp), ('w_split_kind', ctypes.c_int), ('range_flag', vp), ('pro_nosilu', ctypes.c_int),
        ('ksplit', ctypes.c_int), ('kpart', vp), ('w_wino', vp), ('w_wino_fold', ctypes.c_int),
    ]


class GemmDesc(ctypes.Structure):
    _fields_ = [
        ('M', ctypes.c_int), ('N', ctypes.c_int), ('K', ctypes.c_int), ('Z1', ctypes.c_int), ('Z2', ctypes.c_int),
        ('A', vp), ('a_s1', ctypes.c_int64), ('a_s2', ctypes.c_int64), ('lda', ctypes.c_int),
        ('B', vp), ('b_s1', ctypes.c_int64), ('b_s2', ctypes.c_int64), ('ldb', ctypes.c_int), ('b_kn', ctypes.c_int),
        ('C', vp), ('c_s1', ctypes.c_int64), ('c_s2', ctypes.c_int64), ('ldc', ctypes.c_int),
        ('alpha', ctypes.c_float),
        ('bias', vp),
        ('res', vp), ('ld_res', ctypes.c_int),
        ('act', ctypes.c_int),
        ('b_scale', ctypes.c_float),
        ('split', ctypes.c_int), ('split_ea', ctypes.c_int), ('split_eb', ctypes.c_int), ('range_flag', vp),
    ]


_lib: Optional[ctypes.CDLL] = None

# Batched classifier-free guidance marks the unconditional half of a 2B batch with label -1.
# That convention is private to the CFG samplers: a public forward with a negative label raises
# IndexError as nn.Embedding does upstream. The samplers open this scope around their 2B forward.
_null_label_depth = 0


class null_label_scope:
    """Context manager: inside it, native denoisers accept y[b] = -1 as "no label" for row b."""

    def __enter__(self):
        global _null_label_depth
        _null_label_depth += 1
        return self

    def __exit__(self, *exc):
        global _null_label_depth
        _null_label_depth -= 1
        return False


def null_labels_allowed() -> bool:
    return _null_label_depth > 0


class deferred_range_check:
    """Context manager over one sampling loop: native forwards inside it do not sync on the fp16x2
    range flag; on exit every model handle used inside is polled once (dm_*_range_poll) and
    ``flagged`` tells whether any forward met an activation beyond the fp16 range. Those models
    (``flagged_handles``) are then in fallback: their forwards run in the exact fallback arithmetic
    while the caller re-runs the loop, and ``end_fallback()`` returns them to fp16x2."""
    active = None

    def __init__(self):
        self.handles = {}
        self.flagged = False
        self.flagged_handles = []
        self._outer = None

    @staticmethod
    def _key(handle) -> int:
        return int(handle.value if isinstance(handle, ctypes.c_void_p) else handle)

    def register(self, handle, abi: str, device):
        key = self._key(handle)
        if key not in self.handles:
            check(getattr(load(), abi + '_set_range_deferred')(handle, 1), abi + '_set_range_deferred')
            self.handles[key] = (handle, abi, device)

    def _poll(self, handle, abi: str, device, poll: bool):
        L = load()
        check(getattr(L, abi + '_set_range_deferred')(handle, 0), abi + '_set_range_deferred')
        if poll:
            flag = ctypes.c_int()
            check(getattr(L, abi + '_range_poll')(handle, stream_handle(device), ctypes.byref(flag)),
                  abi + '_range_poll')
            if flag.value:
                self.flagged = True
                self.flagged_handles.append((handle, abi))

    @classmethod
    def release(cls, handle):
        """Called before a native handle is destroyed (NativeDenoiser._release_native): every open scope
        that registered it polls it now, folding a raised range flag into the scope (the loop is then
        re-run), and forgets it (also from the handles end_fallback returns to fp16x2) -- so no scope calls
        into a freed handle, and a new handle that reuses the address is registered afresh."""
        key = cls._key(handle)
        scope = cls.active
        while scope is not None:
            entry = scope.handles.pop(key, None)
            if entry is not None:
                scope._poll(*entry, poll=True)
            # the scope stays flagged (its loop re-runs), but end_fallback must not reach the freed handle
            scope.flagged_handles = [(h, a) for h, a in scope.flagged_handles if cls._key(h) != key]
            scope = scope._outer

    def __enter__(self):
        self._outer = deferred_range_check.active
        deferred_range_check.active = self
        return self

    def __exit__(self, exc_type, *exc):
        deferred_range_check.active = self._outer
        for handle, abi, device in self.handles.values():
            self._poll(handle, abi, device, poll=exc_type is None)
        self.handles.clear()
        if self._outer is not None and self.flagged:
            self._outer.flagged = True
            self._outer.flagged_handles.extend(self.flagged_handles)
            self.flagged_handles = []
        return False

    def end_fallback(self):
        """The re-run is done: the flagged models run fp16x2 again from their next forward."""
        for handle, abi in self.flagged_handles:
            check(getattr(load(), abi + '_range_fallback')(handle, 0), abi + '_range_fallback')
        self.flagged_handles = []


def _declare(L: ctypes.CDLL):
    L.dm_abi_version.restype = ctypes.c_int
    L.dm_last_error.restype = ctypes.c_char_p
    L.dm_build_info.restype = ctypes.c_char_p
    L.dm_unet_param_count.argtypes = [ctypes.POINTER(UNetArch), ctypes.POINTER(ctypes.c_int)]
    L.dm_unet_create.argtypes = [ctypes.POINTER(UNetArch), ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_int64),
                                 ctypes.c_int, vp, ctypes.POINTER(vp)]
    L.dm_unet_forward.argtypes = [vp, vp, vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp]
    L.dm_unet_profile.argtypes = [vp, ctypes.c_int]
    L.dm_unet_profile_count.argtypes = [vp, ctypes.POINTER(ctypes.c_int)]
    L.dm_unet_profile_get.argtypes = [vp, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                      ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)]
    L.dm_unet_memory.argtypes = [vp, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
    L.dm_unet_destroy.argtypes = [vp]
    L.dm_unet_destroy.restype = None
    L.dm_sampler_step.argtypes = [ctypes.POINTER(StepDesc), vp]
    L.dm_groupnorm_scratch_bytes.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
    L.dm_groupnorm_scratch_bytes.restype = ctypes.c_int64
    L.dm_groupnorm_nhwc.argtypes = [vp, ctypes.c_int, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_float, vp, vp, vp, vp, ctypes.c_int, ctypes.c_int, vp, vp]
    L.dm_groupnorm_affine.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_float, vp, vp, vp, vp, vp, vp]
    L.dm_pack_conv_weight.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, ctypes.c_int, ctypes.c_int,
                                      vp]
    L.dm_conv2d_nhwc.argtypes = [ctypes.POINTER(ConvDesc), vp]
    L.dm_pack_conv_weight_subpixel.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp, vp]
    L.dm_debug_launch_log.argtypes = [ctypes.c_int]
    L.dm_debug_launch_log_read.argtypes = [ctypes.c_char_p, ctypes.c_int]
    L.dm_conv_weight_wino_bytes.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
    L.dm_conv_weight_wino_bytes.restype = ctypes.c_int64
    L.dm_pack_conv_weight_wino.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp]
    L.dm_conv_weight_split_bytes.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    L.dm_conv_weight_split_bytes.restype = ctypes.c_int64
    L.dm_pack_conv_weight_split.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_int, vp, vp]
    L.dm_unet_set_conv_math.argtypes = [vp, ctypes.c_int]
    L.dm_unet_get_conv_math.argtypes = [vp, ctypes.POINTER(ctypes.c_int)]
    L.dm_unet_set_range_deferred.argtypes = [vp, ctypes.c_int]
    L.dm_unet_range_poll.argtypes = [vp, vp, ctypes.POINTER(ctypes.c_int)]
    L.dm_unet_range_fallback.argtypes = [vp, ctypes.c_int]
    L.dm_unet_range_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int)]
    L.dm_dit_range_fallback.argtypes = [vp, ctypes.c_int]
    L.dm_dit_range_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int)]
    L.dm_dit_set_range_deferred.argtypes = [vp, ctypes.c_int]
    L.dm_dit_range_poll.argtypes = [vp, vp, ctypes.POINTER(ctypes.c_int)]
    L.dm_dit_set_math.argtypes = [vp, ctypes.c_int]
    L.dm_dit_get_math.argtypes = [vp, ctypes.POINTER(ctypes.c_int)]
    L.dm_gemm.argtypes = [ctypes.POINTER(GemmDesc), vp]
    L.dm_softmax_rows.argtypes = [vp, ctypes.c_int64, ctypes.c_int, ctypes.c_int, vp]
    L.dm_timestep_embedding.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp, vp]
    L.dm_unet_set_time_freqs.argtypes = [vp, vp, ctypes.c_int, vp]
    L.dm_dit_param_count.argtypes = [ctypes.POINTER(DiTArch), ctypes.POINTER(ctypes.c_int)]
    L.dm_dit_create.argtypes = [ctypes.POINTER(DiTArch), ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_int64),
                                ctypes.c_int, vp, ctypes.POINTER(vp)]
    L.dm_dit_forward.argtypes = [vp, vp, vp, vp, ctypes.c_int, vp, vp]
    L.dm_dit_set_time_freqs.argtypes = [vp, vp, ctypes.c_int, vp]
    L.dm_dit_profile.argtypes = [vp, ctypes.c_int]
    L.dm_dit_profile_count.argtypes = [vp, ctypes.POINTER(ctypes.c_int)]
    L.dm_dit_profile_get.argtypes = [vp, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                     ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                     ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)]
    L.dm_dit_memory.argtypes = [vp, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
    L.dm_dit_destroy.argtypes = [vp]
    L.dm_dit_destroy.restype = None
    L.dm_unet_share_workspace.argtypes = [vp, vp]
    L.dm_unet_plan_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int)]
    L.dm_dit_plan_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int)]
    L.dm_lincomb.argtypes = [ctypes.c_int, vp, vp, vp, ctypes.c_int64, ctypes.c_int64, vp, vp, ctypes.c_float,
                             ctypes.c_float, vp]
    L.dm_comm_unique_id.argtypes = [vp]
    L.dm_comm_init.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]
    L.dm_comm_info.argtypes = [vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                               ctypes.POINTER(ctypes.c_int)]
    L.dm_allgather_f32.argtypes = [vp, vp, vp, ctypes.c_int64, vp]
    L.dm_comm_destroy.argtypes = [vp]
    L.dm_comm_destroy.restype = None


def load() -> ctypes.CDLL:
    """Load libdm_hip.so (built in-tree by __graft_entry__.build()). Raises if absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(lib_path):
            raise DMError(
                f'dm_hip native library not found at {lib_path}; build it with '
                f'`python -c "import __graft_entry__ as g; g.build()"` (no CPU fallback exists)')
        L = ctypes.CDLL(lib_path)
        _declare(L)
        if L.dm_abi_version() != ABI_VERSION:
            raise DMError(f'dm_hip ABI mismatch: library reports {L.dm_abi_version()}, binding expects {ABI_VERSION}')
        _lib = L
    return _lib


def lib() -> ctypes.CDLL:
    return load()


def exported_symbols():
    """Function names declared in include/dm_hip.h."""
    with open(_HEADER) as f:
        text = f.read()
    text = re.sub(r'/\*.*?\*/', '', text, flags=re.S)
    names = re.findall(r'\b(dm_[a-z0-9_]+)\s*\(', text)
    return sorted(set(names))


def check(rc: int, what: str = 'dm_hip call'):
    if rc == DM_OK:
        return
    msg = load().dm_last_error()
    msg = msg.decode() if msg else ''
    if rc == DM_ERR_ARG:
        raise ValueError(f'{what}: {msg}')
    raise DMError(f'{what} failed ({rc}): {msg}')


def require_device_tensor(t: torch.Tensor, name: str, dtype=torch.float32):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f'{name} must be a torch.Tensor')
    if t.device.type != 'cuda':
        raise RuntimeError(
            f'dm_hip: {name} is on {t.device}; the MI355X engine runs only on ROCm device tensors '
            f'(there is no CPU fallback)')
    if t.dtype != dtype:
        raise TypeError(f'dm_hip: {name} must be {dtype}, got {t.dtype}')
    if not t.is_contiguous():
        raise ValueError(f'dm_hip: {name} must be contiguous')


def stream_handle(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _p(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


# --------------------------------------------------------------------------- ops
def sampler_step(desc: StepDesc, device=None):
    check(load().dm_sampler_step(ctypes.byref(desc), stream_handle(device)), 'dm_sampler_step')


def groupnorm_nhwc(x: torch.Tensor, y: torch.Tensor, B: int, HW: int, C: int, G: int, eps: float,
                   gamma=None, beta=None, mod_scale=None, mod_shift=None, mod_pitch: int = 0, silu: bool = False,
                   x_pitch: int = None, y_pitch: int = None):
    L = load()
    nbytes = L.dm_groupnorm_scratch_bytes(B, HW, G)
    scratch = torch.empty(max(1, nbytes), dtype=torch.uint8, device=x.device)
    check(L.dm_groupnorm_nhwc(x.data_ptr(), x_pitch or C, y.data_ptr(), y_pitch or C, B, HW, C, G, eps,
                              _p(gamma), _p(beta), _p(mod_scale), _p(mod_shift), mod_pitch, int(silu),
                              scratch.data_ptr(), stream_handle(x.device)), 'dm_groupnorm_nhwc')


def groupnorm_affine(x: torch.Tensor, B: int, HW: int, C: int, G: int, eps: float, gamma=None, beta=None,
                     x_pitch: int = None):
    """-> (scale, shift) [B, C] float32 device tensors."""
    L = load()
    scratch = torch.empty(max(1, L.dm_groupnorm_scratch_bytes(B, HW, G)), dtype=torch.uint8, device=x.device)
    scale = torch.empty((B, C), device=x.device)
    shift = torch.empty((B, C), device=x.device)
    check(L.dm_groupnorm_affine(x.data_ptr(), x_pitch or C, B, HW, C, G, eps, _p(gamma), _p(beta),
                                scale.data_ptr(), shift.data_ptr(), scratch.data_ptr(), stream_handle(x.device)),
          'dm_groupnorm_affine')
    return scale, shift


def pack_conv_weight(w: torch.Tensor, out: torch.Tensor, ldw: int, col0: int = 0):
    Cout, Cin, kh, kw = w.shape
    check(load().dm_pack_conv_weight(w.data_ptr(), Cout, Cin, kh * kw, out.data_ptr(), ldw, col0,
                                     stream_handle(w.device)), 'dm_pack_conv_weight')


def pack_conv_weight_subpixel(w: torch.Tensor, out: torch.Tensor):
    """torch 3x3 weight [Cout][Cin][3][3] -> sub-pixel upsample weights [4][Cout][4 Cin] (conv upsample = 2)."""
    Cout, Cin, kh, kw = w.shape
    if (kh, kw) != (3, 3) or out.numel() != 16 * Cout * Cin:
        raise ValueError('sub-pixel packing needs a 3x3 weight and a [4, Cout, 4 Cin] output')
    check(load().dm_pack_conv_weight_subpixel(w.data_ptr(), Cout, Cin, out.data_ptr(), stream_handle(w.device)),
          'dm_pack_conv_weight_subpixel')


SPLIT_FP16X2 = 2  # DM_SPLIT_FP16X2
SPLIT_BF16X3 = 3  # DM_SPLIT_BF16X3
CONV_MATH = {'fp32': 0, 'fp16x2': SPLIT_FP16X2, 'bf16x3': SPLIT_BF16X3}


def pack_conv_weight_split(wp: torch.Tensor, nmat: int, Cin: int, taps: int, kind: int = SPLIT_BF16X3) -> torch.Tensor:
    """Packed fp32 conv weights [nmat * Cout, K] -> split slices (a uint8 device tensor) for
    ConvDesc.w_split with ConvDesc.w_split_kind = kind; taps 9, or 4 for sub-pixel weights (nmat = 4)."""
    rows, K = wp.shape
    Cout = rows // nmat
    nbytes = load().dm_conv_weight_split_bytes(nmat, Cout, K, kind)
    if nbytes <= 0 or Cout * nmat != rows:
        raise ValueError('split packing needs [nmat * Cout, K] weights with K a multiple of 16 and kind 2 or 3')
    out = torch.empty(nbytes, dtype=torch.uint8, device=wp.device)
    check(load().dm_pack_conv_weight_split(wp.data_ptr(), nmat, Cout, K, Cin, taps, kind, out.data_ptr(),
                                           stream_handle(wp.device)), 'dm_pack_conv_weight_split')
    return out


def pack_conv_weight_wino(wp: torch.Tensor, Cin: int, Cin2: int = 0, fold: bool = False) -> torch.Tensor:
    """Packed fp32 3x3 conv weights [Cout, 9 Cin + Cin2] (Cin2: the 1x1 shortcut segment) -> the Winograd F(2,3)
    weight images (a uint8 device tensor) for ConvDesc.w_wino (with ConvDesc.w_split of kind SPLIT_FP16X2);
    fold = True for a conv whose prologue has the SiLU (set ConvDesc.w_wino_fold alike)."""
    Cout, K = wp.shape
    nbytes = load().dm_conv_weight_wino_bytes(Cout, Cin, Cin2)
    if nbytes <= 0 or K != 9 * Cin + Cin2:
        raise ValueError('Winograd packing needs [Cout, 9 Cin + Cin2] weights, Cin % 32 == 0, Cin2 % 64 == 0')
    out = torch.empty(nbytes, dtype=torch.uint8, device=wp.device)
    check(load().dm_pack_conv_weight_wino(wp.data_ptr(), Cout, Cin, Cin2, int(bool(fold)), out.data_ptr(),
                                          stream_handle(wp.device)), 'dm_pack_conv_weight_wino')
    return out


def dit_math(handle, kind: Optional[str] = None) -> str:
    """Set (kind given) and return the GEMM arithmetic of a native DiT handle: 'fp16x2' (default) or
    'fp32' (dm_dit_set_math / dm_dit_get_math)."""
    L = load()
    kinds = {'fp32': 0, 'fp16x2': SPLIT_FP16X2}
    if kind is not None:
        if kind not in kinds:
            raise ValueError(f'DiT math must be one of {sorted(kinds)}')
        check(L.dm_dit_set_math(handle, kinds[kind]), 'dm_dit_set_math')
    k = ctypes.c_int()
    check(L.dm_dit_get_math(handle, ctypes.byref(k)), 'dm_dit_get_math')
    return {v: n for n, v in kinds.items()}[k.value]


def unet_conv_math(handle, kind: Optional[str] = None) -> str:
    """Set (kind given) and return the conv arithmetic of a native UNet handle: 'fp16x2' (default),
    'bf16x3' or 'fp32' (dm_unet_set_conv_math / dm_unet_get_conv_math)."""
    L = load()
    if kind is not None:
        if kind not in CONV_MATH:
            raise ValueError(f'conv math must be one of {sorted(CONV_MATH)}')
        check(L.dm_unet_set_conv_math(handle, CONV_MATH[kind]), 'dm_unet_set_conv_math')
    k = ctypes.c_int()
    check(L.dm_unet_get_conv_math(handle, ctypes.byref(k)), 'dm_unet_get_conv_math')
    return {v: n for n, v in CONV_MATH.items()}[k.value]


def conv2d_nhwc(desc: ConvDesc, device=None):
    check(load().dm_conv2d_nhwc(ctypes.byref(desc), stream_handle(device)), 'dm_conv2d_nhwc')


def gemm(desc: GemmDesc, device=None):
    check(load().dm_gemm(ctypes.byref(desc), stream_handle(device)), 'dm_gemm')


def softmax_rows(x: torch.Tensor, rows: int, L: int, ld: int):
    check(load().dm_softmax_rows(x.data_ptr(), rows, L, ld, stream_handle(x.device)), 'dm_softmax_rows')


def timestep_embedding(t: torch.Tensor, dim: int, kind: int, out: torch.Tensor, freqs: torch.Tensor = None):
    check(load().dm_timestep_embedding(t.data_ptr(), t.shape[0], dim, kind, _p(freqs), out.data_ptr(),
                                       stream_handle(t.device)), 'dm_timestep_embedding')


def unet_profile_enable(handle, enable, abi: str = 'dm_unet'):
    """Per-launch HIP-event profiling of a model's cached plan (abi: 'dm_unet' or 'dm_dit').
    enable: False/0 off, True/1 every forward, N > 1 every N-th forward."""
    check(getattr(load(), abi + '_profile')(handle, int(enable)), abi + '_profile')


def unet_profile_read(handle, abi: str = 'dm_unet'):
    """List of dicts (label, flops, bytes, ms_total, launches) for every op of the cached plan."""
    L = load()
    n = ctypes.c_int()
    check(getattr(L, abi + '_profile_count')(handle, ctypes.byref(n)), abi + '_profile_count')
    out = []
    buf = ctypes.create_string_buffer(128)
    fl, by, ms = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
    nl = ctypes.c_int64()
    get = getattr(L, abi + '_profile_get')
    for i in range(n.value):
        check(get(handle, i, buf, 128, ctypes.byref(fl), ctypes.byref(by), ctypes.byref(ms), ctypes.byref(nl)),
              abi + '_profile_get')
        out.append(dict(label=buf.value.decode(), flops=fl.value, bytes=by.value, ms_total=ms.value,
                        launches=nl.value))
    return out


def launch_log(enable: bool) -> None:
    """Start (clearing it) or stop the library's launch log: the kernel instantiations its conv launchers issue
    (dm_debug_launch_log; a hipGraph plan launches at capture, i.e. on the forward that builds the plan)."""
    check(load().dm_debug_launch_log(1 if enable else 0), 'dm_debug_launch_log')


def launch_log_read() -> list:
    """The kernel instantiations logged since launch_log(True), in launch order."""
    buf = ctypes.create_string_buffer(1 << 20)
    n = load().dm_debug_launch_log_read(buf, len(buf))
    if n < 0:
        raise RuntimeError('dm_debug_launch_log_read failed')
    return [ln for ln in buf.value.decode().split('\n') if ln]


def range_stats(handle, abi: str = 'dm_unet'):
    """(forwards / loops re-run in the fallback arithmetic so far, arithmetic of the next forward) of a native
    model handle (dm_unet_range_stats / dm_dit_range_stats)."""
    n, active = ctypes.c_int64(), ctypes.c_int()
    check(getattr(load(), abi + '_range_stats')(handle, ctypes.byref(n), ctypes.byref(active)), abi + '_range_stats')
    return n.value, {v: k for k, v in CONV_MATH.items()}[active.value]


def plan_stats(handle, abi: str = 'dm_unet'):
    """(plans built so far, plans cached) of a native model handle (dm_unet_plan_stats / dm_dit_plan_stats)."""
    builds, cached = ctypes.c_int64(), ctypes.c_int()
    check(getattr(load(), abi + '_plan_stats')(handle, ctypes.byref(builds), ctypes.byref(cached)),
          abi + '_plan_stats')
    return builds.value, cached.value


def share_workspace(a, b):
    """Let native UNet handle b run over a's plan scratch (forwards of a and b never overlap)."""
    check(load().dm_unet_share_workspace(a, b), 'dm_unet_share_workspace')


def lincomb(mode: int, a: torch.Tensor, b: torch.Tensor, c1, c2, out: torch.Tensor = None) -> torch.Tensor:
    """out = c1 a + c2 b (mode 0), c1 a - c2 b (1), (c1 a - b) / c2 (2) on device tensors of one shape;
    c1 / c2 are python floats (rounded to float32) or [B] float32 device tensors (one per image, dim 0)."""
    for name, t in (('a', a), ('b', b)):
        require_device_tensor(t, name)
    if a.shape != b.shape:
        raise ValueError(f'lincomb: shapes {tuple(a.shape)} and {tuple(b.shape)} differ')
    if out is None:
        out = torch.empty_like(a)
    else:
        require_device_tensor(out, 'out')
        if out.shape != a.shape:
            raise ValueError(f'lincomb: out has shape {tuple(out.shape)}, the operands {tuple(a.shape)}')
    B = a.shape[0] if a.ndim else 1
    row = a.numel() // B if B else 1

    def coef(c):
        if isinstance(c, torch.Tensor) and c.ndim == 1:
            require_device_tensor(c, 'coefficient')
            if c.shape != (B, ):
                raise ValueError(f'per-row coefficients must have shape ({B},), got {tuple(c.shape)}')
            return c.data_ptr(), 0.0
        return None, float(c)
    p1, s1 = coef(c1)
    p2, s2 = coef(c2)
    check(load().dm_lincomb(mode, a.data_ptr(), b.data_ptr(), out.data_ptr(), a.numel(), max(row, 1), p1, p2, s1, s2,
                            stream_handle(a.device)), 'dm_lincomb')
    return out


def source_hash() -> str:
    """sha256 (first 16 hex digits) of the library's sources in the Makefile's order: what dm_build_info
    reports for a library built from this tree."""
    import hashlib
    csrc = os.path.join(os.path.dirname(_HERE), 'csrc')
    with open(os.path.join(csrc, 'Makefile')) as f:
        mk = f.read()
    srcs = re.search(r'^SRCS := (.*)$', mk, re.M).group(1).split()
    hdrs = re.search(r'^HDRS := (.*)$', mk, re.M).group(1).split()
    h = hashlib.sha256()
    for name in srcs + hdrs:
        with open(os.path.join(csrc, name), 'rb') as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def build_info() -> str:
    return load().dm_build_info().decode()
