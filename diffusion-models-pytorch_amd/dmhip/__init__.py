"""ctypes binding of the dm_hip C ABI (include/dm_hip.h).

The product path has no CPU fallback: every entry point requires the native
library and ROCm device tensors, and raises loudly otherwise.
"""
from dmhip._lib import (  # noqa: F401
    DMError,
    lib,
    lib_path,
    load,
    exported_symbols,
    require_device_tensor,
    stream_handle,
    StepDesc,
    ConvDesc,
    GemmDesc,
    UNetArch,
    DiTArch,
    sampler_step,
    groupnorm_nhwc,
    groupnorm_affine,
    conv2d_nhwc,
    pack_conv_weight,
    pack_conv_weight_subpixel,
    pack_conv_weight_split,
    unet_conv_math,
    dit_math,
    SPLIT_FP16X2,
    SPLIT_BF16X3,
    gemm,
    softmax_rows,
    timestep_embedding,
    unet_profile_enable,
    unet_profile_read,
    null_label_scope,
    null_labels_allowed,
    deferred_range_check,
)
