"""Latent-model marker (reference models/base_latent.py:6-24).

Samplers and scripts tell latent denoisers from pixel ones with
``isinstance(model, BaseLatent)`` (as the reference's Streamlit page does,
streamlit/pages/2_Class_conditional_Image_Generation.py:83,90-95): their noise
is drawn at (4, img_size / 8, img_size / 8) and samples are latents that
``decode_latent`` turns into images.
"""
import torch
import torch.nn as nn
from torch import Tensor


class BaseLatent(nn.Module):
    def __init__(self, scale_factor: float = 1.0):
        super().__init__()
        self.register_buffer('scale_factor', torch.tensor(scale_factor))
        self.device = self.scale_factor.device

    def to(self, *args, **kwargs):
        super().to(*args, **kwargs)
        self.device = self.scale_factor.device
        return self

    def forward(self, x: Tensor, timesteps: Tensor):
        raise NotImplementedError

    def encode_latent(self, x: Tensor):
        raise NotImplementedError

    def decode_latent(self, z: Tensor):
        raise NotImplementedError
