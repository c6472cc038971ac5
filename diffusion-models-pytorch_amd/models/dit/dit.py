"""Latent DiT wrapper (models/dit/dit.py:10-36, models/base_latent.py:6-28).

Same constructor (vae_config, vit_config, scale_factor) and forward
(x, timesteps, y=None) -> vit(x, timesteps, y); state_dict loads go to the
transformer, as upstream. The VAE (``AutoEncoderKL.from_pretrained``) is a
network download in the reference and is outside the denoising hot path, so
it is instantiated lazily, only when ``decode_latent`` is called.
"""
from typing import Any, Mapping

from torch import Tensor

from utils.misc import instantiate_from_config
from ..base_latent import BaseLatent


class DiT(BaseLatent):
    def __init__(self, vae_config, vit_config, scale_factor: float = 0.18215):
        super().__init__(scale_factor=scale_factor)
        self.vae_config = vae_config
        self.vae = None
        self.vit = instantiate_from_config(vit_config)

    @property
    def supports_null_label(self):
        return getattr(self.vit, 'supports_null_label', False)

    def decode_latent(self, z: Tensor):
        if self.vae is None:
            self.vae = instantiate_from_config(self.vae_config)
        z = 1. / self.scale_factor * z
        return self.vae.decode(z).sample

    def vit_forward(self, x: Tensor, t: Tensor, y: Tensor):
        return self.vit(x, t, y)

    def forward(self, x: Tensor, timesteps: Tensor, y: Tensor = None):
        return self.vit_forward(x, timesteps, y)

    def load_state_dict(self, state_dict: Mapping[str, Any], strict: bool = True, assign: bool = False):
        return self.vit.load_state_dict(state_dict, strict=strict, assign=assign)
