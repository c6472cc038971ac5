"""UNetCombined (models/adm/unet_combined.py:6-32) on the MI355X engine.

A conditional and an unconditional ADM UNetModel under one module; forward
routes y=None to ``unet_uncond`` and everything else to ``unet_cond``, so the
classifier-free-guidance samplers run the two branches through the two
weight sets. State_dict names (``unet_cond.*``, ``unet_uncond.*``) match the
reference, so combined checkpoints load unchanged.
"""
import weakref

import torch
import torch.nn as nn

from .unet import UNetModel


class UNetCombined(nn.Module):
    def __init__(self, *args, **kwargs):
        super().__init__()
        assert kwargs.get('num_classes') is not None
        self.unet_cond = UNetModel(*args, **kwargs)
        kwargs_uncond = kwargs.copy()
        kwargs_uncond.update({'num_classes': None})
        self.unet_uncond = UNetModel(*args, **kwargs_uncond)
        # one plan workspace for both networks (weak links, not submodules); forwards of the two on different
        # streams are serialised by the engine over that workspace (dm_unet_share_workspace)
        self.unet_cond.__dict__['_ws_peer'] = weakref.ref(self.unet_uncond)
        self.unet_uncond.__dict__['_ws_peer'] = weakref.ref(self.unet_cond)

    def forward(self, x, timesteps, y=None):
        unet = self.unet_uncond if y is None else self.unet_cond
        return unet(x, timesteps, y)

    def combine_weights(self, cond_path, uncond_path, save_path):
        """Merge two single-model checkpoints (tensor-only loads) into one combined state_dict."""
        self.unet_cond.load_state_dict(torch.load(cond_path, map_location='cpu', weights_only=True))
        self.unet_uncond.load_state_dict(torch.load(uncond_path, map_location='cpu', weights_only=True))
        torch.save(self.state_dict(), save_path)
