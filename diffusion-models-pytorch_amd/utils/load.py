"""Checkpoint loading with the reference's key conventions (utils/load.py:7-19).

Only safe loaders are used: safetensors, or torch.load(weights_only=True).
"""
import os

import torch


def load_weights(path: str):
    if os.path.splitext(path)[-1] == '.safetensors':
        from safetensors.torch import load_file
        return load_file(path, device='cpu')
    ckpt = torch.load(path, map_location='cpu', weights_only=True)
    for key in ('state_dict', 'ema', 'model'):
        if key in ckpt:
            return ckpt['ema']['shadow'] if key == 'ema' else ckpt[key]
    return ckpt
