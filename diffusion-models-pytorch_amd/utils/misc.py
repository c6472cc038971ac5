"""Harness helpers restated from the reference utils/misc.py:27-78.

The reference builds configs with OmegaConf (absent here); `load_config`
reproduces the subset the sampling scripts use (YAML file + `a.b=v` dotlist
overrides) on PyYAML, returning attribute-accessible dicts.
"""
import importlib
import math
from typing import Any, Dict, List

import torch
import yaml


def image_norm_to_float(image: torch.Tensor):
    """[-1, 1] -> [0, 1] (reference utils/misc.py:27-31)."""
    assert image.dtype == torch.float32
    assert torch.ge(image, -1).all() and torch.le(image, 1).all()
    return (image + 1) / 2


def amortize(n_samples: int, batch_size: int) -> List[int]:
    """Split n_samples into folds of batch_size plus a remainder (utils/misc.py:41-44)."""
    full, rest = divmod(n_samples, batch_size)
    return [batch_size] * full + ([rest] if rest else [])


class AttrDict(dict):
    def __getattr__(self, item):
        try:
            return self[item]
        except KeyError as e:
            raise AttributeError(item) from e

    def __setattr__(self, key, value):
        self[key] = value


def _wrap(obj):
    if isinstance(obj, dict):
        return AttrDict({k: _wrap(v) for k, v in obj.items()})
    if isinstance(obj, list):
        return [_wrap(v) for v in obj]
    return obj


def _unwrap(obj):
    if isinstance(obj, dict):
        return {k: _unwrap(v) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_unwrap(v) for v in obj]
    return obj


def apply_dotlist(conf: Dict[str, Any], dotlist: List[str]):
    for item in dotlist:
        key, _, raw = item.partition('=')
        value = yaml.safe_load(raw) if raw != '' else None
        node = conf
        parts = key.split('.')
        for p in parts[:-1]:
            node = node.setdefault(p, AttrDict())
        node[parts[-1]] = _wrap(value)
    return conf


def load_config(path: str, dotlist: List[str] = ()):
    with open(path) as f:
        conf = _wrap(yaml.safe_load(f))
    return apply_dotlist(conf, list(dotlist))


def instantiate_from_config(conf, **extra_params):
    """Build `target` with `params` (reference utils/misc.py:71-78)."""
    conf = _unwrap(conf)
    module, cls = conf['target'].rsplit('.', 1)
    cls = getattr(importlib.import_module(module, package=None), cls)
    params = conf.get('params', dict()) or dict()
    params.update(extra_params)
    return cls(**params)
