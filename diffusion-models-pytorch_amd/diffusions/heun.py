"""Heun sampler on the MI355X engine (reference diffusions/heun.py:11-131).

Second-order (trapezoidal) correction of the Euler step: two denoiser forwards per step except the last.
Both stages are one fused kernel each (dm_sampler_step, euler = 1 / 2); the first stage also writes the
derivative, which the second stage averages with its own.
"""
from typing import Dict

import torch
import tqdm
from torch import Tensor

from diffusions.euler import EulerSampler


class HeunSampler(EulerSampler):
    def __init__(self, *args, **kwargs):
        """Heun sampler for DDPM-like diffusion process (arguments as reference heun.py:12-49)."""
        super().__init__(*args, **kwargs)
        self._1st_order_derivative = None
        self._1st_order_xt = None

    def denoise_1st_order(self, model_output: Tensor, xt: Tensor, t: int, t_prev: int):
        """1st order step, same as the Euler sampler (heun.py:56-77)."""
        derivative = torch.empty_like(xt)
        out = self._first_order(model_output, xt, t, t_prev, derivative=derivative)
        self._1st_order_derivative = derivative
        self._1st_order_xt = xt
        return {'sample': out['sample'], 'pred_x0': out['pred_x0']}

    def denoise_2nd_order(self, model_output: Tensor, xt_prev: Tensor, t: int, t_prev: int):
        """2nd order step (heun.py:79-106): x0 predicted at t_prev from x_{t-1}."""
        if self._1st_order_derivative is None:
            raise RuntimeError('denoise_2nd_order needs a preceding denoise_1st_order')
        c = dict(self._predict_coefs(t_prev))
        c.update(coef1=0.0, coef2=0.0, std=0.0, min_logvar=0.0, max_logvar=0.0)
        out = self._step(model_output, xt_prev, t_prev, t_prev - 1, coefs=c, euler=2,
                         ecoefs=self._euler_coefs(t, t_prev), d1=self._1st_order_derivative,
                         x1=self._1st_order_xt)
        self._1st_order_derivative = None
        self._1st_order_xt = None
        return {'sample': out['sample'], 'pred_x0': out['pred_x0']}

    def sample_loop(
            self, model, init_noise: Tensor,
            tqdm_kwargs: Dict = None, model_kwargs: Dict = None,
    ):
        """heun.py:108-131: a 1st-order step, then (unless t_prev < 0) a 2nd-order correction."""
        tqdm_kwargs = dict() if tqdm_kwargs is None else tqdm_kwargs
        model_kwargs = dict() if model_kwargs is None else model_kwargs
        img = init_noise
        seq = self.respaced_seq.tolist()
        seq_prev = [-1] + seq[:-1]
        pbar = tqdm.tqdm(total=len(seq), **tqdm_kwargs)
        for t, t_prev in zip(reversed(seq), reversed(seq_prev)):
            t_batch = torch.full((img.shape[0], ), t, device=img.device, dtype=torch.long)
            model_output = model(img, t_batch, **model_kwargs)
            out = self.denoise_1st_order(model_output, img, t, t_prev)
            img = out['sample']
            if t_prev >= 0:
                t_prev_batch = torch.full((img.shape[0], ), t_prev, device=img.device, dtype=torch.long)
                model_output = model(img, t_prev_batch, **model_kwargs)
                out = self.denoise_2nd_order(model_output, img, t, t_prev)
                img = out['sample']
            pbar.update(1)
            yield out
        pbar.close()
