"""Euler sampler on the MI355X engine (reference diffusions/euler.py:7-66).

Karras et al. (2022) first-order ODE step on the VP schedule, sigma_t = sqrt((1 - ac_t) / ac_t):
    bar_xt = sqrt(1 + sigma_t^2) * xt,  d = (bar_xt - x0) / sigma_t,
    sample = (bar_xt + d * (sigma_prev - sigma_t)) / sqrt(1 + sigma_prev^2).
The 0-dim float32 scalars are computed on the host with the reference's torch expressions (as for DDPM);
predict + update run as one fused kernel (dm_sampler_step, euler = 1).
"""
import torch
from torch import Tensor

from diffusions.ddpm import DDPM


class EulerSampler(DDPM):
    def __init__(
            self,
            total_steps: int = 1000,
            beta_schedule: str = 'linear',
            beta_start: float = 0.0001,
            beta_end: float = 0.02,
            betas: Tensor = None,
            objective: str = 'pred_eps',

            clip_denoised: bool = True,
            respace_type: str = None,
            respace_steps: int = 100,
            respaced_seq: Tensor = None,

            device: torch.device = 'cpu',
            **kwargs,
    ):
        """Euler sampler for DDPM-like diffusion process (arguments as reference euler.py:8-46)."""
        super().__init__(
            total_steps=total_steps,
            beta_schedule=beta_schedule,
            beta_start=beta_start,
            beta_end=beta_end,
            betas=betas,
            objective=objective,
            clip_denoised=clip_denoised,
            respace_type=respace_type,
            respace_steps=respace_steps,
            respaced_seq=respaced_seq,
            device=device,
            **kwargs,
        )
        # euler.py:48 (elementwise float32: IEEE, host-independent)
        self._sig_cpu = ((1 - self._ac_cpu) / self._ac_cpu).sqrt()
        self.sigmas = self._sig_cpu.to(device)

    def _euler_coefs(self, t: int, t_prev: int) -> dict:
        """0-dim float32 scalars of euler.py:53-63 / heun.py:59-98, same torch CPU expressions."""
        key = ('euler', t, t_prev)
        c = self._coef_cache.get(key)
        if c is None:
            sigmas_t = self._sig_cpu[t]
            sigmas_t_prev = self._sig_cpu[t_prev] if t_prev >= 0 else torch.tensor(0.0)
            c = dict(st1=(1 + sigmas_t ** 2).sqrt().item(), sp1=(1 + sigmas_t_prev ** 2).sqrt().item(),
                     dsig=(sigmas_t_prev - sigmas_t).item(), sig_t=sigmas_t.item(), sig_p=sigmas_t_prev.item())
            self._coef_cache[key] = c
        return c

    def _first_order(self, model_output: Tensor, xt: Tensor, t: int, t_prev: int, derivative: Tensor = None):
        c = dict(self._predict_coefs(t))
        c.update(coef1=0.0, coef2=0.0, std=0.0, min_logvar=0.0, max_logvar=0.0)
        return self._step(model_output, xt, t, t_prev, coefs=c, euler=1, ecoefs=self._euler_coefs(t, t_prev),
                          dout=derivative)

    def denoise(self, model_output: Tensor, xt: Tensor, t: int, t_prev: int):
        """Denoise from x_t to x_{t-1} (euler.py:50-66)."""
        out = self._first_order(model_output, xt, t, t_prev)
        return {'sample': out['sample'], 'pred_x0': out['pred_x0']}
