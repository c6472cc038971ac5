"""DDIM sampler (and DDIM inversion) on the MI355X engine.

Mirrors the reference diffusions/ddim.py:12-250. The update reuses the fused
dm_sampler_step kernel with kind = DDIM; the coefficients are the reference's
torch CPU 0-dim expressions (ddim.py:65-73, 99-103).
"""
from typing import Any, Dict

import torch
import tqdm
from torch import Tensor

from diffusions.ddpm import DDPM, _CFGMixin


class DDIM(DDPM):
    kind = 0

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
            eta: float = 0.,

            device: torch.device = 'cpu',
            **kwargs,
    ):
        """Denoising Diffusion Implicit Models (Song et al. 2020). `eta` as upstream."""
        super().__init__(
            total_steps=total_steps, beta_schedule=beta_schedule, beta_start=beta_start, beta_end=beta_end,
            betas=betas, objective=objective, clip_denoised=clip_denoised, respace_type=respace_type,
            respace_steps=respace_steps, respaced_seq=respaced_seq, device=device, **kwargs,
        )
        self.eta = eta

    def _update_coefs(self, t: int, t_prev: int):
        ac_t = self._ac(t)
        ac_p = self._ac(t_prev) if t_prev >= 0 else torch.tensor(1.0)
        var = ((self.eta ** 2) *
               (1. - ac_p) / (1. - ac_t) *
               (1. - ac_t / ac_p))
        return dict(coef1=torch.sqrt(ac_p).item(), coef2=torch.sqrt(1. - ac_p - var).item(),
                    var_mode=0, std=torch.sqrt(var).item(), var_scalar=var, min_logvar=0.0, max_logvar=0.0)

    def _inversion_coefs(self, t: int, t_next: int):
        key = ('inv', t, t_next, self.objective)
        c = self._coef_cache.get(key)
        if c is None:
            ac_n = self._ac(t_next) if t_next < self.total_steps else torch.tensor(0.0)
            c = dict(self._predict_coefs(t))
            c.update(coef1=torch.sqrt(ac_n).item(), coef2=torch.sqrt(1. - ac_n).item(), var_mode=0, std=0.0,
                     var_scalar=torch.tensor(0.0), min_logvar=0.0, max_logvar=0.0)
            self._coef_cache[key] = c
        return c

    def denoise_inversion(self, model_output: Tensor, xt: Tensor, t: int, t_next: int,
                          model_output_uncond: Tensor = None, guidance_scale: float = 1.0):
        """x_{t_next} from x_t, valid for eta = 0 only (reference ddim.py:88-104)."""
        if self.eta != 0.:
            raise ValueError(f'DDIM inversion is only valid when eta=0, get {self.eta}')
        out = self._step(model_output, xt, t, 0, model_output_uncond=model_output_uncond,
                         guidance_scale=guidance_scale, want_noise=False, coefs=self._inversion_coefs(t, t_next))
        return {'sample': out['sample'], 'pred_x0': out['pred_x0'], 'pred_eps': out['pred_eps']}

    def sample_inversion_loop(
            self, model, img: Tensor,
            tqdm_kwargs: Dict = None, model_kwargs: Dict = None,
    ):
        tqdm_kwargs = dict() if tqdm_kwargs is None else tqdm_kwargs
        model_kwargs = dict() if model_kwargs is None else model_kwargs
        seq = self.respaced_seq.tolist()
        pbar = tqdm.tqdm(total=len(seq) - 1, **tqdm_kwargs)
        for t, t_next in zip(seq[:-1], seq[1:]):
            t_batch = torch.full((img.shape[0], ), t, device=img.device, dtype=torch.long)
            model_output = model(img, t_batch, **model_kwargs)
            out = self.denoise_inversion(model_output, img, t, t_next)
            img = out['sample']
            pbar.update(1)
            yield out
        pbar.close()

    def sample_inversion(
            self, model, img: Tensor,
            tqdm_kwargs: Dict = None, model_kwargs: Dict = None,
    ):
        sample = None
        for out in self.sample_inversion_loop(model, img, tqdm_kwargs, model_kwargs):
            sample = out['sample']
        return sample


class DDIMCFG(_CFGMixin, DDIM):
    def __init__(self, guidance_scale: float = 1., cond_kwarg: str = 'y', *args, **kwargs):
        """DDIM with classifier-free guidance (reference ddim.py:135-250)."""
        DDIM.__init__(self, *args, **kwargs)
        self._cfg_init(guidance_scale, cond_kwarg)

    def sample_inversion_loop(
            self, model, img: Tensor, uncond_conditioning: Any = None,
            tqdm_kwargs: Dict = None, model_kwargs: Dict = None,
    ):
        tqdm_kwargs = dict() if tqdm_kwargs is None else tqdm_kwargs
        model_kwargs = dict() if model_kwargs is None else model_kwargs
        if self.cond_kwarg not in model_kwargs.keys():
            raise ValueError(f'Condition argument `{self.cond_kwarg}` not found in model_kwargs.')
        uncond_kwargs = dict(model_kwargs)
        uncond_kwargs[self.cond_kwarg] = uncond_conditioning
        seq = self.respaced_seq.tolist()
        pbar = tqdm.tqdm(total=len(seq) - 1, **tqdm_kwargs)
        for t, t_next in zip(seq[:-1], seq[1:]):
            t_batch = torch.full((img.shape[0], ), t, device=img.device, dtype=torch.long)
            out_c = model(img, t_batch, **model_kwargs)
            out_u = model(img, t_batch, **uncond_kwargs)
            out = self.denoise_inversion(out_c, img, t, t_next, model_output_uncond=out_u,
                                         guidance_scale=self.guidance_scale)
            img = out['sample']
            pbar.update(1)
            yield out
        pbar.close()

    def sample_inversion(
            self, model, img: Tensor,
            clip_denoised: bool = None, eta: float = None,
            guidance_scale: float = None, uncond_conditioning: Any = None,
            tqdm_kwargs: Dict = None, model_kwargs: Dict = None,
    ):
        sample = None
        for out in self.sample_inversion_loop(model, img, uncond_conditioning, tqdm_kwargs, model_kwargs):
            sample = out['sample']
        return sample
