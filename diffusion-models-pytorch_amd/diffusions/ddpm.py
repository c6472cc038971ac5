"""DDPM sampler with the per-step update on the MI355X engine.

Public API and semantics follow the reference diffusions/ddpm.py:13-368
(constructor arguments, ValueError cases, `alphas_cumprod`, `respaced_seq`,
`predict`, `denoise`, `sample_loop`, `sample`, the CFG subclass).

What differs is where the arithmetic runs:
  * scalar coefficients are computed once per (t, t_prev) on the host with the
    reference's own torch CPU 0-dim expressions (ddpm.py:102-120, 222-248) —
    torch's float32 sqrt/pow are not IEEE-rounded, so computing them any
    other way would break bit-parity — and cached;
  * the elementwise work (predict, clamp, eps recompute, CFG combine, mean,
    variance, noise) is ONE fused HIP kernel (dm_sampler_step) per step.
The model output must be a ROCm device tensor; there is no CPU fallback.
"""
import math
from contextlib import contextmanager
from typing import Any, Callable, Dict, Optional

import torch
import tqdm
from torch import Tensor

import dmhip
from diffusions.schedule import get_beta_schedule, get_respaced_seq

_OBJECTIVES = {'pred_eps': 0, 'pred_x0': 1, 'pred_v': 2}
_VAR_TYPES = ('fixed_small', 'fixed_large', 'learned_range')


class DDPM:
    kind = 1  # dm_step_desc.kind

    def __init__(
            self,
            total_steps: int = 1000,
            beta_schedule: str = 'linear',
            beta_start: float = 0.0001,
            beta_end: float = 0.02,
            betas: Tensor = None,
            objective: str = 'pred_eps',

            var_type: str = 'fixed_large',
            clip_denoised: bool = True,
            respace_type: str = None,
            respace_steps: int = 100,
            respaced_seq: Tensor = None,

            device: torch.device = 'cpu',
    ):
        """Denoising Diffusion Probabilistic Models (Ho et al. 2020; Nichol & Dhariwal 2021).

        Arguments as in the reference (diffusions/ddpm.py:14-58).
        """
        if objective not in _OBJECTIVES:
            raise ValueError(f'Invalid objective: {objective}')
        if var_type not in _VAR_TYPES:
            raise ValueError(f'Invalid var_type: {var_type}')
        self.total_steps = total_steps
        self.objective = objective
        self.var_type = var_type
        self.clip_denoised = clip_denoised
        self.device = device

        if betas is None:
            betas = get_beta_schedule(total_steps=total_steps, beta_schedule=beta_schedule,
                                      beta_start=beta_start, beta_end=beta_end)
        assert isinstance(betas, Tensor)
        assert betas.shape == (total_steps, )
        # cumprod in the schedule's dtype (float64 except cosine), then float32
        ac = torch.cumprod(1. - betas, dim=0).to(torch.float)
        self._ac_cpu = ac.cpu()
        self.alphas_cumprod = ac.to(device)

        if respaced_seq is None:
            respaced_seq = get_respaced_seq(total_steps=total_steps, respace_type=respace_type,
                                            respace_steps=respace_steps)
        assert isinstance(respaced_seq, Tensor)
        assert respaced_seq.ndim == 1
        self.respaced_seq = respaced_seq.to(device)

        # Noise source for the stochastic part of the update. Default: the
        # device generator (torch.randn_like on xt's device), as upstream.
        # Parity runs install a CPU-generator source here.
        self.noise_fn: Optional[Callable[[Tensor], Tensor]] = None
        # The reference draws reverse_eps every step even when it is
        # multiplied by zero (DDIM eta=0, t=0; ddim.py:76, ddpm.py:251), which
        # moves the RNG stream (later folds' init noise depends on it). The
        # default does the same; True skips the unused draw (the output is
        # unchanged, reverse_eps is then None).
        self.skip_unused_noise = False
        self._coef_cache: Dict[Any, dict] = {}

    # ------------------------------------------------------------------ setup
    def set_respaced_seq(self, respace_type: str = 'uniform', respace_steps: int = 100):
        self.respaced_seq = get_respaced_seq(total_steps=self.total_steps, respace_type=respace_type,
                                             respace_steps=respace_steps).to(self.device)

    # ------------------------------------------------- host scalar arithmetic
    def _ac(self, t: int):
        return self._ac_cpu[t]

    def _predict_coefs(self, t: int):
        """0-dim float32 coefficients of ddpm.py:102-120 (same torch CPU ops)."""
        ac_t = self._ac(t)
        return dict(
            sqrt_recip_ac=((1. / ac_t) ** 0.5).item(),
            sqrt_recipm1_ac=((1. / ac_t - 1.) ** 0.5).item(),
            sqrt_ac=(ac_t ** 0.5).item(),
            sqrt_one_minus_ac=((1. - ac_t) ** 0.5).item(),
        )

    def _update_coefs(self, t: int, t_prev: int):
        """Mean / variance coefficients of ddpm.py:222-248."""
        ac_t = self._ac(t)
        ac_p = self._ac(t_prev) if t_prev >= 0 else torch.tensor(1.0)
        alphas_t = ac_t / ac_p
        betas_t = 1. - alphas_t
        mean_coef1 = (ac_p ** 0.5) * betas_t / (1. - ac_t)
        mean_coef2 = (alphas_t ** 0.5) * (1. - ac_p) / (1. - ac_t)
        c = dict(coef1=mean_coef1.item(), coef2=mean_coef2.item(), var_mode=0, std=0.0,
                 min_logvar=0.0, max_logvar=0.0)
        if t == 0:
            var = torch.zeros_like(betas_t)
        elif self.var_type == 'fixed_small':
            var = betas_t * (1. - ac_p) / (1. - ac_t)
        elif self.var_type == 'fixed_large':
            var = betas_t
        elif self.var_type == 'learned_range':
            min_var = betas_t * (1. - ac_p) / (1. - ac_t)
            c['min_logvar'] = torch.log(torch.clamp_min(min_var, 1e-20)).item()
            c['max_logvar'] = torch.log(betas_t).item()
            c['var_mode'] = 1
            var = None
        else:
            raise ValueError(f'Invalid var_type: {self.var_type}')
        if var is not None:
            c['std'] = torch.sqrt(var).item()
            c['var_scalar'] = var
        return c

    def _coefs(self, t: int, t_prev: int):
        key = (t, t_prev, self.objective, self.var_type, getattr(self, 'eta', None))
        c = self._coef_cache.get(key)
        if c is None:
            c = dict(self._predict_coefs(t))
            c.update(self._update_coefs(t, t_prev))
            self._coef_cache[key] = c
        return c

    # ------------------------------------------------ closed-form conversions
    # Reference ddpm.py:102-120, 140-172. The coefficients are the reference's torch CPU expressions
    # (0-dim for an int t, [B] vectors for per-image timesteps), the elementwise arithmetic one
    # dm_lincomb launch with separately rounded float32 products (bit-identical to the CPU expression).
    # Non-contiguous tensor arguments are accepted, as by the reference's torch expressions.
    def _row_coefs(self, t, x: Tensor):
        """sqrt(ac_t), sqrt(1 - ac_t) for t: an int / 0-dim tensor (scalars) or [B] timesteps (one per image)."""
        if isinstance(t, Tensor) and t.ndim >= 1:
            tc = t.detach().to('cpu', torch.long).reshape(-1)
            if tc.numel() != x.shape[0]:
                raise ValueError(f't must hold one timestep per image ({x.shape[0]}), got {tc.numel()}')
            a = self._ac_cpu[tc]
            return (a ** 0.5).to(x.device), ((1. - a) ** 0.5).to(x.device)
        c = self._predict_coefs(int(t))
        return c['sqrt_ac'], c['sqrt_one_minus_ac']

    def pred_x0_from_eps(self, xt: Tensor, t: int, eps: Tensor):
        c = self._predict_coefs(int(t))
        return dmhip.lincomb(1, xt.contiguous(), eps.contiguous(), c['sqrt_recip_ac'], c['sqrt_recipm1_ac'])

    def pred_eps_from_x0(self, xt: Tensor, t: int, x0: Tensor):
        c = self._predict_coefs(int(t))
        return dmhip.lincomb(2, xt.contiguous(), x0.contiguous(), c['sqrt_recip_ac'], c['sqrt_recipm1_ac'])

    def pred_x0_from_v(self, xt: Tensor, t: int, v: Tensor):
        c = self._predict_coefs(int(t))
        return dmhip.lincomb(1, xt.contiguous(), v.contiguous(), c['sqrt_ac'], c['sqrt_one_minus_ac'])

    def pred_eps_from_v(self, xt: Tensor, t: int, v: Tensor):
        c = self._predict_coefs(int(t))
        return dmhip.lincomb(0, xt.contiguous(), v.contiguous(), c['sqrt_one_minus_ac'], c['sqrt_ac'])

    def get_v(self, x0: Tensor, eps: Tensor, t: Tensor):
        """v = sqrt(ac_t) eps - sqrt(1 - ac_t) x0 (reference ddpm.py:140-150)."""
        sa, s1m = self._row_coefs(t, x0)
        return dmhip.lincomb(1, eps.contiguous(), x0.contiguous(), sa, s1m)

    def diffuse(self, x0: Tensor, t: Tensor, eps: Tensor = None):
        """Sample from q(x_t | x0) = sqrt(ac_t) x0 + sqrt(1 - ac_t) eps (reference ddpm.py:152-172);
        t holds one timestep per image (or one int for all), eps defaults to torch.randn_like(x0)."""
        eps = torch.randn_like(x0) if eps is None else eps
        sa, s1m = self._row_coefs(t, x0)
        return dmhip.lincomb(0, x0.contiguous(), eps.contiguous(), sa, s1m)

    # ------------------------------------------------------------- the step
    def _draw_noise(self, xt: Tensor, needed: bool) -> Optional[Tensor]:
        if not needed and self.skip_unused_noise:
            return None
        if self.noise_fn is not None:
            noise = self.noise_fn(xt)
        else:
            noise = torch.randn_like(xt)
        if noise.device != xt.device or noise.dtype != torch.float32 or not noise.is_contiguous():
            noise = noise.to(device=xt.device, dtype=torch.float32).contiguous()
        return noise

    def _step(self, model_output: Tensor, xt: Tensor, t: int, t_prev: int,
              model_output_uncond: Tensor = None, guidance_scale: float = 1.0,
              objective: str = None, want_noise: bool = True, predict_only: bool = False,
              coefs: dict = None, euler: int = 0, ecoefs: dict = None, d1: Tensor = None, x1: Tensor = None,
              dout: Tensor = None):
        dmhip.require_device_tensor(xt, 'xt')
        dmhip.require_device_tensor(model_output, 'model_output')
        if model_output_uncond is not None:
            dmhip.require_device_tensor(model_output_uncond, 'model_output_uncond')
        B, C = xt.shape[0], xt.shape[1]
        HW = xt[0, 0].numel() if xt.ndim > 2 else 1
        Cm = model_output.shape[1]
        if model_output.shape[0] != B or model_output.shape[2:] != xt.shape[2:] or Cm not in (C, 2 * C):
            raise ValueError(f'model output shape {tuple(model_output.shape)} does not match xt {tuple(xt.shape)}')
        c = coefs if coefs is not None else self._coefs(t, t_prev)
        learned = (not predict_only) and not euler and self.var_type == 'learned_range' and self.kind == 1 and t != 0
        if learned and Cm != 2 * C:
            raise ValueError('var_type learned_range requires the model to output 2C channels')
        add_noise = (not predict_only) and not euler and t != 0
        needed = add_noise and (learned or c['std'] != 0.0)
        noise = self._draw_noise(xt, needed) if want_noise and not predict_only else None

        sample = torch.empty_like(xt)
        mean = torch.empty_like(xt)
        x0 = torch.empty_like(xt)
        eps = torch.empty_like(xt)
        var_t = torch.empty_like(xt) if learned else None
        d = dmhip.StepDesc()
        d.B, d.C, d.HW, d.Cm = B, C, HW, Cm
        d.xt = xt.data_ptr()
        d.model_out = model_output.data_ptr()
        d.model_out_uncond = model_output_uncond.data_ptr() if model_output_uncond is not None else None
        d.w_uncond = 1 - guidance_scale   # ctypes rounds to float32, as torch does for the python scalar
        d.w_cond = guidance_scale
        d.objective = _OBJECTIVES[objective or self.objective]
        d.clip_denoised = int(bool(self.clip_denoised))
        d.sqrt_recip_ac = c['sqrt_recip_ac']
        d.sqrt_recipm1_ac = c['sqrt_recipm1_ac']
        d.sqrt_ac = c['sqrt_ac']
        d.sqrt_one_minus_ac = c['sqrt_one_minus_ac']
        d.kind = self.kind
        d.coef1, d.coef2 = c['coef1'], c['coef2']
        d.var_mode = 1 if learned else 0
        d.std = c['std']
        d.min_logvar, d.max_logvar = c['min_logvar'], c['max_logvar']
        d.add_noise = int(add_noise)
        d.noise = noise.data_ptr() if noise is not None else None
        d.sample, d.mean, d.pred_x0, d.pred_eps = sample.data_ptr(), mean.data_ptr(), x0.data_ptr(), eps.data_ptr()
        d.var = var_t.data_ptr() if var_t is not None else None
        if euler:
            d.euler = euler
            d.e_st1, d.e_sig_t, d.e_dsig = ecoefs['st1'], ecoefs['sig_t'], ecoefs['dsig']
            d.e_sp1, d.e_sig_p = ecoefs['sp1'], ecoefs['sig_p']
            d.e_d1 = d1.data_ptr() if d1 is not None else None
            d.e_x1 = x1.data_ptr() if x1 is not None else None
            d.e_dout = dout.data_ptr() if dout is not None else None
        dmhip.sampler_step(d, xt.device)
        if learned:
            var = var_t
        else:
            # 0-dim device copy of the scalar variance, made once per (t, t_prev) and cached:
            # a per-step host->device copy would stall the launch stream every step.
            key = ('var_dev', xt.device)
            var = c.get(key)
            if var is None:
                var = c.get('var_scalar', torch.tensor(0.0)).to(xt.device)
                c[key] = var
        return dict(sample=sample, mean=mean, var=var, pred_x0=x0, pred_eps=eps, reverse_eps=noise)

    # ----------------------------------------------------------- public API
    def predict(self, model_output: Tensor, xt: Tensor, t: int):
        """x0 / eps from the network output (reference ddpm.py:174-203)."""
        learned_var = None
        if model_output.shape[1] > xt.shape[1]:
            learned_var = model_output[:, xt.shape[1]:]
        out = self._step(model_output, xt, t, t - 1, predict_only=True)
        return {'pred_x0': out['pred_x0'], 'pred_eps': out['pred_eps'], 'learned_var': learned_var}

    def denoise(self, model_output: Tensor, xt: Tensor, t: int, t_prev: int):
        """Sample from p_theta(x_{t_prev} | x_t) (reference ddpm.py:205-261)."""
        return self._step(model_output, xt, t, t_prev)

    def sample_loop(
            self, model, init_noise: Tensor,
            tqdm_kwargs: Dict = None, model_kwargs: Dict = None,
    ):
        tqdm_kwargs = dict() if tqdm_kwargs is None else tqdm_kwargs
        model_kwargs = dict() if model_kwargs is None else model_kwargs
        img = init_noise
        seq = self.respaced_seq.tolist()
        seq_prev = [-1] + seq[:-1]
        pbar = tqdm.tqdm(total=len(seq), **tqdm_kwargs)
        for t, t_prev in zip(reversed(seq), reversed(seq_prev)):
            t_batch = torch.full((img.shape[0], ), t, device=img.device, dtype=torch.long)
            model_output = model(img, t_batch, **model_kwargs)
            out = self.denoise(model_output, img, t, t_prev)
            img = out['sample']
            pbar.update(1)
            yield out
        pbar.close()

    def sample(
            self, model, init_noise: Tensor,
            tqdm_kwargs: Dict = None, model_kwargs: Dict = None,
    ):
        def run():
            sample = None
            for out in self.sample_loop(model, init_noise, tqdm_kwargs, model_kwargs):
                sample = out['sample']
            return sample
        return self._range_guarded(run, init_noise)

    def _range_guarded(self, run: Callable[[], Tensor], init_noise: Tensor) -> Tensor:
        """Run a whole sampling loop with the fp16x2 range check of the native models deferred to its
        end: one host sync per loop instead of one per forward. If any forward met an activation
        beyond the fp16 range, the loop runs again from the same device RNG state with those models in
        their exact fallback arithmetic, so the result is what the fallback gives; afterwards they run
        fp16x2 again (the fallback is not sticky).
        A caller-installed noise source cannot be rewound: then every forward checks as it goes."""
        if self.noise_fn is not None or not isinstance(init_noise, Tensor) or init_noise.device.type != 'cuda':
            return run()
        dev = init_noise.device
        rng = torch.cuda.get_rng_state(dev)
        with dmhip.deferred_range_check() as scope:
            result = run()
        if scope.flagged:
            torch.cuda.set_rng_state(rng, dev)
            try:
                result = run()
            finally:
                scope.end_fallback()
        return result


class _CFGMixin:
    """Classifier-free guidance loop shared by DDPMCFG / DDIMCFG.

    Conditional and unconditional forwards per step as upstream (ddpm.py:334-348,
    ddim.py:176-188) — batched into one 2B forward when the model accepts a
    per-row null label (``model.supports_null_label``), else two calls; predict
    of both branches, the (1-s)/s combine and the denoise are one fused kernel.
    """

    def _cfg_init(self, guidance_scale: float, cond_kwarg: str):
        self.guidance_scale = guidance_scale
        self.cond_kwarg = cond_kwarg
        self.batch_cfg = True  # run cond + uncond as one 2B forward where the model allows it

    def sample_loop(
            self, model, init_noise: Tensor, uncond_conditioning: Any = None,
            tqdm_kwargs: Dict = None, model_kwargs: Dict = None,
    ):
        tqdm_kwargs = dict() if tqdm_kwargs is None else tqdm_kwargs
        model_kwargs = dict() if model_kwargs is None else model_kwargs
        if self.cond_kwarg not in model_kwargs.keys():
            raise ValueError(f'Condition argument `{self.cond_kwarg}` not found in model_kwargs.')
        uncond_kwargs = dict(model_kwargs)
        uncond_kwargs[self.cond_kwarg] = uncond_conditioning
        img = init_noise
        B = img.shape[0]
        cond = model_kwargs[self.cond_kwarg]
        # One 2B forward instead of two B forwards when the model takes "no label" per row
        # (y < 0, see UNetCategorialAdaGN.forward): every kernel is row-independent, so each
        # half equals the corresponding separate call; the weights are streamed once per step.
        batched = (self.batch_cfg and uncond_conditioning is None and len(model_kwargs) == 1
                   and getattr(model, 'supports_null_label', False) and isinstance(cond, Tensor)
                   and cond.shape == (B, ))
        if batched:
            y2 = torch.cat([cond, torch.full_like(cond, -1)])
        seq = self.respaced_seq.tolist()
        seq_prev = [-1] + seq[:-1]
        pbar = tqdm.tqdm(total=len(seq), **tqdm_kwargs)
        for t, t_prev in zip(reversed(seq), reversed(seq_prev)):
            if batched:
                t2 = torch.full((2 * B, ), t, device=img.device, dtype=torch.long)
                with dmhip.null_label_scope():
                    both = model(torch.cat([img, img]), t2, **{self.cond_kwarg: y2})
                out_c, out_u = both[:B], both[B:]
            else:
                t_batch = torch.full((B, ), t, device=img.device, dtype=torch.long)
                out_c = model(img, t_batch, **model_kwargs)
                out_u = model(img, t_batch, **uncond_kwargs)
            out = self._step(out_c, img, t, t_prev, model_output_uncond=out_u,
                             guidance_scale=self.guidance_scale)
            img = out['sample']
            pbar.update(1)
            yield out
        pbar.close()

    def sample(
            self, model, init_noise: Tensor, uncond_conditioning: Any = None,
            tqdm_kwargs: Dict = None, model_kwargs: Dict = None,
    ):
        def run():
            sample = None
            for out in self.sample_loop(model, init_noise, uncond_conditioning, tqdm_kwargs, model_kwargs):
                sample = out['sample']
            return sample
        return self._range_guarded(run, init_noise)

    @contextmanager
    def hack_objective(self, objective: str):
        tmp = self.objective
        self.objective = objective
        yield
        self.objective = tmp


class DDPMCFG(_CFGMixin, DDPM):
    def __init__(self, guidance_scale: float = 1., cond_kwarg: str = 'y', *args, **kwargs):
        """DDPM with classifier-free guidance (reference ddpm.py:293-368); s=0 uncond, s=1 cond, s>1 guided."""
        DDPM.__init__(self, *args, **kwargs)
        self._cfg_init(guidance_scale, cond_kwarg)
