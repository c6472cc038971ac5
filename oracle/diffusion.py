"""Sampler oracle (TEST INFRASTRUCTURE ONLY) — torch CPU, reference op order.

Each function restates one reference routine; expressions are kept in the
reference's order because float32 results (and torch's non-IEEE 0-dim
sqrt/pow) depend on it.
"""
import math
from typing import Callable, Dict, Optional

import torch
from torch import Tensor


def beta_schedule(total_steps=1000, kind='linear', beta_start=0.0001, beta_end=0.02) -> Tensor:
    """diffusions/schedule.py:5-38"""
    if kind == 'linear':
        return torch.linspace(beta_start, beta_end, total_steps, dtype=torch.float64)
    if kind == 'quad':
        return torch.linspace(beta_start ** 0.5, beta_end ** 0.5, total_steps, dtype=torch.float64) ** 2
    if kind == 'const':
        return torch.full((total_steps, ), fill_value=beta_end, dtype=torch.float64)
    if kind == 'cosine':
        def abar(s):
            return math.cos((s + 0.008) / 1.008 * math.pi / 2) ** 2
        return torch.tensor([min(1 - abar((i + 1) / total_steps) / abar(i / total_steps), 0.999)
                             for i in range(total_steps)])
    raise ValueError(kind)


def respaced_seq(total_steps=1000, kind='uniform', steps=100) -> Tensor:
    """diffusions/schedule.py:41-73"""
    if kind in ('uniform', 'uniform-leading'):
        return torch.arange(0, total_steps, total_steps // steps).long()
    if kind == 'uniform-linspace':
        return torch.linspace(0, total_steps - 1, steps).long()
    if kind == 'uniform-trailing':
        return torch.arange(total_steps - 1, -1, -(total_steps // steps)).long().flip(dims=[0])
    if kind == 'quad':
        return torch.floor(torch.linspace(0, math.sqrt(total_steps * 0.8), steps) ** 2).long()
    if kind is None or kind == 'none':
        return torch.arange(0, total_steps).long()
    raise ValueError(kind)


def alphas_cumprod(betas: Tensor) -> Tensor:
    """diffusions/ddpm.py:81-82"""
    return torch.cumprod(1. - betas, dim=0).to(torch.float)


def predict(ac: Tensor, out: Tensor, xt: Tensor, t: int, objective='pred_eps', clip=True):
    """diffusions/ddpm.py:102-120, 174-203"""
    learned_var = None
    if out.shape[1] > xt.shape[1]:
        out, learned_var = torch.split(out, xt.shape[1], dim=1)
    a = ac[t]
    if objective == 'pred_eps':
        x0 = (1. / a) ** 0.5 * xt - (1. / a - 1.) ** 0.5 * out
    elif objective == 'pred_x0':
        x0 = out
    elif objective == 'pred_v':
        x0 = a ** 0.5 * xt - (1. - a) ** 0.5 * out
    else:
        raise ValueError(objective)
    if clip:
        x0.clamp_(-1., 1.)
    eps = ((1. / a) ** 0.5 * xt - x0) / (1. / a - 1.) ** 0.5
    return x0, eps, learned_var


def pred_x0_from_eps(ac: Tensor, xt: Tensor, t: int, eps: Tensor) -> Tensor:
    """diffusions/ddpm.py:102-105"""
    return (1. / ac[t]) ** 0.5 * xt - (1. / ac[t] - 1.) ** 0.5 * eps


def pred_eps_from_x0(ac: Tensor, xt: Tensor, t: int, x0: Tensor) -> Tensor:
    """diffusions/ddpm.py:107-110"""
    return ((1. / ac[t]) ** 0.5 * xt - x0) / (1. / ac[t] - 1.) ** 0.5


def pred_x0_from_v(ac: Tensor, xt: Tensor, t: int, v: Tensor) -> Tensor:
    """diffusions/ddpm.py:112-115"""
    return ac[t] ** 0.5 * xt - (1. - ac[t]) ** 0.5 * v


def pred_eps_from_v(ac: Tensor, xt: Tensor, t: int, v: Tensor) -> Tensor:
    """diffusions/ddpm.py:117-120"""
    return (1. - ac[t]) ** 0.5 * xt + ac[t] ** 0.5 * v


def _per_image(c: Tensor, ndim: int) -> Tensor:
    while c.ndim < ndim:
        c = c.unsqueeze(-1)
    return c


def get_v(ac: Tensor, x0: Tensor, eps: Tensor, t: Tensor) -> Tensor:
    """diffusions/ddpm.py:140-150"""
    sa = _per_image(ac[t] ** 0.5, x0.ndim)
    s1m = _per_image((1. - ac[t]) ** 0.5, x0.ndim)
    return sa * eps - s1m * x0


def diffuse(ac: Tensor, x0: Tensor, t: Tensor, eps: Tensor) -> Tensor:
    """diffusions/ddpm.py:152-172"""
    sa = _per_image(ac[t] ** 0.5, x0.ndim)
    s1m = _per_image((1. - ac[t]) ** 0.5, x0.ndim)
    return sa * x0 + s1m * eps


def ddpm_denoise(ac, out, xt, t, t_prev, var_type='fixed_large', objective='pred_eps', clip=True,
                 noise_fn: Callable[[Tensor], Tensor] = torch.randn_like) -> Dict[str, Tensor]:
    """diffusions/ddpm.py:205-261"""
    x0, eps, lv = predict(ac, out, xt, t, objective, clip)
    a_t = ac[t]
    a_p = ac[t_prev] if t_prev >= 0 else torch.tensor(1.0)
    alpha = a_t / a_p
    beta = 1. - alpha
    mean = (a_p ** 0.5) * beta / (1. - a_t) * x0 + (alpha ** 0.5) * (1. - a_p) / (1. - a_t) * xt
    if t == 0:
        var = torch.zeros_like(beta)
    elif var_type == 'fixed_small':
        var = beta * (1. - a_p) / (1. - a_t)
    elif var_type == 'fixed_large':
        var = beta
    elif var_type == 'learned_range':
        lo = torch.log(torch.clamp_min(beta * (1. - a_p) / (1. - a_t), 1e-20))
        hi = torch.log(beta)
        frac = (lv + 1) / 2
        var = torch.exp(frac * hi + (1 - frac) * lo)
    else:
        raise ValueError(var_type)
    noise = noise_fn(xt)
    sample = mean if t == 0 else mean + torch.sqrt(var) * noise
    return dict(sample=sample, mean=mean, var=var, pred_x0=x0, pred_eps=eps, reverse_eps=noise)


def ddim_denoise(ac, out, xt, t, t_prev, eta=0.0, objective='pred_eps', clip=True,
                 noise_fn: Callable[[Tensor], Tensor] = torch.randn_like) -> Dict[str, Tensor]:
    """diffusions/ddim.py:57-86"""
    x0, eps, _ = predict(ac, out, xt, t, objective, clip)
    a_t = ac[t]
    a_p = ac[t_prev] if t_prev >= 0 else torch.tensor(1.0)
    var = (eta ** 2) * (1. - a_p) / (1. - a_t) * (1. - a_t / a_p)
    mean = torch.sqrt(a_p) * x0 + torch.sqrt(1. - a_p - var) * eps
    noise = noise_fn(xt)
    sample = mean if t == 0 else mean + torch.sqrt(var) * noise
    return dict(sample=sample, mean=mean, var=var, pred_x0=x0, pred_eps=eps, reverse_eps=noise)


def ddim_invert(ac, out, xt, t, t_next, total_steps, objective='pred_eps', clip=True):
    """diffusions/ddim.py:88-104 (eta = 0)"""
    x0, eps, _ = predict(ac, out, xt, t, objective, clip)
    a_n = ac[t_next] if t_next < total_steps else torch.tensor(0.0)
    return dict(sample=torch.sqrt(a_n) * x0 + torch.sqrt(1. - a_n) * eps, pred_x0=x0, pred_eps=eps)


def sample_loop(model: Callable, ac: Tensor, seq: Tensor, init_noise: Tensor, sampler='ddim', eta=0.0,
                var_type='fixed_large', objective='pred_eps', clip=True,
                noise_fn: Callable[[Tensor], Tensor] = torch.randn_like,
                guidance_scale: Optional[float] = None, y: Optional[Tensor] = None):
    """diffusions/ddpm.py:263-281 (and the CFG loops ddpm.py:319-351 / ddim.py:161-191 when
    guidance_scale is given): yields each step's output dict."""
    img = init_noise
    ts = seq.tolist()
    prev = [-1] + ts[:-1]
    for t, tp in zip(reversed(ts), reversed(prev)):
        tb = torch.full((img.shape[0], ), t, dtype=torch.long)
        if guidance_scale is None:
            out = model(img, tb)
            obj = objective
        else:
            oc = model(img, tb, y)
            ou = model(img, tb, None)
            ec = predict(ac, oc, img, t, objective, clip)[1]
            eu = predict(ac, ou, img, t, objective, clip)[1]
            out = (1 - guidance_scale) * eu + guidance_scale * ec
            if sampler == 'ddpm' and var_type == 'learned_range':
                out = torch.cat([out, oc[:, out.shape[1]:]], dim=1)
            obj = 'pred_eps'
        if sampler == 'ddim':
            res = ddim_denoise(ac, out, img, t, tp, eta, obj, clip, noise_fn)
        else:
            res = ddpm_denoise(ac, out, img, t, tp, var_type, obj, clip, noise_fn)
        img = res['sample']
        yield res


def sigmas(ac: Tensor) -> Tensor:
    """diffusions/euler.py:48, heun.py:51"""
    return ((1 - ac) / ac).sqrt()


def euler_denoise(ac: Tensor, sig: Tensor, out: Tensor, xt: Tensor, t: int, t_prev: int,
                  objective='pred_eps', clip=True) -> Dict[str, Tensor]:
    """diffusions/euler.py:50-66 (= HeunSampler.denoise_1st_order, heun.py:56-77, which keeps `derivative`)"""
    sigmas_t = sig[t]
    sigmas_t_prev = sig[t_prev] if t_prev >= 0 else torch.tensor(0.0)
    pred_x0, _, _ = predict(ac, out, xt, t, objective, clip)
    bar_xt = (1 + sigmas_t ** 2).sqrt() * xt
    derivative = (bar_xt - pred_x0) / sigmas_t
    bar_sample = bar_xt + derivative * (sigmas_t_prev - sigmas_t)
    sample = bar_sample / (1 + sigmas_t_prev ** 2).sqrt()
    return dict(sample=sample, pred_x0=pred_x0, derivative=derivative)


def heun_denoise_2nd(ac: Tensor, sig: Tensor, out: Tensor, xt_prev: Tensor, t: int, t_prev: int,
                     d1: Tensor, xt1: Tensor, objective='pred_eps', clip=True) -> Dict[str, Tensor]:
    """diffusions/heun.py:79-106"""
    sigmas_t = sig[t]
    sigmas_t_prev = sig[t_prev] if t_prev >= 0 else torch.tensor(0.0)
    pred_x0, _, _ = predict(ac, out, xt_prev, t_prev, objective, clip)
    bar_xt_prev = (1 + sigmas_t_prev ** 2).sqrt() * xt_prev
    derivative = (bar_xt_prev - pred_x0) / sigmas_t_prev
    derivative = (derivative + d1) / 2
    bar_xt = (1 + sigmas_t ** 2).sqrt() * xt1
    bar_sample = bar_xt + derivative * (sigmas_t_prev - sigmas_t)
    sample = bar_sample / (1 + sigmas_t_prev ** 2).sqrt()
    return dict(sample=sample, pred_x0=pred_x0)
