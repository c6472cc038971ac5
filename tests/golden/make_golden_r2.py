"""Round-2 fixtures, generated from the REFERENCE implementation (build container only).

    python tests/golden/make_golden_r2.py [ddpm1000|drift|ddpmcfg]

Like make_golden.py this imports /root/reference through the bare-package shim
and runs the reference's own sampler and model classes on CPU. New here:

* ddpm1000.npz — BASELINE config C2's path: the CIFAR-10 UNet through the
  reference DDPM (fixed_large, all 1000 steps, diffusions/ddpm.py:205-281) at
  B=2. The per-step `randn_like` draw is replaced by tests/golden/noise.py's
  StepNoise (seeded numpy) while the reference runs, so the GPU test can replay
  it without a 25 MB noise file; 31 steps (t = 999 ... 0) are kept.
* drift.npz — the reference's own float32 vs float64 drift on the trajectories
  whose engine error is largest (DDIM-50 CIFAR, all 50 steps; ADM UNetCombined
  DDIMCFG-6; AdaGN DDIMCFG-10; DDIM inversion + reconstruction; DDPM-1000 is in
  ddpm1000.npz). Each is run twice with the same inputs: the reference module
  as is (fp32) and the same module in float64 (see `Float64Reference`); both
  trajectories are stored (the float64 one rounded to float32). The GPU tests
  require the engine to be at least as close to the float64 trajectory as
  the reference's fp32 run is, within 1.5x (tests/conftest.py check_free_running).
* ddpmcfg.npz — DDPMCFG (diffusions/ddpm.py:319-351) with learned_range,
  i.e. the concat of the conditional branch's variance channels (:344-345):
  through UNetCombined (two calls) and through a learned-range
  UNetCategorialAdaGN (which the engine runs as one batched 2B forward).
"""
import copy
import os
import sys
from contextlib import contextmanager

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402
from noise import StepNoise  # noqa: E402

REF_TAG = 'xyfJASON/diffusion-models-pytorch @ 2024-12-20 (/root/reference)'


def _common():
    return dict(torch=torch.__version__, threads=torch.get_num_threads(), reference=REF_TAG,
                coef_probe_sha=mg.coef_probe_sha())


@contextmanager
def patched_randn_like(source):
    """Route the reference's torch.randn_like (ddpm.py:251, ddim.py:76) to `source`."""
    orig = torch.randn_like
    torch.randn_like = lambda x, *a, **k: source(x)
    try:
        yield
    finally:
        torch.randn_like = orig


class Float64Reference:
    """The same reference module evaluated in float64.

    A deep copy is converted with .double(); float32 tensors entering any
    Linear / Conv / GroupNorm (the sinusoid tables are built in float32 from
    integer t) are cast to float64. ADM keeps three fp32 islands for its fp16
    mode (GroupNorm32 `x.float()`, QKVAttention `softmax(weight.float())`,
    `h = x.type(self.dtype)`, adm/nn.py:17-19, adm/unet.py:371,406,673); during
    the call `Tensor.float()` leaves float64 tensors as they are and the
    models' `dtype` attribute is float64, so those run in float64 too.
    The sampler arithmetic is the reference's own, on float64 state (its 0-dim
    float32 coefficients promote)."""

    def __init__(self, model):
        self.m = copy.deepcopy(model).double().eval()

        def pre(mod, args):
            return tuple(a.double() if torch.is_tensor(a) and a.dtype == torch.float32 else a for a in args)
        for mod in self.m.modules():
            if isinstance(mod, (torch.nn.Linear, torch.nn.Conv1d, torch.nn.Conv2d, torch.nn.GroupNorm)):
                mod.register_forward_pre_hook(pre)
            if getattr(mod, 'dtype', None) == torch.float32:
                mod.dtype = torch.float64

    def __call__(self, *args, **kwargs):
        orig = torch.Tensor.float

        def keep64(t, *a, **k):
            return t if t.dtype == torch.float64 else orig(t, *a, **k)
        torch.Tensor.float = keep64
        try:
            return self.m(*args, **kwargs)
        finally:
            torch.Tensor.float = orig


def run_pair(loop_fn, model, init, noise_seed=None, keys=('sample', 'pred_eps')):
    """Run loop_fn(model, init) -> iterable of step dicts with the fp32 reference and its float64
    copy on the same inputs. Returns (fp32 per-step dicts, per-step max-abs drift per key, float64
    per-step dicts)."""
    out32, out64 = [], []
    for m, x, dst in ((model, init, out32), (Float64Reference(model), init.double(), out64)):
        src = StepNoise(noise_seed) if noise_seed is not None else None
        ctx = patched_randn_like(src) if src is not None else _null()
        with ctx, torch.no_grad():
            for out in loop_fn(m, x):
                dst.append({k: out[k].detach().clone() for k in keys if out.get(k) is not None})
    drift = {k: np.array([float((a[k].double() - b[k]).abs().max()) for a, b in zip(out32, out64)])
             for k in keys if k in out32[0]}
    return out32, drift, out64


@contextmanager
def _null():
    yield


def make_ddpm1000():
    torch.set_num_threads(8)
    schedule, ddpm, ddim, unet = mg.import_reference()
    meta = _common()
    model = unet.UNet(**mg.ARCHS['cifar10']).eval()
    meta['cifar10_weights_sha256'] = mg.synthetic(model)
    d = ddpm.DDPM(var_type='fixed_large')   # T = 1000, respace None -> all 1000 steps
    torch.manual_seed(2022)
    init = torch.randn((2, 3, 32, 32))
    seed = 1000
    outs, drift, o64 = run_pair(lambda m, x: d.sample_loop(m, x, tqdm_kwargs=dict(disable=True)), model, init,
                           noise_seed=seed)
    assert len(outs) == 1000
    keep = sorted(set(range(0, 1000, 40)) | {1, 2, 997, 998, 999})
    arr = dict(init=init, drift_sample=drift['sample'], drift_pred_eps=drift['pred_eps'], keep=np.array(keep))
    for i in keep:
        arr[f'step{i}_sample'] = outs[i]['sample']
        arr[f'step{i}_pred_eps'] = outs[i]['pred_eps']
        arr[f'step{i}_sample64'] = o64[i]['sample'].float()   # float64 run, rounded for storage
        if i > 0:   # the input of step i, for the teacher-forced check
            arr[f'step{i - 1}_sample'] = outs[i - 1]['sample']
    meta.update(keep=keep, noise_seed=seed, sampler=dict(var_type='fixed_large', total_steps=1000),
                noise='tests/golden/noise.py StepNoise(noise_seed): draw k = PCG64([seed, k]) float32 normal',
                max_drift_sample=float(drift['sample'].max()), max_drift_pred_eps=float(drift['pred_eps'].max()))
    mg.save('ddpm1000', meta, **arr)


def make_drift():
    torch.set_num_threads(8)
    schedule, ddpm, ddim, unet = mg.import_reference()
    import models.unet_categorial_adagn as ua  # noqa: E402
    import models.adm.unet_combined as admc  # noqa: E402
    meta = _common()
    arr = {}
    # DDIM-50 CIFAR-10, B=2 (trajectory.npz's run), all 50 steps
    model = unet.UNet(**mg.ARCHS['cifar10']).eval()
    meta['cifar10_weights_sha256'] = mg.synthetic(model)
    d = ddim.DDIM(respace_type='uniform', respace_steps=50, eta=0.0)
    torch.manual_seed(2022)
    init = torch.randn((2, 3, 32, 32))
    outs, drift, o64 = run_pair(lambda m, x: d.sample_loop(m, x, tqdm_kwargs=dict(disable=True)), model, init)
    arr['ddim50_init'] = init
    arr['ddim50_sample'] = torch.stack([o['sample'] for o in outs])
    arr['ddim50_pred_eps'] = torch.stack([o['pred_eps'] for o in outs])
    arr['ddim50_drift_sample'], arr['ddim50_drift_pred_eps'] = drift['sample'], drift['pred_eps']
    arr['ddim50_sample64'] = torch.stack([o['sample'] for o in o64]).float()
    # ADM UNetCombined (adm_tiny arch), DDIMCFG-6 s=2.5 (adm.npz cfg6)
    comb = admc.UNetCombined(**mg.ADM_ARCHS['adm_tiny']).eval()
    meta['combined_tiny_weights_sha256'] = mg.synthetic(comb)
    d = ddim.DDIMCFG(guidance_scale=2.5, respace_type='uniform', respace_steps=6, eta=0.0)
    torch.manual_seed(37)
    init = torch.randn((2, 3, 16, 16))
    labels = torch.tensor([2, 3])
    outs, drift, o64 = run_pair(lambda m, x: d.sample_loop(m, x, model_kwargs=dict(y=labels),
                                                      tqdm_kwargs=dict(disable=True)), comb, init)
    arr['cfg6_sample'] = torch.stack([o['sample'] for o in outs])
    arr['cfg6_drift_sample'] = drift['sample']
    arr['cfg6_sample64'] = torch.stack([o['sample'] for o in o64]).float()
    # AdaGN DDIMCFG-10 s=3 on tiny_updown (adagn.npz cfg)
    model = ua.UNetCategorialAdaGN(**mg.ADAGN_ARCHS['tiny_updown']).eval()
    meta['tiny_updown_weights_sha256'] = mg.synthetic(model)
    d = ddim.DDIMCFG(guidance_scale=3.0, respace_type='uniform', respace_steps=10, eta=0.0)
    torch.manual_seed(5)
    init = torch.randn((2, 3, 16, 16))
    labels = torch.tensor([1, 4])
    outs, drift, o64 = run_pair(lambda m, x: d.sample_loop(m, x, model_kwargs=dict(y=labels),
                                                      tqdm_kwargs=dict(disable=True)), model, init)
    arr['adagn_cfg10_sample'] = torch.stack([o['sample'] for o in outs])
    arr['adagn_cfg10_drift_sample'] = drift['sample']
    arr['adagn_cfg10_sample64'] = torch.stack([o['sample'] for o in o64]).float()
    # DDIM inversion (4 steps) feeding reconstruction (5 steps) on the tiny UNet (inversion.npz)
    model = unet.UNet(**mg.ARCHS['tiny']).eval()
    meta['tiny_weights_sha256'] = mg.synthetic(model)
    d = ddim.DDIM(respace_type='uniform', respace_steps=5, eta=0.0)
    g = torch.Generator().manual_seed(31)
    img = torch.rand((2, 3, 16, 16), generator=g) * 2 - 1

    def inv_rec(m, x):
        for out in d.sample_inversion_loop(m, x, tqdm_kwargs=dict(disable=True)):
            x = out['sample']
            yield out
        yield from d.sample_loop(m, x, tqdm_kwargs=dict(disable=True))
    outs, drift, o64 = run_pair(inv_rec, model, img)
    arr['invrec_sample'] = torch.stack([o['sample'] for o in outs])
    arr['invrec_drift_sample'] = drift['sample']
    arr['invrec_sample64'] = torch.stack([o['sample'] for o in o64]).float()
    meta['invrec_steps'] = [4, 5]
    mg.save('drift', meta, **arr)


def make_ddpmcfg():
    torch.set_num_threads(8)
    schedule, ddpm, ddim, unet = mg.import_reference()
    import models.unet_categorial_adagn as ua  # noqa: E402
    import models.adm.unet_combined as admc  # noqa: E402
    meta = _common()
    arr = {}
    # UNetCombined (adm_tiny arch, learned sigma), DDPMCFG-8 learned_range s=2.5, noise pinned per step
    comb = admc.UNetCombined(**mg.ADM_ARCHS['adm_tiny']).eval()
    meta['combined_tiny_weights_sha256'] = mg.synthetic(comb)
    d = ddpm.DDPMCFG(guidance_scale=2.5, var_type='learned_range', respace_type='uniform', respace_steps=8)
    torch.manual_seed(41)
    init = torch.randn((2, 3, 16, 16))
    labels = torch.tensor([2, 3])
    outs, drift, o64 = run_pair(lambda m, x: d.sample_loop(m, x, model_kwargs=dict(y=labels),
                                                      tqdm_kwargs=dict(disable=True)), comb, init, noise_seed=41,
                           keys=('sample', 'pred_eps', 'reverse_eps'))
    arr['adm_init'], arr['adm_labels'] = init, labels
    for i, o in enumerate(outs):
        arr[f'adm_step{i}_sample'], arr[f'adm_step{i}_pred_eps'] = o['sample'], o['pred_eps']
    arr['adm_drift_sample'] = drift['sample']
    arr['adm_sample64'] = torch.stack([o['sample'] for o in o64]).float()
    meta['adm'] = dict(guidance_scale=2.5, var_type='learned_range', respace_type='uniform', respace_steps=8,
                       noise_seed=41)
    # UNetCategorialAdaGN with learned-sigma outputs (out_channels = 2C), cosine schedule (the CFG-CIFAR
    # diffusion config), DDPMCFG-6 learned_range s=3
    arch = dict(mg.ADAGN_ARCHS['tiny_updown'], out_channels=6)
    model = ua.UNetCategorialAdaGN(**arch).eval()
    meta['adagn_learned_weights_sha256'] = mg.synthetic(model)
    meta['adagn_learned_arch'] = arch
    d = ddpm.DDPMCFG(guidance_scale=3.0, beta_schedule='cosine', var_type='learned_range', respace_type='uniform',
                     respace_steps=6)
    torch.manual_seed(43)
    init = torch.randn((2, 3, 16, 16))
    labels = torch.tensor([1, 4])
    outs, drift, o64 = run_pair(lambda m, x: d.sample_loop(m, x, model_kwargs=dict(y=labels),
                                                      tqdm_kwargs=dict(disable=True)), model, init, noise_seed=43,
                           keys=('sample', 'pred_eps', 'reverse_eps'))
    arr['adagn_init'], arr['adagn_labels'] = init, labels
    for i, o in enumerate(outs):
        arr[f'adagn_step{i}_sample'], arr[f'adagn_step{i}_pred_eps'] = o['sample'], o['pred_eps']
    arr['adagn_drift_sample'] = drift['sample']
    arr['adagn_sample64'] = torch.stack([o['sample'] for o in o64]).float()
    meta['adagn'] = dict(guidance_scale=3.0, beta_schedule='cosine', var_type='learned_range',
                         respace_type='uniform', respace_steps=6, noise_seed=43)
    mg.save('ddpmcfg', meta, **arr)


if __name__ == '__main__':
    which = sys.argv[1:] or ['ddpmcfg', 'drift', 'ddpm1000']
    for w in which:
        dict(ddpm1000=make_ddpm1000, drift=make_drift, ddpmcfg=make_ddpmcfg)[w]()
