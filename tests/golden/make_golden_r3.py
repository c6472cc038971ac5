"""Round-3 fixtures (build container only).

    python tests/golden/make_golden_r3.py [convert|stepacc|dit]

* convert.npz -- the closed-form conversions of the REFERENCE sampler (diffusions/ddpm.py:102-172:
  pred_x0_from_eps, pred_eps_from_x0, pred_x0_from_v, pred_eps_from_v, get_v, diffuse) on seeded
  inputs, run by importing /root/reference (make_golden.py's bare-package shim).
* stepacc.npz -- per-step accuracy against float64, free of trajectory chaos. For the free-running
  trajectories of drift.npz (ADM UNetCombined DDIMCFG-6, AdaGN DDIMCFG-10, DDIM inversion +
  reconstruction, DDIM-50 CIFAR-10) every step i is recomputed from the SAME input x_i -- the
  reference's float64 trajectory state before step i, rounded to float32 -- once by the reference
  module in float32 (`ref32`) and once by its float64 copy (`ref64`, kept in float64). A GPU test then
  runs the engine's single step from x_i and compares |engine - ref64| with |ref32 - ref64|: whether the
  engine is as accurate as the fp32 reference on each step, which the free-running comparison cannot
  tell (a 2^-22 relative perturbation of the model output alone moves the ADM CFG-6 end point by
  1.4e-4 ... 2.5e-4 from float64).
* dit_r3.npz -- DiT-XL/2 (32x32 latents) DDIMCFG-3, s = 4, B = 2, from oracle/dit.py (PARITY UNPINNED:
  the reference DiT needs timm, absent here).
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402

REF_TAG = 'xyfJASON/diffusion-models-pytorch @ 2024-12-20 (/root/reference)'


def _common():
    return dict(torch=torch.__version__, threads=torch.get_num_threads(), reference=REF_TAG,
                coef_probe_sha=mg.coef_probe_sha())


def _load(name):
    with np.load(os.path.join(HERE, name + '.npz'), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def make_convert():
    torch.set_num_threads(8)
    schedule, ddpm, ddim, unet = mg.import_reference()
    meta = _common()
    g = torch.Generator().manual_seed(17)
    arr = {}
    cases = [('linear', 1000), ('cosine', 1000)]
    meta['cases'] = {}
    for kind, T in cases:
        d = ddpm.DDPM(total_steps=T, beta_schedule=kind)
        name = f'{kind}{T}'
        x0 = torch.randn((4, 3, 8, 8), generator=g)
        eps = torch.randn((4, 3, 8, 8), generator=g)
        xt = torch.randn((4, 3, 8, 8), generator=g)
        tvec = torch.tensor([0, 250, 777, T - 1])
        arr[f'{name}_x0'], arr[f'{name}_eps'], arr[f'{name}_xt'], arr[f'{name}_tvec'] = x0, eps, xt, tvec
        arr[f'{name}_diffuse'] = d.diffuse(x0, tvec, eps)
        arr[f'{name}_get_v'] = d.get_v(x0, eps, tvec)
        ts = [0, 1, 500, T - 1]
        for t in ts:
            arr[f'{name}_t{t}_x0_from_eps'] = d.pred_x0_from_eps(xt, t, eps)
            arr[f'{name}_t{t}_eps_from_x0'] = d.pred_eps_from_x0(xt, t, x0)
            arr[f'{name}_t{t}_x0_from_v'] = d.pred_x0_from_v(xt, t, eps)
            arr[f'{name}_t{t}_eps_from_v'] = d.pred_eps_from_v(xt, t, eps)
        meta['cases'][name] = dict(beta_schedule=kind, total_steps=T, ts=ts)
    mg.save('convert', meta, **arr)


def _single(loop_fn, seq, d, t, tp):
    """One step (t -> tp) of a reference sampler loop: respaced_seq reduced to the pair."""
    keep = d.respaced_seq
    d.respaced_seq = torch.tensor([tp, t] if tp >= 0 else [t])
    try:
        return next(iter(loop_fn()))['sample']
    finally:
        d.respaced_seq = keep


def make_stepacc():
    from make_golden_r2 import Float64Reference
    torch.set_num_threads(8)
    schedule, ddpm, ddim, unet = mg.import_reference()
    import models.unet_categorial_adagn as ua  # noqa: E402
    import models.adm.unet_combined as admc  # noqa: E402
    drift, adm = _load('drift'), _load('adm')
    meta = _common()
    arr = {}

    def run(name, model, d, init, traj64, labels=None, steps=None, inversion_first=0):
        """Every step from x_i = fp32(traj64[i - 1]) (x_0 = init), by the fp32 module and its float64 copy."""
        m64 = Float64Reference(model)
        seq = d.respaced_seq.tolist()
        pairs = list(zip(reversed(seq), reversed([-1] + seq[:-1])))
        inv = list(zip(seq[:-1], seq[1:]))
        plan = [('inv', a, b) for a, b in inv[:inversion_first]] if inversion_first else []
        plan += [('den', a, b) for a, b in pairs]
        if steps is not None:
            plan = plan[:steps]
        xs, o32, o64 = [], [], []
        for i, (kind, t, tn) in enumerate(plan):
            x = init if i == 0 else torch.from_numpy(traj64[i - 1])
            outs = []
            for m, xin in ((model, x), (m64, x.double())):
                kw = dict(model_kwargs=dict(y=labels)) if labels is not None else {}
                with torch.no_grad():
                    if kind == 'inv':
                        keep = d.respaced_seq
                        d.respaced_seq = torch.tensor([t, tn])
                        try:
                            o = next(iter(d.sample_inversion_loop(m, xin, tqdm_kwargs=dict(disable=True))))['sample']
                        finally:
                            d.respaced_seq = keep
                    else:
                        o = _single(lambda: d.sample_loop(m, xin, tqdm_kwargs=dict(disable=True), **kw), seq, d, t, tn)
                outs.append(o)
            xs.append(x.float())
            o32.append(outs[0].float())
            o64.append(outs[1].double())
        arr[f'{name}_x'] = torch.stack(xs)
        arr[f'{name}_ref32'] = torch.stack(o32)
        arr[f'{name}_ref64'] = torch.stack(o64)
        e = [(a.double() - b).abs() for a, b in zip(o32, o64)]
        meta[name] = dict(steps=[[k, t, tn] for k, t, tn in plan],
                          ref32_max=[float(v.max()) for v in e],
                          ref32_rms=[float(v.pow(2).mean().sqrt()) for v in e])
        print(name, 'ref32 vs ref64 max', ['%.2e' % v for v in meta[name]['ref32_max']], flush=True)

    # ADM UNetCombined (adm_tiny), DDIMCFG-6 s = 2.5 (drift.npz cfg6)
    comb = admc.UNetCombined(**mg.ADM_ARCHS['adm_tiny']).eval()
    meta['combined_tiny_weights_sha256'] = mg.synthetic(comb)
    d = ddim.DDIMCFG(guidance_scale=2.5, respace_type='uniform', respace_steps=6, eta=0.0)
    run('cfg6', comb, d, torch.from_numpy(adm['cfg6_init']), drift['cfg6_sample64'],
        labels=torch.from_numpy(adm['ddpm8_labels']))
    # AdaGN DDIMCFG-10 s = 3 on tiny_updown (drift.npz adagn_cfg10)
    model = ua.UNetCategorialAdaGN(**mg.ADAGN_ARCHS['tiny_updown']).eval()
    meta['tiny_updown_weights_sha256'] = mg.synthetic(model)
    d = ddim.DDIMCFG(guidance_scale=3.0, respace_type='uniform', respace_steps=10, eta=0.0)
    torch.manual_seed(5)
    init = torch.randn((2, 3, 16, 16))
    run('adagn_cfg10', model, d, init, drift['adagn_cfg10_sample64'], labels=torch.tensor([1, 4]))
    meta['adagn_cfg10_labels'] = [1, 4]
    # DDIM inversion (4 steps) + reconstruction (5 steps) on the tiny UNet (drift.npz invrec)
    model = unet.UNet(**mg.ARCHS['tiny']).eval()
    meta['tiny_weights_sha256'] = mg.synthetic(model)
    d = ddim.DDIM(respace_type='uniform', respace_steps=5, eta=0.0)
    g = torch.Generator().manual_seed(31)
    img = torch.rand((2, 3, 16, 16), generator=g) * 2 - 1
    run('invrec', model, d, img, drift['invrec_sample64'], inversion_first=4)
    # DDIM-50 CIFAR-10 (drift.npz ddim50), the first 12 steps (t = 980 ... 760, where x0 amplifies most)
    model = unet.UNet(**mg.ARCHS['cifar10']).eval()
    meta['cifar10_weights_sha256'] = mg.synthetic(model)
    d = ddim.DDIM(respace_type='uniform', respace_steps=50, eta=0.0)
    run('ddim50', model, d, torch.from_numpy(drift['ddim50_init']), drift['ddim50_sample64'], steps=12)
    mg.save('stepacc', meta, **arr)


def make_dit():
    sys.path[:0] = [REPO, os.path.join(REPO, 'diffusion-models-pytorch_amd')]
    from oracle import diffusion as od  # noqa: E402
    import make_dit_golden as mdg  # noqa: E402
    torch.set_num_threads(8)
    meta = dict(torch=torch.__version__, generator='oracle/dit.py (parity unpinned: timm absent)')
    arch = mdg.ARCHS['dit_xl2']
    model, sha, _ = mdg.oracle_model(arch)
    meta['dit_xl2_weights_sha256'] = sha
    ac = od.alphas_cumprod(od.beta_schedule(1000, 'linear'))
    seq = od.respaced_seq(1000, 'uniform', 3)
    torch.manual_seed(47)
    init = torch.randn((2, 4, 32, 32))
    labels = torch.tensor([207, 360])
    arr = dict(xl2_cfg3_init=init, xl2_cfg3_labels=labels)
    from oracle.dit import OracleDiT  # noqa: E402
    m64 = OracleDiT(model.sd, dtype=torch.float64, **model.arch)
    runs = []
    for m, x in ((model, init), (m64, init.double())):
        runs.append([o['sample'] for o in od.sample_loop(m, ac, seq, x, sampler='ddim', eta=0.0, guidance_scale=4.0,
                                                         y=labels, clip=False)])
        print('dit run done', flush=True)
    for i, s32 in enumerate(runs[0]):
        arr[f'xl2_cfg3_step{i}_sample'] = s32
    arr['xl2_cfg3_sample64'] = torch.stack(runs[1]).float()
    arr['xl2_cfg3_drift_sample'] = np.array([float((a.double() - b).abs().max()) for a, b in zip(*runs)])
    print('drift', arr['xl2_cfg3_drift_sample'], flush=True)
    # clip_denoised false: the DiT-XL/2 YAML (weights/facebookresearch/DiT/DiT-XL-2-256x256.yaml:37)
    meta['xl2_cfg3'] = dict(guidance_scale=4.0, respace_type='uniform', respace_steps=3, eta=0.0,
                            clip_denoised=False)
    mg.save('dit_r3', meta, **arr)


class _Perturbed:
    """The fp32 reference module with its output multiplied by (1 + 2^ex s), s a seeded +-1 pattern: ex = -22
    is the rounding level of the fp32 forward itself (one ulp is 2^-23 relative), ex = -20 the level at
    which the engine's forwards differ from the reference's (~1e-6 relative, tests/test_gpu_parity.py)."""

    def __init__(self, model, seed, ex):
        self.m, self.g, self.ex = model, torch.Generator().manual_seed(1000 + seed), ex

    def __call__(self, *a, **k):
        out = self.m(*a, **k)
        s = torch.randint(0, 2, out.shape, generator=self.g).float() * 2 - 1
        return out * (1 + s * 2.0 ** self.ex)


def make_chaos():
    """chaos.npz -- how far free-running fp32 trajectories of the REFERENCE scatter around its float64 one
    when only the last bits of the model output change: each drift.npz trajectory (ADM UNetCombined
    DDIMCFG-6, AdaGN DDIMCFG-10, inversion + reconstruction) re-run by the reference in fp32 with the
    model output perturbed by 2^-22 and by 2^-20 relative (_Perturbed), 8 seeds each; per seed and step the
    max-abs distance to the float64 trajectory (drift.npz *_sample64): `<name>_e64_p22`, `<name>_e64_p20`.
    An engine whose forward differs from the reference's at the 2^-20 level lands inside that spread, not
    at the unperturbed fp32 run's distance."""
    torch.set_num_threads(8)
    schedule, ddpm, ddim, unet = mg.import_reference()
    import models.unet_categorial_adagn as ua  # noqa: E402
    import models.adm.unet_combined as admc  # noqa: E402
    drift, adm = _load('drift'), _load('adm')
    meta = _common()
    arr = {}
    seeds = 8

    def run(name, model, loop_fn, init, traj64):
        for ex in (-22, -20):
            e = np.zeros((seeds, len(traj64)))
            for s in range(seeds):
                pm = _Perturbed(model, s, ex)
                with torch.no_grad():
                    for i, out in enumerate(loop_fn(pm, init)):
                        e[s, i] = float((out['sample'].double() - torch.from_numpy(traj64[i]).double()).abs().max())
            arr[f'{name}_e64_p{-ex}'] = e
            print(name, f'2^{ex}-perturbed fp32 reference vs float64, max over steps per seed',
                  ['%.2e' % v for v in e.max(1)], flush=True)

    comb = admc.UNetCombined(**mg.ADM_ARCHS['adm_tiny']).eval()
    meta['combined_tiny_weights_sha256'] = mg.synthetic(comb)
    d = ddim.DDIMCFG(guidance_scale=2.5, respace_type='uniform', respace_steps=6, eta=0.0)
    labels = torch.from_numpy(adm['ddpm8_labels'])
    run('cfg6', comb, lambda m, x: d.sample_loop(m, x, model_kwargs=dict(y=labels), tqdm_kwargs=dict(disable=True)),
        torch.from_numpy(adm['cfg6_init']), drift['cfg6_sample64'])
    model = ua.UNetCategorialAdaGN(**mg.ADAGN_ARCHS['tiny_updown']).eval()
    meta['tiny_updown_weights_sha256'] = mg.synthetic(model)
    d2 = ddim.DDIMCFG(guidance_scale=3.0, respace_type='uniform', respace_steps=10, eta=0.0)
    torch.manual_seed(5)
    init = torch.randn((2, 3, 16, 16))
    run('adagn_cfg10', model, lambda m, x: d2.sample_loop(m, x, model_kwargs=dict(y=torch.tensor([1, 4])),
                                                          tqdm_kwargs=dict(disable=True)),
        init, drift['adagn_cfg10_sample64'])
    model = unet.UNet(**mg.ARCHS['tiny']).eval()
    meta['tiny_weights_sha256'] = mg.synthetic(model)
    d3 = ddim.DDIM(respace_type='uniform', respace_steps=5, eta=0.0)
    g = torch.Generator().manual_seed(31)
    img = torch.rand((2, 3, 16, 16), generator=g) * 2 - 1

    def inv_rec(m, x):
        for out in d3.sample_inversion_loop(m, x, tqdm_kwargs=dict(disable=True)):
            x = out['sample']
            yield out
        yield from d3.sample_loop(m, x, tqdm_kwargs=dict(disable=True))
    run('invrec', model, inv_rec, img, drift['invrec_sample64'])
    meta['perturbation'] = 'model output * (1 + 2^ex s), ex in (-22, -20), s = +-1 from torch.Generator(1000 + seed)'
    meta['seeds'] = seeds
    mg.save('chaos', meta, **arr)


if __name__ == '__main__':
    which = sys.argv[1:] or ['convert', 'stepacc', 'dit', 'chaos']
    for w in which:
        dict(convert=make_convert, stepacc=make_stepacc, dit=make_dit, chaos=make_chaos)[w]()
