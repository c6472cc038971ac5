"""Classifier-free-guidance sampling — drop-in for the reference scripts/sample_cfg.py.

Same CLI (config, seed, weights, guidance_scale, class_ids,
n_samples_each_class, save_dir, batch_size, sampler, respace_type,
respace_steps, var_type, ddim_eta). Reference semantics kept on purpose
(sample_cfg.py:169-177): each fold draws `bs` (not bspp) images per rank and
`gather(...)[:bs]` keeps rank 0's images; `--shard` switches to proper
per-rank sharding (bspp per rank) for throughput runs.

Latent denoisers (models.base_latent.BaseLatent, e.g. DiT-XL/2 with
weights/facebookresearch/DiT/DiT-XL-2-256x256.yaml) cannot run through the
reference script (it draws image-shaped noise); for them this script follows
the reference's only latent sampling driver, the Streamlit class-conditional
page (streamlit/pages/2_Class_conditional_Image_Generation.py:46-60, 90-103):
  * noise of shape (4, img_size / 8, img_size / 8) (:91-95);
  * the diffusion's YAML params are honoured, `clip_denoised: false` and
    `var_type` included (:51-59 instantiate the sampler from them);
  * the unconditional branch is the null class (DiT y=None), run together with
    the conditional one as one 2B forward.
Multi-GPU follows sample_uncond's seed + rank sharding (the
reference has no multi-GPU latent path): every rank samples bspp latents per
fold and the fold is gathered once. Latents are decoded with the model's VAE
when one can be built (`decode_latent`); the reference's VAE is a network
download (models/dit/autoencoder.py), so without it the clamp-free latents are
written as `{idx}.npy` (float32 [4, S, S]) instead of PNGs.
"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import diffusions  # noqa: E402
from models.base_latent import BaseLatent  # noqa: E402
from scripts.sample_uncond import build_model  # noqa: E402
from utils.harness import DistEnv, per_process_batch  # noqa: E402
from utils.misc import amortize, image_norm_to_float, load_config  # noqa: E402
from utils.png import save_image  # noqa: E402


def get_parser():
    p = argparse.ArgumentParser()
    p.add_argument('-c', '--config', type=str, required=True)
    p.add_argument('--seed', type=int, default=2022)
    p.add_argument('--weights', type=str, required=True, help="Path to model weights, or 'synthetic'")
    p.add_argument('--guidance_scale', type=float, required=True)
    p.add_argument('--class_ids', type=int, nargs='+', default=None)
    p.add_argument('--n_samples_each_class', type=int, required=True)
    p.add_argument('--save_dir', type=str, required=True)
    p.add_argument('--batch_size', type=int, default=500)
    p.add_argument('--sampler', type=str, choices=['ddpm', 'ddim'], default='ddpm')
    p.add_argument('--respace_type', type=str, default='uniform')
    p.add_argument('--respace_steps', type=int, default=None)
    p.add_argument('--var_type', type=str, default=None)
    p.add_argument('--ddim_eta', type=float, default=0.0)
    p.add_argument('--shard', action='store_true', help='shard each fold across ranks (not reference behaviour)')
    return p


def build_cfg_diffuser(args, conf, device, latent=False):
    """Reference sample_cfg.py:111-138; for latent models the Streamlit page's build_diffuser
    (streamlit/pages/2_...py:46-60: every YAML diffusion param, clip_denoised included)."""
    dp = conf.diffusion.params
    common = dict(
        total_steps=dp.total_steps, beta_schedule=dp.beta_schedule, beta_start=dp.beta_start,
        beta_end=dp.beta_end, objective=dp.objective,
        respace_type=None if args.respace_steps is None else args.respace_type,
        respace_steps=args.respace_steps or dp.total_steps, device=device, guidance_scale=args.guidance_scale,
    )
    if latent:
        common['clip_denoised'] = dp.get('clip_denoised', True)
    if args.sampler == 'ddpm':
        return diffusions.ddpm.DDPMCFG(var_type=args.var_type or dp.get('var_type', None), **common)
    return diffusions.ddim.DDIMCFG(eta=args.ddim_eta, **common)


@torch.no_grad()
def main(argv=None):
    args, unknown = get_parser().parse_known_args(argv)
    unknown = [(a[2:] if a.startswith('--') else a) for a in unknown]
    conf = load_config(args.config, [f'{k}={v}' for k, v in zip(unknown[::2], unknown[1::2])])
    env = DistEnv()
    torch.manual_seed(args.seed + env.rank)
    model = build_model(conf, args.weights, env.device)
    latent = isinstance(model, BaseLatent)
    diffuser = build_cfg_diffuser(args, conf, env.device, latent=latent)
    size = conf.data.params.img_size
    img_shape = (4, size // 8, size // 8) if latent else (conf.data.img_channels, size, size)
    shard = args.shard or latent
    bspp = per_process_batch(args.n_samples_each_class, args.batch_size, env.world)
    class_ids = args.class_ids if args.class_ids is not None else range(conf.data.num_classes)
    for c in class_ids:
        os.makedirs(os.path.join(args.save_dir, f'class{c}'), exist_ok=True)
        idx = 0
        for i, bs in enumerate(amortize(args.n_samples_each_class, bspp * env.world)):
            n = bspp if shard else bs
            init_noise = torch.randn((n, *img_shape), device=env.device)
            labels = torch.full((n, ), fill_value=c, device=env.device, dtype=torch.long)
            samples = diffuser.sample(model=model, init_noise=init_noise, model_kwargs=dict(y=labels),
                                      tqdm_kwargs=dict(desc=f'Fold {i}', disable=not env.is_main))
            samples = env.gather(samples if latent else samples.clamp(-1, 1))[:bs]
            if env.is_main:
                idx = save_fold(model, samples, os.path.join(args.save_dir, f'class{c}'), idx, latent)
    env.barrier()
    env.close()


def save_fold(model, samples, out_dir, idx, latent):
    """One PNG per image; latents are decoded first (Streamlit page :102-103), or kept as .npy when the
    model's VAE cannot be built offline."""
    if latent:
        try:
            samples = model.decode_latent(samples).clamp(-1, 1)
        except NotImplementedError:
            for z in samples:
                np.save(os.path.join(out_dir, f'{idx}.npy'), z.float().cpu().numpy())
                idx += 1
            return idx
    for x in samples:
        save_image(image_norm_to_float(x.cpu()), os.path.join(out_dir, f'{idx}.png'))
        idx += 1
    return idx


if __name__ == '__main__':
    main()
