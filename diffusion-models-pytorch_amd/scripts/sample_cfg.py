"""Classifier-free-guidance sampling — drop-in for the reference scripts/sample_cfg.py.

Same CLI (config, seed, weights, guidance_scale, class_ids,
n_samples_each_class, save_dir, batch_size, sampler, respace_type,
respace_steps, var_type, ddim_eta). Reference semantics kept on purpose
(sample_cfg.py:169-177): each fold draws `bs` (not bspp) images per rank and
`gather(...)[:bs]` keeps rank 0's images; `--shard` switches to proper
per-rank sharding (bspp per rank) for throughput runs.
"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import diffusions  # noqa: E402
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


def build_cfg_diffuser(args, conf, device):
    """Reference sample_cfg.py:111-138."""
    dp = conf.diffusion.params
    common = dict(
        total_steps=dp.total_steps, beta_schedule=dp.beta_schedule, beta_start=dp.beta_start,
        beta_end=dp.beta_end, objective=dp.objective,
        respace_type=None if args.respace_steps is None else args.respace_type,
        respace_steps=args.respace_steps or dp.total_steps, device=device, guidance_scale=args.guidance_scale,
    )
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
    diffuser = build_cfg_diffuser(args, conf, env.device)
    model = build_model(conf, args.weights, env.device)
    img_shape = (conf.data.img_channels, conf.data.params.img_size, conf.data.params.img_size)
    bspp = per_process_batch(args.n_samples_each_class, args.batch_size, env.world)
    class_ids = args.class_ids if args.class_ids is not None else range(conf.data.num_classes)
    for c in class_ids:
        os.makedirs(os.path.join(args.save_dir, f'class{c}'), exist_ok=True)
        idx = 0
        for i, bs in enumerate(amortize(args.n_samples_each_class, bspp * env.world)):
            n = bspp if args.shard else bs
            init_noise = torch.randn((n, *img_shape), device=env.device)
            labels = torch.full((n, ), fill_value=c, device=env.device, dtype=torch.long)
            samples = diffuser.sample(model=model, init_noise=init_noise, model_kwargs=dict(y=labels),
                                      tqdm_kwargs=dict(desc=f'Fold {i}', disable=not env.is_main)).clamp(-1, 1)
            samples = env.gather(samples)[:bs]
            if env.is_main:
                for x in samples:
                    save_image(image_norm_to_float(x.cpu()), os.path.join(args.save_dir, f'class{c}', f'{idx}.png'))
                    idx += 1
    env.barrier()
    env.close()


if __name__ == '__main__':
    main()
