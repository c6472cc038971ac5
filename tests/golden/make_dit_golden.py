"""Generate the DiT fixtures (tests/golden/dit.npz/.json) from the CPU ORACLE.

The reference DiT (models/dit/model.py) imports timm, which is not installed
here, so it cannot be executed; these fixtures come from oracle/dit.py, the
restatement of model.py + timm 0.9.12 PatchEmbed / Attention / Mlp. Parity of
the DiT path is therefore UNPINNED: the GPU tests check the HIP
path against this restatement, not against reference outputs.
    python tests/golden/make_dit_golden.py
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, 'diffusion-models-pytorch_amd')]

from oracle import diffusion as od  # noqa: E402
from oracle.dit import OracleDiT  # noqa: E402
from utils.synthetic import state_dict_sha256, synthetic_state_dict  # noqa: E402

ARCHS = {
    'dit_tiny': dict(input_size=8, patch_size=2, in_channels=4, hidden_size=64, depth=2, num_heads=4,
                     mlp_ratio=4.0, class_dropout_prob=0.1, num_classes=10, learn_sigma=True),
    'dit_s2': dict(input_size=16, patch_size=2, in_channels=4, hidden_size=384, depth=12, num_heads=6,
                   mlp_ratio=4.0, class_dropout_prob=0.1, num_classes=1000, learn_sigma=True),
    # DiT-XL/2 at the 256x256 config's latent size (weights/facebookresearch/DiT/DiT-XL-2-256x256.yaml)
    'dit_xl2': dict(input_size=32, patch_size=2, in_channels=4, hidden_size=1152, depth=28, num_heads=16,
                    mlp_ratio=4.0, class_dropout_prob=0.1, num_classes=1000, learn_sigma=True),
}


def state_dict_shapes(arch):
    """Key order / shapes of the reference DiT state_dict (pos_embed first: a direct Parameter)."""
    D, p, C = arch['hidden_size'], arch['patch_size'], arch['in_channels']
    T = (arch['input_size'] // p) ** 2
    Hm = int(D * arch['mlp_ratio'])
    oc = 2 * C if arch['learn_sigma'] else C
    ncls = arch['num_classes'] + int(arch['class_dropout_prob'] > 0)
    keys = [('pos_embed', [1, T, D]), ('x_embedder.proj.weight', [D, C, p, p]), ('x_embedder.proj.bias', [D]),
            ('t_embedder.mlp.0.weight', [D, 256]), ('t_embedder.mlp.0.bias', [D]),
            ('t_embedder.mlp.2.weight', [D, D]), ('t_embedder.mlp.2.bias', [D]),
            ('y_embedder.embedding_table.weight', [ncls, D])]
    for b in range(arch['depth']):
        keys += [(f'blocks.{b}.attn.qkv.weight', [3 * D, D]), (f'blocks.{b}.attn.qkv.bias', [3 * D]),
                 (f'blocks.{b}.attn.proj.weight', [D, D]), (f'blocks.{b}.attn.proj.bias', [D]),
                 (f'blocks.{b}.mlp.fc1.weight', [Hm, D]), (f'blocks.{b}.mlp.fc1.bias', [Hm]),
                 (f'blocks.{b}.mlp.fc2.weight', [D, Hm]), (f'blocks.{b}.mlp.fc2.bias', [D]),
                 (f'blocks.{b}.adaLN_modulation.1.weight', [6 * D, D]),
                 (f'blocks.{b}.adaLN_modulation.1.bias', [6 * D])]
    keys += [('final_layer.linear.weight', [p * p * oc, D]), ('final_layer.linear.bias', [p * p * oc]),
             ('final_layer.adaLN_modulation.1.weight', [2 * D, D]),
             ('final_layer.adaLN_modulation.1.bias', [2 * D])]
    return keys


def oracle_model(arch):
    keys = state_dict_shapes(arch)
    sd = synthetic_state_dict({k: torch.empty(s) for k, s in keys})
    oc = 2 * arch['in_channels'] if arch['learn_sigma'] else arch['in_channels']
    model = OracleDiT(sd, patch_size=arch['patch_size'], num_heads=arch['num_heads'], depth=arch['depth'],
                      num_classes=arch['num_classes'], out_channels=oc)
    return model, state_dict_sha256(sd), keys


def main():
    torch.set_num_threads(8)
    meta = dict(torch=torch.__version__, generator='oracle/dit.py (parity unpinned: timm absent)', archs=ARCHS)
    fx = {}
    g = torch.Generator().manual_seed(41)
    for name, arch in ARCHS.items():
        model, sha, keys = oracle_model(arch)
        meta[f'{name}_weights_sha256'] = sha
        meta[f'{name}_state_dict'] = [[k, s] for k, s in keys]
        B = 1 if name == 'dit_xl2' else 2
        S = arch['input_size']
        x = torch.randn((B, arch['in_channels'], S, S), generator=g)
        t = torch.tensor([999, 12][:B])
        y = torch.tensor([7, 3][:B])
        fx[f'{name}_out_y'] = model(x, t, y)
        fx[f'{name}_out_null'] = model(x, t, None)
        fx[f'{name}_x'], fx[f'{name}_t'], fx[f'{name}_labels'] = x, t, y
        print(name, 'done', flush=True)
    # DDIMCFG-5 (s = 4) on dit_tiny, learned-sigma outputs, labels [3, 7]
    model, _, _ = oracle_model(ARCHS['dit_tiny'])
    ac = od.alphas_cumprod(od.beta_schedule(1000, 'linear'))
    seq = od.respaced_seq(1000, 'uniform', 5)
    torch.manual_seed(43)
    init = torch.randn((2, 4, 8, 8))
    labels = torch.tensor([3, 7])
    fx['cfg5_init'], fx['cfg5_labels'] = init, labels
    for i, out in enumerate(od.sample_loop(model, ac, seq, init, sampler='ddim', eta=0.0, guidance_scale=4.0,
                                           y=labels)):
        fx[f'cfg5_step{i}_sample'] = out['sample']
    meta['cfg5'] = dict(guidance_scale=4.0, respace_type='uniform', respace_steps=5, eta=0.0)
    arrays = {k: v.detach().numpy() for k, v in fx.items()}
    np.savez_compressed(os.path.join(HERE, 'dit.npz'), **arrays)
    with open(os.path.join(HERE, 'dit.json'), 'w') as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print({k: v.shape for k, v in arrays.items()})


if __name__ == '__main__':
    main()
