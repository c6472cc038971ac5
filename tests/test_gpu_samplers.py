"""Euler and Heun samplers (reference diffusions/euler.py, heun.py) on the engine.

Golden fixtures: tests/golden/samplers.npz, generated from the reference modules themselves
(tests/golden/make_golden.py samplers). Updates: bit-identical to the oracle (oracle/diffusion.py,
reference op order) on this host and within a few ulp of the golden file from the build container's CPU
(torch 0-dim sqrt/pow round host-dependently). Trajectories: per step <= 1e-4.
"""
import numpy as np
import pytest
import torch

from diffusions import EulerSampler, HeunSampler
from tests.test_gpu_parity import TOL, _model

pytestmark = pytest.mark.gpu


def test_euler_heun_updates_bit_exact(cuda, golden):
    from oracle import diffusion as od
    arrays, meta = golden('samplers')
    ac = od.alphas_cumprod(od.beta_schedule(1000, 'linear'))
    sig = od.sigmas(ac)
    for i, (t, tp) in enumerate(meta['update_pairs']):
        xt, out = (torch.from_numpy(arrays[f'upd{i}_{k}']) for k in ('xt', 'out'))
        e = EulerSampler(respace_type='uniform', respace_steps=10, device=cuda)
        got = e.denoise(out.to(cuda), xt.to(cuda), t, tp)
        ref = od.euler_denoise(ac, sig, out.clone(), xt, t, tp)
        for k, gk in (('sample', 'euler_sample'), ('pred_x0', 'euler_x0')):
            g = got[k].cpu().numpy()
            assert np.array_equal(g, ref[k].numpy()), (t, k, np.abs(g - ref[k].numpy()).max())
            assert np.allclose(g, arrays[f'upd{i}_{gk}'], rtol=1e-5, atol=2e-5), (t, k)
        if tp < 0:
            continue
        h = HeunSampler(respace_type='uniform', respace_steps=10, device=cuda)
        h.denoise_1st_order(out.to(cuda), xt.to(cuda), t, tp)
        xp, out2 = (torch.from_numpy(arrays[f'upd{i}_{k}']) for k in ('xprev', 'out2'))
        got2 = h.denoise_2nd_order(out2.to(cuda), xp.to(cuda), t, tp)
        ref2 = od.heun_denoise_2nd(ac, sig, out2.clone(), xp, t, tp, ref['derivative'], xt)
        for k, gk in (('sample', 'heun2_sample'), ('pred_x0', 'heun2_x0')):
            g = got2[k].cpu().numpy()
            assert np.array_equal(g, ref2[k].numpy()), (t, k, np.abs(g - ref2[k].numpy()).max())
            assert np.allclose(g, arrays[f'upd{i}_{gk}'], rtol=1e-5, atol=2e-5), (t, k)


def test_heun_second_order_needs_first():
    h = HeunSampler(respace_type='uniform', respace_steps=10)
    with pytest.raises(RuntimeError):
        h.denoise_2nd_order(torch.zeros(1), torch.zeros(1), 900, 800)


@pytest.mark.parametrize('name,cls', [('euler5', EulerSampler), ('heun5', HeunSampler)])
def test_euler_heun_trajectories(cuda, golden, report, name, cls):
    arrays, meta = golden('samplers')
    fmeta = golden('forward')[1]
    model, sha = _model(fmeta, 'tiny', cuda)
    assert sha == meta['tiny_weights_sha256']
    d = cls(respace_type='uniform', respace_steps=5, device=cuda)
    init = torch.from_numpy(arrays[f'{name}_init']).to(cuda)
    worst = 0.0
    for i, out in enumerate(d.sample_loop(model, init, tqdm_kwargs=dict(disable=True))):
        err = np.abs(out['sample'].cpu().numpy() - arrays[f'{name}_step{i}_sample']).max()
        worst = max(worst, err)
        assert err <= TOL, (name, i, err)
    report(f'{name}_tiny_worst_step_maxabs_vs_reference', worst)


@pytest.mark.parametrize('sampler,mode', [('euler', 'interpolate'), ('heun', 'sample'), ('ddim', 'progressive')])
def test_sample_uncond_script(cuda, tmp_path, sampler, mode):
    """scripts/sample_uncond.py end to end on the engine (MNIST config, synthetic weights, 2 steps):
    the reference's sampler x mode matrix (sample_uncond.py:22-27, 179-276) writes one PNG per image."""
    import os
    from scripts import sample_uncond
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cfg = os.path.join(root, 'diffusion-models-pytorch_amd', 'configs', 'ddpm_mnist.yaml')
    sample_uncond.main(['-c', cfg, '--weights', 'synthetic', '--n_samples', '3', '--batch_size', '2',
                        '--save_dir', str(tmp_path), '--sampler', sampler, '--mode', mode,
                        '--respace_steps', '4', '--n_interpolate', '3', '--n_progressive', '2'])
    files = sorted(os.listdir(tmp_path))
    assert files == ['0.png', '1.png', '2.png'], files


def test_ddim_inversion_reconstruction_trajectory(cuda, golden, report):
    """DDIM.sample_inversion_loop then sample_loop on the engine vs the reference (ddim.py:88-132,
    sample_uncond.py:297-304; tests/golden/inversion.npz). Every step teacher-forced from the reference's
    previous sample <= 1e-4; free-running (inversion feeding reconstruction): tests/conftest.py
    check_free_running. x0 = sqrt(1/ac_t) x - ... amplifies a 1e-6 forward difference by up to ~160 at
    t ~ 960 and the reference's own fp32 run drifts 3e-4 from its float64 run here
    (tests/golden/drift.npz invrec, make_golden_r2.py)."""
    from tests.conftest import check_chaos_envelope, check_free_running
    dg = golden('drift')[0]
    drift = dg['invrec_drift_sample']
    from diffusions import DDIM
    arrays, meta = golden('inversion')
    model, sha = _model(golden('forward')[1], 'tiny', cuda)
    assert sha == meta['tiny_weights_sha256']
    d = DDIM(respace_type='uniform', respace_steps=5, eta=0.0, device=cuda)
    seq = d.respaced_seq.tolist()
    ref = lambda k: torch.from_numpy(arrays[k]).to(cuda)  # noqa: E731
    tb = lambda t: torch.full((2, ), t, dtype=torch.long, device=cuda)  # noqa: E731
    forced = 0.0
    for i, (t, tn) in enumerate(zip(seq[:-1], seq[1:])):
        x = ref('img') if i == 0 else ref(f'inv_step{i - 1}_sample')
        out = d.denoise_inversion(model(x, tb(t)), x, t, tn)
        err = np.abs(out['sample'].cpu().numpy() - arrays[f'inv_step{i}_sample']).max()
        forced = max(forced, err)
        assert err <= TOL, ('inv', i, err)
    prev = [-1] + seq[:-1]
    for i, (t, tp) in enumerate(zip(reversed(seq), reversed(prev))):
        x = ref(f'inv_step{meta["inv_steps"] - 1}_sample') if i == 0 else ref(f'rec_step{i - 1}_sample')
        out = d.denoise(model(x, tb(t)), x, t, tp)
        err = np.abs(out['sample'].cpu().numpy() - arrays[f'rec_step{i}_sample']).max()
        forced = max(forced, err)
        assert err <= TOL, ('rec', i, err)
    free, free64 = 0.0, 0.0
    x = ref('img')
    for i, out in enumerate(d.sample_inversion_loop(model, x, tqdm_kwargs=dict(disable=True))):
        err, e64 = check_free_running(out['sample'].cpu().numpy(), arrays[f'inv_step{i}_sample'],
                                      dg['invrec_sample64'][i], drift, i)
        free, free64 = max(free, err), max(free64, e64)
        x = out['sample']
    n_inv = i + 1
    assert n_inv == meta['inv_steps']
    for i, out in enumerate(d.sample_loop(model, x, tqdm_kwargs=dict(disable=True))):
        err, e64 = check_free_running(out['sample'].cpu().numpy(), arrays[f'rec_step{i}_sample'],
                                      dg['invrec_sample64'][n_inv + i], drift, n_inv + i)
        free, free64 = max(free, err), max(free64, e64)
    report('ddim_inversion_reconstruction_tiny_teacher_forced_maxabs_vs_reference', forced)
    report('ddim_inversion_reconstruction_tiny_free_running_maxabs_vs_reference', free)
    report('ddim_inversion_reconstruction_tiny_reference_fp32_vs_fp64_drift', float(drift.max()))
    report('ddim_inversion_reconstruction_tiny_free_running_maxabs_vs_float64', free64)
    check_chaos_envelope(golden, 'invrec', free64, report, 'ddim_inversion_reconstruction_tiny')


def test_sample_uncond_reconstruction(cuda, tmp_path):
    """--mode reconstruction (sample_uncond.py:279-336): inverts every image under --input_dir and writes
    [input, reconstruction] as one nrow=2 grid per image; a missing --input_dir is a ValueError."""
    import os
    from PIL import Image
    from scripts import sample_uncond
    from utils.png import read_png_rgb
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cfg = os.path.join(root, 'diffusion-models-pytorch_amd', 'configs', 'ddpm_cifar10.yaml')
    src = tmp_path / 'in'
    src.mkdir()
    rng = np.random.default_rng(1)
    for k in range(3):
        Image.fromarray(rng.integers(0, 256, (32, 32, 3), dtype=np.uint8)).save(src / f'{k}.png')
    out = tmp_path / 'out'
    args = ['-c', cfg, '--weights', 'synthetic', '--n_samples', '3', '--batch_size', '2', '--save_dir', str(out),
            '--sampler', 'ddim', '--respace_steps', '3', '--mode', 'reconstruction']
    with pytest.raises(ValueError):
        sample_uncond.main(args)
    sample_uncond.main(args + ['--input_dir', str(src)])
    assert sorted(os.listdir(out)) == ['0.png', '1.png', '2.png']
    grid = read_png_rgb(str(out / '1.png'))
    assert grid.shape == (36, 70, 3)
    # the left tile is the input image itself ((x+1)/2 of its normalised value round-trips the bytes)
    assert np.array_equal(grid[2:34, 2:34], np.asarray(Image.open(src / '1.png')))
