"""Benchmark: images/sec of DDIM-50 sampling with the CIFAR-10 UNet on MI355X.

BASELINE.json metric "images/sec at DDIM-50, CIFAR-10 UNet 32x32, bs=256;
1/2/4/8 GPU". One bench *step* = one sampling fold of the reference harness
(scripts/sample_uncond.py:184-190): B=256 init-noise images per GPU pushed
through the 50 DDIM steps (model forward + fused update on each), clamped,
and all-gathered over RCCL when N > 1. Weights are the deterministic
synthetic CIFAR-10 UNet (35.7M params, rank-independent); noise is drawn on
device from a per-rank seed (2022 + rank, as the reference seeds).

Timing: W untimed warmup folds, then K folds bracketed by barrier +
torch.cuda.synchronize(); the MAX over ranks is reported; `value` = images of
all ranks / that time.

Roofline: HIP events around every launch of the forward during the timed
region (dm_unet_profile) give each kernel family's average launch duration;
the dominant family (most GPU time) is reported with its algorithmic (fp32)
FLOPs per launch against the peak of the instructions it issues: the fp32 MFMA
peak (157.3 TF) for the fp32 kernels; for the split kernels, which issue each
fp32 product as P 16-bit piece products, the dense bf16/fp16 MFMA peak / P
(fp16x2, the default: P = 3, 2500 / 3 = 833.3 TF of fp32-equivalent work;
bf16x3: P = 6, 416.7 TF).

CPU baseline: the oracle (a torch-CPU restatement of the reference path,
bit-equal to it at equal thread count) timed on all usable host cores, rank 0 /
N=1 only: one warm-up step and 8 timed denoising steps of the same B=256 fold
(about 10 s of CPU work: the 3-step sample of round 3 scattered 0.79-0.88 img/s
between boxes), extrapolated x50.
"""
import argparse
import ctypes
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, 'diffusion-models-pytorch_amd')
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = 'images/sec at DDIM-50, CIFAR-10 UNet 32×32, bs=256; 1/2/4/8 GPU'
FP32_PEAK_TFLOPS = 157.3   # MI355X dense fp32 (MFMA f32 = vector rate), MI355X_MICROARCH.md
BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (no sparsity), MI355X_MICROARCH.md
SPLIT_PRODUCTS = {2: 3, 3: 6}  # conv_patch3_kernel<..., NP>: fp16x2 issues 3, bf16x3 6 piece products per product
HBM_PEAK_GBS = 8000.0
PROFILE_EVERY = 10   # per-launch events cost ~5 % when on every launch; 1 forward in 10 is observed


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=3, help='timed folds')
    ap.add_argument('--warmup', type=int, default=1, help='untimed folds')
    ap.add_argument('--workload', default='c3', choices=sorted(WORKLOADS) + ['stub'],
                    help='; '.join(f'{k}: {v}' for k, v in sorted(WORKLOADS.items())))
    ap.add_argument('--batch', type=int, default=None, help='images per GPU per fold (default: the workload\'s)')
    ap.add_argument('--respace-steps', type=int, default=None, help='denoising steps (default: the workload\'s)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-batch', type=int, default=256, help='batch of the timed CPU denoising step')
    ap.add_argument('--profile-json', default=None, help='write the per-op profile here (rank 0)')
    ap.add_argument('--no-profile', action='store_true',
                    help='no per-launch HIP events in the timed region (roofline fields then null)')
    return ap.parse_args()


def pmc_traffic(label, workload='c3', build=None, launches_per_forward=None, root=ROOT):
    """HBM bytes per launch of `label` from the newest committed PMC summary of this workload
    (profiles/rNN_vM_pmc.json, FETCH_SIZE x2 + WRITE_SIZE passes of this bench, tools/gpu_profile.sh;
    summaries without a "workload" field are of the default c3 run) -- only from a summary of the SAME library
    build (its "build" = dm_build_info() of this run) in which `label` ran as many launches per network forward
    as in this run; none such: (None, None), and the roofline's traffic is null."""
    import glob
    import re

    def order(path):
        m = re.search(r'r(\d+)_v(\d+)(?:_c\d)?_pmc\.json$', path)
        return (int(m.group(1)), int(m.group(2))) if m else (-1, -1)
    files = sorted(glob.glob(os.path.join(root, 'profiles', 'r*_v*_pmc.json')), key=order)
    for path in reversed(files):
        with open(path) as f:
            summary = json.load(f)
        if summary.get('workload', 'c3') != workload or build is None or summary.get('build') != build:
            continue
        k = summary.get('kernels', {}).get(label)
        if not k or not k.get('hbm_bytes_per_launch') or launches_per_forward is None or \
                k.get('launches_per_forward') is None or abs(k['launches_per_forward'] - launches_per_forward) > 1e-6:
            continue
        return float(k['hbm_bytes_per_launch']), os.path.relpath(path, root)
    return None, None


def cpu_model_name():
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or 'unknown'


def usable_cores():
    """CPUs this process may run on: the affinity mask, capped by a cgroup v2 CPU quota if one is set."""
    n = len(os.sched_getaffinity(0))
    try:
        with open('/sys/fs/cgroup/cpu.max') as f:
            quota, period = f.read().split()[:2]
        if quota != 'max':
            n = min(n, max(1, int(-(-int(quota) // int(period)))))
    except (OSError, ValueError):
        pass
    return n


def cpu_baseline(sd, batch, n_steps, timed_steps=8):
    """Oracle (reference op sequence on torch CPU) per BASELINE.md §4: all usable host cores, one warm-up
    step at the config's batch, then `timed_steps` denoising steps (forward + DDIM update) timed at that
    batch; images/sec = batch / (t_step x n_steps) (the per-step cost does not depend on t)."""
    from oracle.unet import OracleUNet
    from oracle import diffusion as od
    threads = usable_cores()
    prev_threads = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        model = OracleUNet(sd, dim=128)
        ac = od.alphas_cumprod(od.beta_schedule(1000, 'linear'))
        seq = od.respaced_seq(1000, 'uniform', n_steps).tolist()
        g = torch.Generator().manual_seed(2022)
        x = torch.randn((batch, 3, 32, 32), generator=g)
        pairs = list(zip(reversed(seq), reversed([-1] + seq[:-1])))
        with torch.no_grad():
            t, tp = pairs[0]
            x = od.ddim_denoise(ac, model(x, torch.full((batch, ), t)), x, t, tp)['sample']  # warm-up
            t0 = time.perf_counter()
            for t, tp in pairs[1:1 + timed_steps]:
                x = od.ddim_denoise(ac, model(x, torch.full((batch, ), t)), x, t, tp)['sample']
            dt = (time.perf_counter() - t0) / timed_steps
    finally:
        torch.set_num_threads(prev_threads)
    return dict(value=batch / (dt * n_steps), unit='images/sec', cores=threads, kind='port',
                sample=f'{timed_steps} of {n_steps} DDIM steps (UNet forward + update) timed at B={batch} after '
                       f'1 warm-up step, torch CPU on {threads} threads ({cpu_model_name()}, '
                       f'{os.cpu_count()} logical CPUs on the host); {dt:.2f} s per step, extrapolated x{n_steps}')


def cpu_baseline_cfg(name, model_sd, arch, batch, n_steps, guidance_scale, timed_steps, clip=True):
    """Secondary workloads (bounded sample): the oracle of the ADM (c4: oracle/adm.py,
    UNetCombined routing) or DiT (c5: oracle/dit.py) denoiser on all usable host cores, one warm-up
    step, then `timed_steps` DDIMCFG steps (cond + uncond forward, predict, combine, update) at `batch`;
    images/sec = batch / (t_step x n_steps)."""
    from oracle import diffusion as od
    threads = usable_cores()
    prev_threads = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        if name == 'c4':
            from oracle.adm import OracleADMCombined
            model = OracleADMCombined(model_sd, **arch)
            shape = (batch, 3, arch['image_size'], arch['image_size'])
        else:
            from oracle.dit import OracleDiT
            model = OracleDiT(model_sd, **arch)
            shape = (batch, arch['in_channels'], arch['input_size'], arch['input_size'])
        ac = od.alphas_cumprod(od.beta_schedule(1000, 'linear'))
        seq = od.respaced_seq(1000, 'uniform', n_steps)
        g = torch.Generator().manual_seed(2022)
        x = torch.randn(shape, generator=g)
        y = torch.zeros((batch, ), dtype=torch.long)
        sub = torch.tensor(seq.tolist()[-(timed_steps + 1):])   # the first timed_steps + 1 steps of the loop
        with torch.no_grad():
            it = od.sample_loop(model, ac, sub, x, sampler='ddim', eta=0.0, guidance_scale=guidance_scale, y=y,
                                clip=clip)
            next(it)   # warm-up step
            t0 = time.perf_counter()
            for _ in range(timed_steps):
                next(it)
            dt = (time.perf_counter() - t0) / timed_steps
    finally:
        torch.set_num_threads(prev_threads)
    return dict(value=batch / (dt * n_steps), unit='images/sec', cores=threads, kind='port',
                sample=f'{timed_steps} of {n_steps} DDIMCFG steps (cond + uncond forward + update) timed at B={batch} '
                       f'after 1 warm-up step, torch CPU on {threads} threads ({cpu_model_name()}, '
                       f'{os.cpu_count()} logical CPUs on the host); {dt:.2f} s per step, extrapolated x{n_steps}')


WINO_PRODUCTS = 2.0 / 3.0   # conv_wino_kernel: F(2,3) issues 12 K-rows per output pair where the direct conv issues 18


def roofline(prof, workload='c3', build=None, launches_per_forward=None):
    """Roofline of the dominant kernel family (most GPU time in the timed region). launches_per_forward: label ->
    launches per network forward in this run (pmc_traffic's match key)."""
    fam = {}
    for op in prof:
        f = fam.setdefault(op['label'], dict(flops=0.0, bytes=0.0, ms=0.0, launches=0))
        f['flops'] += op['flops'] * op['launches']
        f['bytes'] += op['bytes'] * op['launches']
        f['ms'] += op['ms_total']
        f['launches'] += op['launches']
    dom_name, dom = max(fam.items(), key=lambda kv: kv[1]['ms'])
    avg_ms = dom['ms'] / max(1, dom['launches'])
    flops_per_launch = dom['flops'] / max(1, dom['launches'])
    bytes_per_launch = dom['bytes'] / max(1, dom['launches'])
    if flops_per_launch > 0:
        achieved = flops_per_launch / (avg_ms * 1e-3) / 1e12
        split = dom_name.startswith('conv_patch3_kernel')
        np_ = int(dom_name.rstrip('>').split(',')[-1]) if split else 0
        if dom_name.startswith('gemm_kernel') and dom_name.endswith(',true>'):   # <..., B_KN, SPLIT>: fp16x2
            split, np_ = True, 2
        if dom_name.startswith(('conv_k32_kernel', 'conv_k32s_kernel', 'linear_k32_kernel', 'conv_wino_kernel',
                                 'conv_wino_wide_kernel')):
            split, np_ = True, 2   # fp16x2 only
        wino = dom_name.startswith(('conv_wino_kernel', 'conv_wino_wide_kernel'))
        prods = SPLIT_PRODUCTS.get(np_, 0)
        # FLOPs are the direct convolution's (2 M N K) for every conv kernel; the Winograd kernel issues WINO_PRODUCTS
        # of its products, so its peak in those FLOPs is the issue peak / WINO_PRODUCTS
        peak = round(BF16_PEAK_TFLOPS / prods / (WINO_PRODUCTS if wino else 1.0), 1) if split else FP32_PEAK_TFLOPS
        roof = dict(bound='mfma', achieved=round(achieved, 2), peak=peak, unit='TFLOP/s',
                    frac=round(achieved / peak, 4), traffic=None)
        if split:
            kind = {2: 'fp16x2', 3: 'bf16x3'}[np_]
            issued = achieved * prods * (WINO_PRODUCTS if wino else 1.0)
            roof['peak_basis'] = (f'fp32-equivalent: dense 16-bit MFMA {BF16_PEAK_TFLOPS:.0f} TF / {prods} '
                                  f'piece products per fp32 product ({kind})' +
                                  (' / (2/3): achieved and peak in direct-convolution FLOPs (2 M N 9 Cin), of which '
                                   'the Winograd F(2,3) kernel issues 2/3 as products (12 K-rows per output pixel pair '
                                   'where the direct conv takes 18; its ResBlock-shortcut variants issue their 1x1 '
                                   'segment at the direct count, so this peak is an upper bound for those)'
                                   if wino else '') +
                                  f'; issued 16-bit MFMA rate {issued:.1f} TF of {BF16_PEAK_TFLOPS:.0f}; vs the fp32 '
                                  f'MFMA peak {achieved / FP32_PEAK_TFLOPS:.3f}')
    else:
        achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
        roof = dict(bound='hbm', achieved=round(achieved, 1), peak=HBM_PEAK_GBS, unit='GB/s',
                    frac=round(achieved / HBM_PEAK_GBS, 4), traffic=None)
    lpf = (launches_per_forward or {}).get(dom_name)
    traffic, traffic_src = pmc_traffic(dom_name, workload, build, lpf)
    roof.update(traffic=traffic, traffic_source=traffic_src, algorithmic_bytes_per_launch=bytes_per_launch,
                traffic_over_algorithmic=round(traffic / bytes_per_launch, 3) if traffic and bytes_per_launch else None,
                kernel=dom_name, avg_launch_ms=round(avg_ms, 4), launches=dom['launches'], launches_per_forward=lpf,
                build=build,
                algorithmic_per_launch=flops_per_launch if flops_per_launch > 0 else bytes_per_launch)
    total_gpu_ms = sum(f['ms'] for f in fam.values())
    total_flops = sum(f['flops'] for f in fam.values())
    return roof, total_gpu_ms, total_flops, fam


WORKLOADS = {
    'c3': 'DDIM-50 CIFAR-10 UNet, B=256 per GPU (BASELINE configs[2]; the headline metric)',
    'c2': 'DDPM-1000 fixed_large CIFAR-10 UNet, B=256 (BASELINE configs[1])',
    'c4': 'ADM guided-diffusion 256x256 UNetCombined, DDIMCFG-100 s=3, B=64 (BASELINE configs[3])',
    'c5': 'DiT-XL/2 latent 4x32x32, DDIMCFG-250 s=3, clip_denoised false, B=32 per GPU (BASELINE configs[4])',
}


def build_workload(name, args, dev, rank):
    """-> dict(metric, fold(), handles [(handle, abi, forwards per fold)], images, workload, config, sd_cpu).
    Every workload is one sampling fold of the reference harness on device-resident synthetic inputs."""
    from diffusions import DDIM, DDIMCFG, DDPM
    from utils.misc import instantiate_from_config, load_config
    from utils.synthetic import init_synthetic_
    gen = torch.Generator(device=dev)
    gen.manual_seed(2022 + rank)
    cfgdir = os.path.join(PKG, 'configs')
    if name in ('c2', 'c3'):
        from models.unet import UNet
        model = UNet().eval()
        init_synthetic_(model)
        sd_cpu = {k: v.clone() for k, v in model.state_dict().items()}
        model = model.to(dev)
        B = args.batch or 256
        steps = args.respace_steps or (50 if name == 'c3' else 1000)
        if name == 'c3':
            diffuser = DDIM(respace_type='uniform', respace_steps=steps, eta=0.0, device=dev)
            label = f'DDIM-{steps} (eta=0)'
            metric = METRIC
        else:
            diffuser = DDPM(var_type='fixed_large', respace_type=None if steps == 1000 else 'uniform',
                            respace_steps=steps, device=dev)
            label = f'DDPM-{steps} fixed_large'
            metric = f'images/sec at DDPM-{steps}, CIFAR-10 UNet 32x32, bs={B}'
        shape = (B, 3, 32, 32)

        def fold():
            return diffuser.sample(model, torch.randn(shape, device=dev, generator=gen),
                                   tqdm_kwargs=dict(disable=True)).clamp(-1, 1)
        model(torch.zeros(shape, device=dev), torch.zeros((B, ), dtype=torch.long, device=dev))  # plan
        return dict(metric=metric, fold=fold, images=B, shape=shape, diffuser=diffuser, sd_cpu=sd_cpu,
                    handles=[(model.native_handle(dev), 'dm_unet', len(diffuser.respaced_seq))],
                    workload=f'{label} sampling fold, CIFAR-10 UNet (dim 128, mults 1-2-2-2, 35.7M params, '
                             f'synthetic weights), 3x32x32, B={B} per GPU', denoise_steps=steps)
    if name == 'c4':
        conf = load_config(os.path.join(cfgdir, 'adm256_combined.yaml'))
        model = instantiate_from_config(conf.model).eval()
        init_synthetic_(model)
        sd_cpu = {k: v.clone() for k, v in model.state_dict().items()}
        model = model.to(dev)
        B = args.batch or 64
        steps = args.respace_steps or 100
        diffuser = DDIMCFG(guidance_scale=3.0, respace_type='uniform', respace_steps=steps, eta=0.0, device=dev)
        shape = (B, 3, 256, 256)
        y = torch.zeros((B, ), dtype=torch.long, device=dev)

        def fold():
            return diffuser.sample(model, torch.randn(shape, device=dev, generator=gen), model_kwargs=dict(y=y),
                                   tqdm_kwargs=dict(disable=True)).clamp(-1, 1)
        t0 = torch.zeros((B, ), dtype=torch.long, device=dev)
        model(torch.zeros(shape, device=dev), t0, y)
        model(torch.zeros(shape, device=dev), t0, None)
        return dict(metric=f'images/sec at ADM-256 UNetCombined DDIMCFG-{steps} (s=3), bs={B}', fold=fold, images=B,
                    shape=shape, diffuser=diffuser, sd_cpu=sd_cpu, shared_workspace=True,
                    cpu=dict(arch=dict(conf.model.params), batch=1, timed_steps=1, guidance_scale=3.0),
                    handles=[(model.unet_cond.native_handle(dev), 'dm_unet', len(diffuser.respaced_seq)),
                             (model.unet_uncond.native_handle(dev), 'dm_unet', len(diffuser.respaced_seq))],
                    workload=f'DDIMCFG-{steps} (s=3, eta=0) sampling fold, guided-diffusion 256x256 UNetCombined '
                             f'(2 x 552.8M params, synthetic weights; cond + uncond forwards per step), 3x256x256, '
                             f'B={B} per GPU', denoise_steps=steps)
    if name == 'c5':
        conf = load_config(os.path.join(cfgdir, 'dit_xl2_256.yaml'))
        model = instantiate_from_config(conf.model).eval()
        init_synthetic_(model.vit)
        sd_cpu = {k: v.clone() for k, v in model.vit.state_dict().items()}
        vp = model.vit
        dit_arch = dict(patch_size=vp.arch['patch_size'], num_heads=vp.arch['num_heads'], depth=vp.arch['depth'],
                        num_classes=vp.arch['num_classes'], out_channels=vp.arch['out_channels'],
                        in_channels=vp.arch['in_channels'], input_size=vp.arch['input_size'])
        model = model.to(dev)
        B = args.batch or 32
        steps = args.respace_steps or 250
        dp = conf.diffusion.params
        diffuser = DDIMCFG(guidance_scale=3.0, respace_type='uniform', respace_steps=steps, eta=0.0,
                           clip_denoised=dp.clip_denoised, device=dev)
        shape = (B, 4, 32, 32)   # latent 4 x img/8 x img/8 (streamlit page 2 :91-95)
        y = torch.zeros((B, ), dtype=torch.long, device=dev)

        def fold():
            return diffuser.sample(model, torch.randn(shape, device=dev, generator=gen), model_kwargs=dict(y=y),
                                   tqdm_kwargs=dict(disable=True))
        import dmhip
        with dmhip.null_label_scope():   # the 2B batched CFG forward's plan
            model(torch.zeros((2 * B, 4, 32, 32), device=dev), torch.zeros((2 * B, ), dtype=torch.long, device=dev),
                  torch.cat([y, torch.full_like(y, -1)]))
        return dict(metric=f'images/sec at DiT-XL/2 DDIMCFG-{steps} (s=3), latent 4x32x32, bs={B}', fold=fold,
                    images=B, shape=shape, diffuser=diffuser, sd_cpu=sd_cpu,
                    cpu=dict(arch=dit_arch, batch=2, timed_steps=3, guidance_scale=3.0, clip=dp.clip_denoised),
                    handles=[(model.vit.native_handle(dev), 'dm_dit', len(diffuser.respaced_seq))],
                    workload=f'DDIMCFG-{steps} (s=3, eta=0, clip_denoised false) sampling fold, DiT-XL/2 (675M '
                             f'params, synthetic weights; cond + null-class rows as one 2B forward), latent 4x32x32, '
                             f'B={B} per GPU', denoise_steps=steps)
    raise ValueError(f'unknown workload {name}')


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """`bench.py --gpus N` without a launcher: start N fresh child processes of this script, one per GPU, with
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set (the process-per-GPU layout of accelerate's launch that the
    reference's harness runs under, scripts/sample_uncond.py:119,131,190), wait for all of them and forward
    rank 0's JSON line. Runs before this process makes any HIP call (torch.cuda.device_count() does not
    initialise the GPU), and never execs: the children are new processes. Returns the exit code."""
    import subprocess
    backend = os.environ.get('DM_DIST_BACKEND', 'nccl')
    if backend == 'nccl' and torch.cuda.device_count() < n:
        print(f'bench.py: --gpus {n} but only {torch.cuda.device_count()} GPU(s) visible', file=sys.stderr)
        return 2
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR='127.0.0.1', MASTER_PORT=port)
        env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')   # RCCL over dmabuf IPC on this pool
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else None, text=True))
    # poll every rank: the first non-zero exit ends the others (a dead rank would leave rank 0 blocked in a
    # collective forever -- ADVICE r4); rank 0's stdout is drained by a thread meanwhile
    import threading
    import time
    out_buf = []
    reader = threading.Thread(target=lambda: out_buf.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    codes = [None] * n
    while any(c is None for c in codes):
        for r, p in enumerate(procs):
            if codes[r] is None:
                codes[r] = p.poll()
        if any(c not in (None, 0) for c in codes):
            for r, p in enumerate(procs):
                if codes[r] is None:
                    p.terminate()
            for r, p in enumerate(procs):
                if codes[r] is None:
                    try:
                        codes[r] = p.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        codes[r] = p.wait()
            break
        time.sleep(0.2)
    reader.join(timeout=30)
    out0 = out_buf[0] if out_buf else ''
    if out0:
        sys.stdout.write(out0)
        sys.stdout.flush()
    bad = [(r, c) for r, c in enumerate(codes) if c != 0]
    if bad:
        print(f'bench.py: rank(s) failed: {bad}', file=sys.stderr)
        return 1
    return 0


def build_stub(args, dev, rank):
    """Harness-only workload (`--workload stub`, CPU, no HIP library): exercises the launch, barrier,
    max-over-ranks timing and gather of the bench without a GPU (tests/test_distributed.py)."""
    gen = torch.Generator(device=dev)
    gen.manual_seed(2022 + rank)
    B = args.batch or 4
    shape = (B, 3, 8, 8)

    def fold():
        return torch.randn(shape, generator=gen, device=dev).clamp(-1, 1)
    return dict(metric='harness stub', fold=fold, images=B, shape=shape, handles=[], sd_cpu=None,
                workload='stub fold (harness test, no model)', denoise_steps=0, diffuser=None)


def main():
    args = parse()
    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus:
        print(f'bench.py: --gpus {args.gpus} but WORLD_SIZE={world}', file=sys.stderr)
        sys.exit(2)
    # DM_DIST_BACKEND=gloo rehearses the N > 1 path with several ranks on one GPU (host-side gather);
    # the measured configuration is nccl (RCCL over xGMI), one rank per GPU.
    backend = os.environ.get('DM_DIST_BACKEND', 'nccl')
    stub = args.workload == 'stub'
    if stub:
        backend = 'gloo'
    gpu = local_rank % max(1, torch.cuda.device_count())
    if world > 1:
        if not stub:
            torch.cuda.set_device(gpu)
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', gpu))
        else:
            dist.init_process_group(backend)
        if dist.get_world_size() != args.gpus:
            print(f'bench.py: --gpus {args.gpus} but the process group has {dist.get_world_size()} ranks',
                  file=sys.stderr)
            sys.exit(2)
    dev = torch.device('cpu') if stub else torch.device('cuda', gpu)
    sync = (lambda: None) if stub else torch.cuda.synchronize

    if stub:
        wl = build_stub(args, dev, rank)
    else:
        import dmhip
        from dmhip._lib import check as _check
        dmhip.load()
        wl = build_workload(args.workload, args, dev, rank)
    B, shape = wl['images'], wl['shape']
    gathered = torch.empty((world * B, *shape[1:]), device=dev) if world > 1 else None
    comm, gather_path, gather_check = None, None, None
    if world > 1:
        gather_path = 'torch.distributed' if backend == 'nccl' else f'{backend} (host)'
        gather_check = f'not run ({backend} host gather)' if backend != 'nccl' else 'not run (DM_GATHER=torch)'
    if world > 1 and backend == 'nccl' and os.environ.get('DM_GATHER') != 'torch':
        from dmhip.comm import Comm   # the C-ABI RCCL all-gather (dm_allgather_f32), bootstrapped over the group
        # every rank gets the communicator or every rank gathers with torch.distributed
        comm = Comm.try_from_process_group()
        if comm is None:
            print(f'bench.py: rank {rank}: dm_comm could not be set up on every rank; gathering with torch.distributed',
                  file=sys.stderr)
            gather_path = 'torch.distributed (dm_comm unavailable on some rank)'
            gather_check = 'not run (dm_comm unavailable on some rank)'
        else:
            # before the timed region: the C-ABI gather of a rank-tagged fold against all_gather_into_tensor, agreed
            # over the ranks; on any difference every rank drops to torch.distributed
            n_el = 1
            for d_ in shape[1:]:
                n_el *= int(d_)
            probe = torch.arange(B * n_el, dtype=torch.float32, device=dev).view(B, *shape[1:]) + rank
            got, ref = torch.empty_like(gathered), torch.empty_like(gathered)
            comm.allgather(probe, got)
            dist.all_gather_into_tensor(ref, probe)
            same = torch.tensor([1 if torch.equal(got, ref) else 0], dtype=torch.int32, device=dev)
            dist.all_reduce(same, op=dist.ReduceOp.MIN)
            gather_check = 'equal on every rank' if int(same.item()) else 'differed on some rank'
            if int(same.item()):
                gather_path = 'dm_allgather_f32 (RCCL, C ABI; equal to all_gather_into_tensor at start)'
            else:
                comm.close()
                comm = None
                gather_path = 'torch.distributed (dm_allgather_f32 differed from all_gather_into_tensor)'

    def fold():
        x = wl['fold']()
        if world > 1:   # the reference's accelerator.gather of the fold (sample_uncond.py:190): one all-gather
            if comm is not None:
                comm.allgather(x, gathered)
            elif backend == 'nccl':
                dist.all_gather_into_tensor(gathered, x)
            else:
                parts = [torch.empty(tuple(x.shape)) for _ in range(world)]
                dist.all_gather(parts, x.cpu())
                gathered.copy_(torch.cat(parts))
            return gathered
        return x

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        fold()
    # HIP events around every launch of every PROFILE_EVERY-th forward of the timed region
    for h, abi, _ in wl['handles']:
        dmhip.unet_profile_enable(h, 0 if args.no_profile else PROFILE_EVERY, abi=abi)
    barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        fold()
    sync()
    barrier()
    elapsed = time.perf_counter() - t0
    ranks = None
    if world > 1:
        # what each rank saw, for a record that verifies itself: its device, its own fold time,
        # the RCCL communicator's own view (ncclCommCount / ncclCommUserRank / device through dm_comm_info)
        mine = dict(rank=rank, device=str(dev), fold_ms=round(elapsed / args.steps * 1e3, 3))
        if not stub:
            props = torch.cuda.get_device_properties(gpu)
            mine.update(gpu_name=props.name, pci_bus_id=getattr(props, 'pci_bus_id', None),
                        pci_device_id=getattr(props, 'pci_device_id', None))
        if comm is not None:
            n_, r_, d_ = comm.info()
            mine.update(comm_nranks=n_, comm_rank=r_, comm_device=d_)
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
        tt = torch.tensor([elapsed], device=dev if backend == 'nccl' else 'cpu', dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = tt.item()
        comm_n = sorted({r.get('comm_nranks') for r in per_rank}, key=str)
        ranks = dict(process_group_size=dist.get_world_size(), backend=backend,
                     comm_nranks=comm_n[0] if len(comm_n) == 1 else comm_n,
                     distinct_devices=len({(r.get('pci_bus_id'), r.get('pci_device_id'), r['device'])
                                           for r in per_rank}),
                     gather_check=gather_check, per_rank=per_rank)
    prof, kernel_s, wbytes_t, wsbytes_t = [], 0.0, 0, 0
    # launches per network forward of each kernel label: each handle's ops with the label, weighted by its forwards
    lpf, nfwd = {}, sum(f for _, _, f in wl['handles'])
    for h, abi, fwd_per_fold in wl['handles']:
        p = dmhip.unet_profile_read(h, abi=abi)
        prof += p
        for op in p:
            lpf[op['label']] = lpf.get(op['label'], 0.0) + fwd_per_fold / max(1, nfwd)
        observed = max((op['launches'] for op in p), default=0)   # forwards of this handle that ran with events
        if observed:
            kernel_s += sum(op['ms_total'] for op in p) * 1e-3 * fwd_per_fold * args.steps / observed
        wbytes, wsbytes = ctypes.c_int64(), ctypes.c_int64()
        _check(getattr(dmhip.load(), abi + '_memory')(h, ctypes.byref(wbytes), ctypes.byref(wsbytes)), abi + '_memory')
        wbytes_t += wbytes.value
        # UNetCombined's two networks run over one shared scratch slab (dm_unet_share_workspace): count it once
        wsbytes_t = max(wsbytes_t, wsbytes.value) if wl.get('shared_workspace') else wsbytes_t + wsbytes.value
        dmhip.unet_profile_enable(h, False, abi=abi)

    roof, total_gpu_ms, total_flops, fam = None, 0.0, 0.0, {}
    if not args.no_profile and prof:
        roof, total_gpu_ms, total_flops, fam = roofline(prof, args.workload, None if stub else dmhip.build_info(), lpf)

    if rank == 0:
        images = world * B * args.steps
        if stub:
            math = 'fp32'
        else:
            h0, abi0, _ = wl['handles'][0]
            math = dmhip.unet_conv_math(h0) if abi0 == 'dm_unet' else dmhip.dit_math(h0)
        line = dict(
            metric=wl['metric'],
            value=round(images / elapsed, 4),
            unit='images/sec',
            n_gpus=world,
            steps=args.steps,
            warmup=args.warmup,
            ms_per_step=round(elapsed / args.steps * 1e3, 2),
            higher_is_better=True,
            scaling='weak',
            vs_baseline=None,
            dtype=f'f32 via {math} split MFMA' if math != 'fp32' else 'f32',
            data='synthetic',
            config=dict(workload=wl['workload'], global_batch=world * B, parallelism=f'dp{world}',
                        denoise_steps=wl['denoise_steps'], weights_gb=round(wbytes_t / 1e9, 3),
                        workspace_gb=round(wsbytes_t / 1e9, 3), conv_math=math,
                        # the reference draws randn_like every step even at eta=0 (ddim.py:76): so does the bench
                        skip_unused_noise=wl['diffuser'].skip_unused_noise if wl['diffuser'] else None,
                        gather=gather_path),
            roofline=roof,
            ranks=ranks,
            step_level=dict(model_tflops=round(total_flops / (total_gpu_ms * 1e-3) / 1e12, 2) if total_gpu_ms else None,
                            # observed forwards are 1 in PROFILE_EVERY: their event-summed launch time scaled to
                            # all forwards, over the wall time. The events bracket every launch of an observed
                            # forward, which makes that forward a few % slower than the unobserved ones: the ratio
                            # can exceed 1 and is no kernel-busy fraction
                            sampled_forward_time_over_wall=round(kernel_s / elapsed, 4) if kernel_s else None),
        )
        if args.workload != 'c3':
            line['config']['bench_workload'] = args.workload
        line['cpu_baseline'] = None
        if world == 1 and not args.no_cpu_baseline and wl['sd_cpu'] is not None:
            if args.workload in ('c2', 'c3'):
                line['cpu_baseline'] = cpu_baseline(wl['sd_cpu'], args.cpu_batch, wl['denoise_steps'])
            else:
                c = wl['cpu']
                line['cpu_baseline'] = cpu_baseline_cfg(args.workload, wl['sd_cpu'], c['arch'], c['batch'],
                                                        wl['denoise_steps'], c['guidance_scale'], c['timed_steps'],
                                                        clip=c.get('clip', True))
            line['gpu_over_cpu'] = round(line['value'] / line['cpu_baseline']['value'], 1)
        if args.profile_json:
            with open(args.profile_json, 'w') as f:
                json.dump(dict(families=fam, ops=prof), f, indent=1)
        print(json.dumps(line), flush=True)
    if comm is not None:
        comm.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
