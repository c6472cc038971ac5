"""Microbenchmark of the GEMM kernel on the attention shapes of the CIFAR-10 UNet (B=256, 16x16, C=256).

    python tools/gemm_bench.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'diffusion-models-pytorch_amd')]

import torch  # noqa: E402

import dmhip  # noqa: E402


def bench(name, M, N, K, Z1=1, Z2=1, b_kn=0, res=False, iters=20, split=False, pro=False, ea=6, eb=6, qkv=False):
    dev = torch.device('cuda', 0)
    A = torch.randn((Z1 * Z2, M, K), device=dev)
    B = torch.randn((Z1 * Z2, K, N) if b_kn else (Z1 * Z2, N, K), device=dev)
    C = torch.empty((Z1 * Z2, M, N), device=dev)
    R = torch.randn((M, N), device=dev) if res else None
    d = dmhip.GemmDesc()
    d.M, d.N, d.K, d.Z1, d.Z2 = M, N, K, Z1, Z2
    d.A, d.a_s1, d.a_s2, d.lda = A.data_ptr(), Z2 * M * K, M * K, K
    d.B, d.b_s1, d.b_s2, d.ldb, d.b_kn = B.data_ptr(), Z2 * K * N, K * N, (N if b_kn else K), b_kn
    if qkv:  # the UNet's layout: q / k (/ v) are column blocks of one [Z][L][3C] qkv buffer (C = K = N here)
        Q = torch.randn((Z1 * Z2, M, 3 * K), device=dev)
        if not b_kn:  # S = q k^T; PV keeps its contiguous A (the softmax rows) and reads v from qkv
            d.A, d.a_s1, d.a_s2, d.lda = Q.data_ptr(), M * 3 * K, 0, 3 * K
        d.B, d.b_s1, d.b_s2, d.ldb = Q.data_ptr() + (4 * 2 * K if b_kn else 4 * K), M * 3 * K, 0, 3 * K
    d.C, d.c_s1, d.c_s2, d.ldc = C.data_ptr(), Z2 * M * N, M * N, N
    d.alpha = 1.0
    if res:
        d.res, d.ld_res = R.data_ptr(), N
    if pro:  # GroupNorm affine prologue on A (the QKV projection), 256 rows per image
        sc, sh = torch.rand((M // 256, K), device=dev) + 0.5, torch.rand((M // 256, K), device=dev) - 0.5
        d.pro_scale, d.pro_shift, d.pro_rows = sc.data_ptr(), sh.data_ptr(), 256
    if split:
        d.split, d.split_ea, d.split_eb = 2, ea, eb
    for _ in range(3):
        dmhip.gemm(d, dev)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        dmhip.gemm(d, dev)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    tf = 2.0 * Z1 * Z2 * M * N * K / ms / 1e9
    print(f'{name:16s} {"fp16x2" if split else "fp32":7s} {ms:8.4f} ms {tf:6.1f} TF/s', flush=True)


if __name__ == '__main__':
    dmhip.load()
    for sp in (False, True):
        bench('qkv_gn_k256', 65536, 768, 256, pro=True, split=sp)
        bench('qkv_k256', 65536, 768, 256, split=sp)
        bench('proj_res', 65536, 256, 256, res=True, split=sp)
        bench('S', 256, 256, 256, Z1=256, split=sp)
        bench('PV_kn', 256, 256, 256, Z1=256, b_kn=1, split=sp, ea=14)
        bench('S_qkv', 256, 256, 256, Z1=256, split=sp, qkv=True)
        bench('PV_kn_qkv', 256, 256, 256, Z1=256, b_kn=1, split=sp, ea=14, qkv=True)
        bench('big_4096', 4096, 4096, 4096, iters=5, split=sp)
