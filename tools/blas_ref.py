"""Library ceiling for the fp16x2 token GEMMs: torch (hipBLASLt) fp16 GEMMs with the contraction tripled
(C = [a1 | a0 | a0] [w0 | w1 | w0]^T, fp32 accumulate) at the shapes linear_k32 runs, timed with HIP
events. Only a measuring stick for the hand-written kernel (nothing in the engine calls it).
    python tools/blas_ref.py"""
import torch

SHAPES = {  # name: (M, N, K) of the fp32 GEMM
    'dit_qkv': (16384, 3456, 1152), 'dit_proj': (16384, 1152, 1152), 'dit_fc1': (16384, 4608, 1152),
    'dit_fc2': (16384, 1152, 4608), 'unet_qkv': (65536, 768, 256), 'adm_qkv32': (65536, 1536, 512),
}


def main():
    dev = torch.device('cuda:0')
    for name, (M, N, K) in SHAPES.items():
        a = torch.randn((M, 3 * K), device=dev, dtype=torch.float16)
        w = torch.randn((N, 3 * K), device=dev, dtype=torch.float16)
        for _ in range(3):
            c = torch.matmul(a, w.t())
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 20
        e0.record()
        for _ in range(n):
            c = torch.matmul(a, w.t())
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / n
        tf16 = 2 * M * N * 3 * K / (ms * 1e-3) / 1e12
        print(f'{name:10s} M {M:6d} N {N:5d} K {K:5d}: {ms * 1e3:8.1f} us  fp16 {tf16:7.1f} TF  '
              f'fp32-equivalent {tf16 / 3:6.1f} TF ({tf16 / 3 / 833.3:.3f} of 833)', flush=True)
        del a, w, c


if __name__ == '__main__':
    main()
