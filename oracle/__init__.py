"""CPU oracle for the denoising hot path — TEST INFRASTRUCTURE ONLY.

A torch-CPU restatement of the reference algorithm (xyfJASON/diffusion-models-pytorch
@ 2024-12-20) for the path in SURVEY.md §8:
  * oracle.diffusion : schedule, DDPM / DDIM denoise + sample loops, CFG
  * oracle.unet      : the DDPM UNet forward (functional, from a state_dict)

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, and only as the checker / the CPU baseline — never as the thing
measured or shipped. The product path (diffusions.*, models.*, dmhip) never
imports it and fails loudly without the HIP library.

Pinning: tests/golden/*.npz hold outputs of the reference itself, generated in
the survey container by tests/golden/make_golden.py (which imports
/root/reference); tests/test_oracle_golden.py checks this restatement against
them (bit-exact for schedule/index/update arithmetic, fp32-tolerance for the
network forward, whose oneDNN summation order depends on the thread count).
"""
