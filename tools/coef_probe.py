"""Print torch-CPU 0-dim coefficient bits for the DDPM/DDIM schedules (cross-host check)."""
import hashlib, sys, torch
print('cpu capability', torch.backends.cpu.get_cpu_capability(), torch.__version__)
betas = torch.linspace(0.0001, 0.02, 1000, dtype=torch.float64)
ac = torch.cumprod(1. - betas, dim=0).to(torch.float)
vals = []
for t in range(1000):
    a = ac[t]
    p = ac[t - 1] if t > 0 else torch.tensor(1.0)
    vals += [((1. / a) ** 0.5).item(), ((1. / a - 1.) ** 0.5).item(), (a ** 0.5).item(), ((1. - a) ** 0.5).item(),
             torch.sqrt(p).item(), torch.sqrt(1. - p - 0.0 * a).item(), ((p ** 0.5) * (1 - a / p) / (1. - a)).item()]
h = hashlib.sha256(torch.tensor(vals).numpy().tobytes()).hexdigest()
print('coef sha', h)
x = torch.rand(100000, generator=torch.Generator().manual_seed(0)) + 0.5
print('vec sqrt sha', hashlib.sha256(torch.sqrt(x).numpy().tobytes()).hexdigest())
print('vec pow sha', hashlib.sha256((x ** 0.5).numpy().tobytes()).hexdigest())
s = [torch.sqrt(x[i]).item() for i in range(2000)]
print('0dim sqrt sha', hashlib.sha256(torch.tensor(s).numpy().tobytes()).hexdigest())
