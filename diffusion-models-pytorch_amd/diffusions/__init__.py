"""MI355X-native diffusion samplers, API-compatible with the reference `diffusions` package.

Covered (hot path): schedule, DDPM(+CFG), DDIM(+CFG, inversion), and from §8(f) the
Euler and Heun samplers (diffusions/euler.py, heun.py).
Not provided: DDPM-IP, guidance (out of this round's scope).
"""
from diffusions import schedule, ddpm, ddim, euler, heun  # noqa: F401
from diffusions.schedule import get_beta_schedule, get_respaced_seq  # noqa: F401
from diffusions.ddpm import DDPM, DDPMCFG  # noqa: F401
from diffusions.ddim import DDIM, DDIMCFG  # noqa: F401
from diffusions.euler import EulerSampler  # noqa: F401
from diffusions.heun import HeunSampler  # noqa: F401
