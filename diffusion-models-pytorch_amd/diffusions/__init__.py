"""MI355X-native diffusion samplers, API-compatible with the reference `diffusions` package.

Covered (hot path): schedule, DDPM(+CFG), DDIM(+CFG, inversion).
Not provided: Euler/Heun samplers, DDPM-IP, guidance (out of this round's scope).
"""
from diffusions import schedule, ddpm, ddim  # noqa: F401
from diffusions.schedule import get_beta_schedule, get_respaced_seq  # noqa: F401
from diffusions.ddpm import DDPM, DDPMCFG  # noqa: F401
from diffusions.ddim import DDIM, DDIMCFG  # noqa: F401
