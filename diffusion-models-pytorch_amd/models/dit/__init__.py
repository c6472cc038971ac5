"""DiT denoiser with the reference's module paths (models.dit.model.DiT, models.dit.dit.DiT)."""
