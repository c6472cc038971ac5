"""ADM (guided-diffusion) denoisers with the reference's module paths (models.adm.unet, models.adm.unet_combined)."""
