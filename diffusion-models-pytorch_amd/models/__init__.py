"""Denoisers with the reference's module paths (models.unet.UNet, ...)."""
