"""models/dit/autoencoder.py stand-in: the reference wraps diffusers' AutoencoderKL loaded with
``from_pretrained('stabilityai/sd-vae-ft-ema')`` — a network fetch of third-party weights used only
to decode latents after sampling. It is not part of this engine."""


class AutoEncoderKL:
    def __init__(self, *args, **kwargs):
        raise NotImplementedError('AutoEncoderKL needs diffusers and a downloaded VAE checkpoint; latent decoding '
                                  'is outside the MI355X sampling engine')
