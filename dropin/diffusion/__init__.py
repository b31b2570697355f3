"""Drop-in shim: `from diffusion import DDPM, DDIM` resolves to the MI355X build."""
from diffusion_models_collection_amd.diffusion import DDPM, DDIM  # noqa: F401

__all__ = ['DDPM', 'DDIM']
