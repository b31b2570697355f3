"""Drop-in shim: the reference's `from models import UNet, DiT, DiM` resolves to the MI355X build."""
from diffusion_models_collection_amd.models import UNet, DiT, DiM  # noqa: F401

__all__ = ['UNet', 'DiT', 'DiM']
