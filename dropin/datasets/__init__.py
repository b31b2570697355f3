"""Drop-in shim for the reference's datasets package."""
from diffusion_models_collection_amd.datasets import *  # noqa: F401,F403
from diffusion_models_collection_amd.datasets import __getattr__  # noqa: F401
