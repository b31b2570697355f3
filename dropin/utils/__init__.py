"""Drop-in shim for the reference's utils package (trainer imported lazily)."""
from diffusion_models_collection_amd.utils import *  # noqa: F401,F403
from diffusion_models_collection_amd.utils import __getattr__  # noqa: F401
