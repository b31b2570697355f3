"""Drop-in shim: `from utils.trainer import DiffusionTrainer`."""
from diffusion_models_collection_amd.utils.trainer import DiffusionTrainer  # noqa: F401
