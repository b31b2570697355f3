"""MI355X-native (gfx950) diffusion training + sampling hot path of sunyzhi55/Diffusion_Models_Collection.

Public API mirrors the reference:
    from diffusion_models_collection_amd.models import UNet
    from diffusion_models_collection_amd.diffusion import DDPM, DDIM
    from diffusion_models_collection_amd.utils.trainer import DiffusionTrainer
The `dropin/` directory at the repo root exposes the same modules under the reference's top-level names
(models, diffusion, utils) so the reference's train.py / sample.py run unchanged.
"""
__version__ = "0.1.0"
