"""Drop-in shim: `from utils.helpers import ...`."""
from diffusion_models_collection_amd.utils.helpers import *  # noqa: F401,F403
from diffusion_models_collection_amd.utils.helpers import (set_seed, resolve_image_size, count_parameters,  # noqa
                                                           get_device, save_config, load_config,
                                                           normalize_to_neg_one_to_one, unnormalize_to_zero_to_one,
                                                           setup_distributed, create_gif)
