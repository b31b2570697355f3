"""Utils package (utils/__init__.py of the reference). The trainer is imported lazily."""
from .helpers import (set_seed, count_parameters, get_device, save_config, load_config,
                      normalize_to_neg_one_to_one, unnormalize_to_zero_to_one, setup_distributed,
                      resolve_image_size, create_gif)


def __getattr__(name):
    if name == "DiffusionTrainer":
        from .trainer import DiffusionTrainer
        return DiffusionTrainer
    raise AttributeError(name)


__all__ = ['DiffusionTrainer', 'set_seed', 'count_parameters', 'get_device', 'save_config', 'load_config',
           'normalize_to_neg_one_to_one', 'unnormalize_to_zero_to_one', 'setup_distributed']
