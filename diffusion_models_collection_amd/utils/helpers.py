"""Helpers with the reference API (utils/helpers.py of sunyzhi55/Diffusion_Models_Collection).

set_seed (:12-19), resolve_image_size (:22-34), count_parameters, get_device, save_config, load_config
(:57-70), normalize helpers, setup_distributed (:83-90) and create_gif (:93-133). setup_distributed keeps
the reference's `backend='nccl'` default, which on ROCm is RCCL over xGMI.
"""
import os
import random
from pathlib import Path

import numpy as np
import torch


def set_seed(seed=42):
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    torch.cuda.manual_seed_all(seed)
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False


def resolve_image_size(image_size):
    if isinstance(image_size, int):
        return (image_size, image_size)
    if isinstance(image_size, (list, tuple)) and len(image_size) == 2:
        h, w = image_size
        if not (isinstance(h, int) and isinstance(w, int)):
            raise ValueError("image_size values must be integers")
        return (h, w)
    raise ValueError("image_size must be int or a pair (H, W)")


def count_parameters(model):
    return sum(p.numel() for p in model.parameters() if p.requires_grad)


def get_device(device_id=None):
    if device_id is not None:
        return torch.device(f'cuda:{device_id}')
    return torch.device('cuda' if torch.cuda.is_available() else 'cpu')


def save_config(config, save_path):
    import json
    with Path(save_path).open('w', encoding='utf-8') as f:
        json.dump(config, f, indent=4)


def load_config(config_path):
    import importlib.util
    import sys
    path = Path(config_path)
    spec = importlib.util.spec_from_file_location("config", path)
    config_module = importlib.util.module_from_spec(spec)
    sys.modules["config"] = config_module
    spec.loader.exec_module(config_module)
    return config_module.config


def normalize_to_neg_one_to_one(img):
    return img * 2 - 1


def unnormalize_to_zero_to_one(img):
    return (img + 1) * 0.5


def setup_distributed(rank, world_size, backend='nccl', port='12355'):
    """Process-group init; 'nccl' is RCCL on ROCm. MASTER_ADDR defaults to 127.0.0.1."""
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', str(port))
    torch.distributed.init_process_group(backend, rank=rank, world_size=world_size)


def create_gif(images_list, save_path, fps=20):
    from PIL import Image
    frames = []
    for img in images_list:
        if isinstance(img, torch.Tensor):
            img = img.cpu().numpy()
        if img.ndim == 3 and (img.shape[0] == 1 or img.shape[0] == 3):
            img = np.transpose(img, (1, 2, 0))
        if img.max() <= 1.0:
            img = (img * 255).astype(np.uint8)
        else:
            img = img.astype(np.uint8)
        if img.ndim == 3 and img.shape[2] == 1:
            img = img.squeeze(2)
        frames.append(Image.fromarray(img))
    frames[0].save(save_path, save_all=True, append_images=frames[1:], duration=1000 / fps, loop=0)
