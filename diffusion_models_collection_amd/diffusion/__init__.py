"""Diffusion schedulers (diffusion/__init__.py of the reference)."""
from .ddpm import DDPM
from .ddim import DDIM

__all__ = ['DDPM', 'DDIM']
