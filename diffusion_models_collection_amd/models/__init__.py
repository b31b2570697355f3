"""Backbone registry (models/__init__.py of the reference): `from models import UNet, DiT, DiM`.

UNet (the hot path) and DiT run on the gfx950 kernels. DiM is outside this round's scope
(§8f); it is importable so the reference's train.py / sample.py import line works, and raises on construction.
"""
from .dit import DiT
from .unet import UNet


class _NotInScope:
    def __init__(self, *args, **kwargs):
        raise NotImplementedError(f"{type(self).__name__} is not implemented on the MI355X path yet "
                                  "(SURVEY.md §8f next rows); use model_type='unet' or 'dit'")


class DiM(_NotInScope):
    pass


__all__ = ['UNet', 'DiT', 'DiM']
