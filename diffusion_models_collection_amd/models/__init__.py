"""Backbone registry (models/__init__.py of the reference): `from models import UNet, DiT, DiM`.

UNet is the MI355X hot path. DiT / DiM are outside this round's scope; they are
importable so the reference's train.py / sample.py import line works, and raise on construction.
"""
from .unet import UNet


class _NotInScope:
    def __init__(self, *args, **kwargs):
        raise NotImplementedError(f"{type(self).__name__} is not implemented on the MI355X path yet "
                                  "(SURVEY.md §8f next rows); use model_type='unet'")


class DiT(_NotInScope):
    pass


class DiM(_NotInScope):
    pass


__all__ = ['UNet', 'DiT', 'DiM']
