"""datasets package (reference: datasets/__init__.py): the DiffusionDataset / CustomImageDataset API over a uint8
image bank, plus the device-resident loader that replaces the reference's DataLoader on the training path."""
from .base_dataset import CustomImageDataset, DiffusionDataset, ImageTransform, from_arrays

__all__ = ["DiffusionDataset", "CustomImageDataset", "ImageTransform", "from_arrays", "DeviceLoader",
           "get_dataloader", "get_dataset"]


def __getattr__(name):   # the loader binds libdmc.so: imported on first use
    if name in ("DeviceLoader", "get_dataloader", "get_dataset", "load_batch"):
        from . import loader
        return getattr(loader, name)
    raise AttributeError(name)
