"""Datasets of the reference's training path, decoded ONCE into a uint8 image bank.

Reference: datasets/base_dataset.py:11-156 (DiffusionDataset over torchvision's CIFAR10/CIFAR100/MNIST/FashionMNIST/
CelebA, get_default_transform :100-133), datasets/custom_dataset.py:13-170 (CustomImageDataset). The reference decodes
and transforms every image on every epoch in DataLoader worker processes; here the deterministic part of its
transform (Resize + CenterCrop, with torchvision's size and crop arithmetic on the same PIL calls) is applied once
on the host, and the bank [N, H, W, C] uint8 goes to device memory (datasets/loader.py) where one kernel per batch
does the per-epoch part (RandomHorizontalFlip, ToTensor, Normalize).

torchvision is not needed: the on-disk layouts torchvision downloads are read directly --
  cifar10 / cifar100: `cifar-10-batches-bin` / `cifar-100-binary` (record = label byte(s) + 3072 CHW bytes), or the
      python layout `cifar-10-batches-py` / `cifar-100-python` through a restricted unpickler that can rebuild only
      numpy arrays, lists, dicts and bytes (nothing else in the file can run);
  mnist / fashionmnist: `MNIST/raw` / `FashionMNIST/raw` idx files (optionally .gz);
  celeba: `celeba/img_align_celeba/*.jpg` + `celeba/list_eval_partition.txt`.
There is no network: download=True only checks that the files are present.
"""
import gzip
import json
import pickle
import struct
from pathlib import Path
from typing import Optional

import numpy as np
import torch


class ImageTransform:
    """The reference's default transform (datasets/base_dataset.py:100-133, custom_dataset.py:150-170) as data:
    Resize(size) -> CenterCrop(size) [RGB only] -> RandomHorizontalFlip(flip_p) [train, RGB] -> ToTensor ->
    Normalize(mean, std). `prepare` applies the deterministic part to one PIL image or HWC uint8 array; the random
    flip and the normalisation run on the device (dmc_load_batch). Calling it on a PIL image / uint8 array gives
    the CPU tensor the reference's transform returns (used by Dataset.__getitem__)."""

    def __init__(self, size, crop: bool, flip_p: float, mean, std):
        self.size = size           # int (shorter side) or (h, w), torchvision Resize semantics
        self.crop = crop
        self.flip_p = float(flip_p)
        self.mean = [float(m) for m in mean]
        self.std = [float(s) for s in std]

    def out_hw(self):
        if isinstance(self.size, int):
            return (self.size, self.size) if self.crop else None
        return tuple(self.size)

    def prepare(self, img) -> np.ndarray:
        """Resize + CenterCrop -> HWC uint8 (torchvision.transforms.functional resize/center_crop arithmetic)."""
        from PIL import Image
        if isinstance(img, np.ndarray):
            img = Image.fromarray(img if img.ndim == 3 and img.shape[2] > 1 else img.reshape(img.shape[:2]))
        w, h = img.size
        if isinstance(self.size, int):
            short, long_ = (w, h) if w <= h else (h, w)
            new_short, new_long = self.size, int(self.size * long_ / short)
            ow, oh = (new_short, new_long) if w <= h else (new_long, new_short)
        else:
            oh, ow = self.size
        if (oh, ow) != (h, w):
            img = img.resize((ow, oh), Image.BILINEAR)
        if self.crop:
            th, tw = (self.size, self.size) if isinstance(self.size, int) else tuple(self.size)
            if (th, tw) != (oh, ow):
                if th > oh or tw > ow:
                    raise ValueError(f"CenterCrop {th}x{tw} larger than the resized image {oh}x{ow}")
                top, left = int(round((oh - th) / 2.0)), int(round((ow - tw) / 2.0))
                img = img.crop((left, top, left + tw, top + th))
        a = np.asarray(img, dtype=np.uint8)
        return a[:, :, None] if a.ndim == 2 else a

    def __call__(self, img):
        a = self.prepare(img)
        if self.flip_p > 0 and torch.rand(1).item() < self.flip_p:     # RandomHorizontalFlip (host path)
            a = a[:, ::-1]
        t = torch.from_numpy(np.array(a)).permute(2, 0, 1).float().div(255)
        return t.sub_(torch.tensor(self.mean)[:, None, None]).div_(torch.tensor(self.std)[:, None, None])


class _SafeUnpickler(pickle.Unpickler):
    """Rebuilds numpy arrays and builtin containers only (the CIFAR python batches hold nothing else)."""
    _ALLOWED = {("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
                ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "scalar"),
                ("numpy._core.multiarray", "scalar"), ("_codecs", "encode")}

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refusing to load {module}.{name} from a dataset file")


def _load_batch_py(path: Path):
    with open(path, "rb") as f:
        d = _SafeUnpickler(f, encoding="bytes").load()
    d = {(k.decode() if isinstance(k, bytes) else k): v for k, v in d.items()}
    data = np.asarray(d["data"], dtype=np.uint8).reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1)
    labels = d.get("labels", d.get("fine_labels"))
    return data, np.asarray(labels, dtype=np.int64)


def _load_cifar_bin(path: Path, label_bytes: int):
    raw = np.fromfile(path, dtype=np.uint8)
    rec = label_bytes + 3072
    if raw.size % rec:
        raise ValueError(f"{path}: size {raw.size} is not a multiple of the {rec}-byte CIFAR record")
    raw = raw.reshape(-1, rec)
    labels = raw[:, label_bytes - 1].astype(np.int64)     # cifar-100: (coarse, fine) -> fine
    data = raw[:, label_bytes:].reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1)
    return np.ascontiguousarray(data), labels


def _read_idx(path: Path):
    op = gzip.open if path.suffix == ".gz" else open
    with op(path, "rb") as f:
        buf = f.read()
    zero, dtype, ndim = struct.unpack(">HBB", buf[:4])
    if zero != 0 or dtype != 0x08:
        raise ValueError(f"{path}: not an unsigned-byte idx file")
    dims = struct.unpack(">" + "I" * ndim, buf[4:4 + 4 * ndim])
    return np.frombuffer(buf, dtype=np.uint8, offset=4 + 4 * ndim).reshape(dims)


def _find(root: Path, *names):
    for n in names:
        for cand in (root / n, root / (n + ".gz")):
            if cand.exists():
                return cand
    return None


def _read_raw(name: str, root: Path, train: bool):
    """-> (images [N,h,w,c] uint8 at the stored size, labels int64 [N] or None, list of paths or None)"""
    if name in ("cifar10", "cifar100"):
        c10 = name == "cifar10"
        bdir = root / ("cifar-10-batches-bin" if c10 else "cifar-100-binary")
        pdir = root / ("cifar-10-batches-py" if c10 else "cifar-100-python")
        if bdir.is_dir():
            files = ([bdir / f"data_batch_{i}.bin" for i in range(1, 6)] if train else [bdir / "test_batch.bin"]) \
                if c10 else [bdir / ("train.bin" if train else "test.bin")]
            parts = [_load_cifar_bin(f, 1 if c10 else 2) for f in files]
        elif pdir.is_dir():
            files = ([pdir / f"data_batch_{i}" for i in range(1, 6)] if train else [pdir / "test_batch"]) \
                if c10 else [pdir / ("train" if train else "test")]
            parts = [_load_batch_py(f) for f in files]
        else:
            raise FileNotFoundError(f"{name}: neither {bdir} nor {pdir} exists (no network: place the dataset there)")
        return np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts]), None
    if name in ("mnist", "fashionmnist"):
        raw = root / ("MNIST" if name == "mnist" else "FashionMNIST") / "raw"
        pre = "train" if train else "t10k"
        fi, fl = _find(raw, f"{pre}-images-idx3-ubyte"), _find(raw, f"{pre}-labels-idx1-ubyte")
        if fi is None or fl is None:
            raise FileNotFoundError(f"{name}: idx files missing under {raw} (no network: place the dataset there)")
        return _read_idx(fi)[:, :, :, None], _read_idx(fl).astype(np.int64), None
    if name == "celeba":
        base = root / "celeba"
        part = base / "list_eval_partition.txt"
        if not part.exists():
            raise FileNotFoundError(f"celeba: {part} missing (no network: place the dataset there)")
        want = "0" if train else "2"    # torchvision split 'train' = 0, 'test' = 2
        names = [ln.split()[0] for ln in part.read_text().splitlines() if ln.strip() and ln.split()[1] == want]
        return None, None, [base / "img_align_celeba" / n for n in names]
    raise ValueError(name)


def _decode_all(paths, transform: ImageTransform, mode: str):
    from concurrent.futures import ThreadPoolExecutor
    from PIL import Image

    def one(p):
        with Image.open(p) as im:
            return transform.prepare(im.convert(mode))
    with ThreadPoolExecutor(max_workers=8) as ex:
        arrs = list(ex.map(one, paths))
    if not arrs:
        raise ValueError("no images found")
    shapes = {a.shape for a in arrs}
    if len(shapes) != 1:
        raise ValueError(f"images of different sizes after the transform: {sorted(shapes)[:4]}")
    return np.stack(arrs)


class _BankDataset:
    """Common part: `images` uint8 [N, H, W, C] (transform's deterministic part applied), `labels` int64 [N]."""

    images: np.ndarray
    labels: Optional[np.ndarray]
    transform: Optional[ImageTransform]
    conditional: bool

    def __len__(self):
        return int(self.images.shape[0])

    def __getitem__(self, idx):
        a = self.images[idx]
        if self.transform is not None:
            img = self.transform(a)
        else:
            img = torch.from_numpy(np.ascontiguousarray(a)).permute(2, 0, 1).float().div(255)
        if self.conditional:
            return img, int(self.labels[idx]) if self.labels is not None else 0
        return img


class DiffusionDataset(_BankDataset):
    """datasets/base_dataset.py:11-95 with the same constructor and item semantics (img, or (img, label) when
    conditional; CelebA's dummy label 0)."""

    SUPPORTED_DATASETS = ("cifar10", "cifar100", "mnist", "fashionmnist", "celeba")

    def __init__(self, dataset_name: str, root: str = "./data", train: bool = True,
                 transform: Optional[ImageTransform] = None, download: bool = True, conditional: bool = False):
        dataset_name = dataset_name.lower()
        if dataset_name not in self.SUPPORTED_DATASETS:
            raise ValueError(f"Dataset {dataset_name} not supported. "
                             f"Supported datasets: {list(self.SUPPORTED_DATASETS)}")
        if transform is not None and not isinstance(transform, ImageTransform):
            raise TypeError("transform must be an ImageTransform (DiffusionDataset.get_default_transform)")
        self.dataset_name, self.conditional, self.transform = dataset_name, conditional, transform
        images, labels, paths = _read_raw(dataset_name, Path(root), train)
        if paths is not None:
            tr = transform or ImageTransform(64, True, 0.0, [0.5] * 3, [0.5] * 3)
            images, labels = _decode_all(paths, tr, "RGB"), np.zeros(len(paths), dtype=np.int64)
        elif transform is not None and transform.out_hw() != images.shape[1:3]:
            images = np.stack([transform.prepare(a) for a in images])
        self.images, self.labels = np.ascontiguousarray(images), labels

    @staticmethod
    def get_default_transform(image_size=32, dataset_name="cifar10", train=True):
        """datasets/base_dataset.py:100-133."""
        if dataset_name.lower() in ("mnist", "fashionmnist"):
            return ImageTransform(image_size, False, 0.0, [0.5], [0.5])
        return ImageTransform(image_size, True, 0.5 if train else 0.0, [0.5] * 3, [0.5] * 3)

    @staticmethod
    def get_num_classes(dataset_name):
        return {"cifar10": 10, "cifar100": 100, "mnist": 10, "fashionmnist": 10, "celeba": 0}.get(
            dataset_name.lower(), 0)

    @staticmethod
    def get_image_channels(dataset_name):
        return 1 if dataset_name.lower() in ("mnist", "fashionmnist") else 3


class CustomImageDataset(_BankDataset):
    """datasets/custom_dataset.py:13-147: images from a directory; labels from class subdirectories (use_subdirs)
    or a JSON {filename: label} file, remapped to consecutive indices. Images are decoded once (RGB) through the
    transform's Resize + CenterCrop."""

    SUPPORTED_EXTENSIONS = (".jpg", ".jpeg", ".png", ".bmp", ".tiff", ".webp")

    def __init__(self, root: str, transform: Optional[ImageTransform] = None, conditional: bool = False,
                 label_file: Optional[str] = None, use_subdirs: bool = False):
        self.root, self.transform, self.conditional, self.use_subdirs = Path(root), transform, conditional, use_subdirs
        if conditional and not (use_subdirs or label_file):
            raise ValueError("CustomImageDataset with conditional=True requires either use_subdirs=True or a "
                             "label_file.")
        self.image_paths, labels, self.class_to_idx = [], [], {}
        if use_subdirs:
            classes = sorted(p for p in self.root.iterdir() if p.is_dir())
            self.class_to_idx = {c.name: i for i, c in enumerate(classes)}
            for c in classes:
                for p in c.iterdir():
                    if p.is_file() and p.suffix.lower() in self.SUPPORTED_EXTENSIONS:
                        self.image_paths.append(p)
                        labels.append(self.class_to_idx[c.name])
        elif label_file:
            with open(label_file, "r", encoding="utf-8") as f:
                lab = json.load(f)
            for fn, l in lab.items():
                if (self.root / fn).exists():
                    self.image_paths.append(self.root / fn)
                    labels.append(l)
            self.class_to_idx = {l: i for i, l in enumerate(sorted(set(labels)))}
            labels = [self.class_to_idx[l] for l in labels]
        else:
            self.image_paths = [p for p in self.root.iterdir()
                                 if p.is_file() and p.suffix.lower() in self.SUPPORTED_EXTENSIONS]
        tr = transform or ImageTransform(32, True, 0.0, [0.5] * 3, [0.5] * 3)
        self.images = _decode_all(self.image_paths, tr, "RGB")
        self.labels = np.asarray(labels, dtype=np.int64) if labels else None

    @property
    def num_classes(self):
        return len(self.class_to_idx) if self.conditional else 0

    @staticmethod
    def get_default_transform(image_size=32, dataset_type="rgb", train=True):
        """datasets/custom_dataset.py:150-170."""
        return ImageTransform(image_size, True, 0.5 if train else 0.0, [0.5] * 3, [0.5] * 3)


def from_arrays(images: np.ndarray, labels=None, conditional: bool = False, transform=None) -> _BankDataset:
    """A bank dataset over an in-memory uint8 [N, H, W, C] array (synthetic data, benchmarks, tests)."""
    ds = _BankDataset()
    ds.images = np.ascontiguousarray(images, dtype=np.uint8)
    ds.labels = None if labels is None else np.asarray(labels, dtype=np.int64)
    ds.conditional, ds.transform = conditional, transform
    return ds


__all__ = ["DiffusionDataset", "CustomImageDataset", "ImageTransform", "from_arrays"]
