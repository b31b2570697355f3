"""Device-resident batch loader: the reference's DataLoader (train.py:107-128) with the dataset in HBM.

The bank (uint8 [N, H, W, C], datasets/base_dataset.py) is copied to the device once. Every epoch the sample order
comes from the SAME torch samplers the reference's DataLoader uses -- `RandomSampler` (shuffle=True, one world) or
`DistributedSampler(num_replicas, rank, shuffle=True)` (`set_epoch` per epoch) -- driven exactly as
`torch.utils.data.DataLoader.__iter__` drives them (it draws the loader's base seed from torch's CPU generator
before the sampler's own draw), so for the same `torch.manual_seed` the batches hold the same images as the
reference's. The epoch's index list goes to the device in one copy; each batch is then ONE kernel
(`dmc_load_batch`: gather, RandomHorizontalFlip, ToTensor, Normalize -> NCHW fp32) with no host work per batch.

RandomHorizontalFlip: the reference draws `torch.rand(1) < 0.5` per sample inside its worker processes, whose
generators are seeded from that base seed plus the worker id, so its flip pattern is not reproducible across
worker counts. Here a sample's flip is a counter hash of (seed, epoch, position in the epoch): p = 0.5,
deterministic, recomputable, no host RNG traffic.
"""
import numpy as np
import torch
from torch.utils.data import DataLoader, DistributedSampler

from .. import _lib as L
from .._lib import LIB, check, ptr

ctypes_f = L._c_f


def load_batch(bank, idx, mean, std, out=None, flips=None, flip_seed=0, flip_p=0.0, pos0=0, labels=None,
               labels_out=None):
    """dmc_load_batch over device tensors: bank uint8 [N,H,W,C], idx int32 [B] (validated by the caller)."""
    N, H, W, C = bank.shape
    B = idx.numel()
    if not bank.is_cuda:
        raise L.DMCError("dmc_load_batch: the image bank must be in device memory")
    if bank.dtype != torch.uint8 or not bank.is_contiguous():
        raise L.DMCError("dmc_load_batch: bank must be a contiguous uint8 [N,H,W,C] tensor")
    if idx.dtype != torch.int32 or idx.device != bank.device or not idx.is_contiguous():
        raise L.DMCError("dmc_load_batch: idx must be a contiguous int32 tensor on the bank's device")
    if out is None:
        out = torch.empty(B, C, H, W, dtype=torch.float32, device=bank.device)
    if tuple(out.shape) != (B, C, H, W) or out.dtype != torch.float32 or not out.is_contiguous():
        raise L.DMCError(f"dmc_load_batch: out must be fp32 [{B},{C},{H},{W}]")
    if flips is not None and (flips.dtype != torch.uint8 or flips.numel() != B):
        raise L.DMCError("dmc_load_batch: flips must be uint8 [B]")
    if (labels is None) != (labels_out is None):
        raise L.DMCError("dmc_load_batch: labels and labels_out go together")
    m = (ctypes_f * C)(*[float(v) for v in mean])
    s = (ctypes_f * C)(*[float(v) for v in std])
    thresh = min(int(round(float(flip_p) * 4294967296.0)), 0xFFFFFFFF)
    check(LIB.dmc_load_batch(ptr(bank), N, H, W, C, ptr(idx), B, ptr(flips), flip_seed & 0xFFFFFFFF, thresh, int(pos0),
                             m, s, ptr(out), ptr(labels), ptr(labels_out), L.stream()), "dmc_load_batch")
    return out



def epoch_seed(seed: int, epoch: int) -> int:
    """Flip-hash seed of an epoch (splitmix-style mix of (seed, epoch))."""
    z = (int(seed) * 0x9E3779B97F4A7C15 + int(epoch) * 0xBF58476D1CE4E5B9 + 1) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 30)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return (z ^ (z >> 31)) & 0xFFFFFFFF


class _Range(torch.utils.data.Dataset):
    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return i


class DeviceLoader:
    """Iterable of device batches: x fp32 [B, C, H, W] (and labels int64 [B] when the dataset is conditional).

    DeviceLoader(dataset, batch_size, shuffle=True, sampler=None, drop_last=True, device=None, seed=0) mirrors
    DataLoader(dataset, batch_size, shuffle, sampler, drop_last, pin_memory=True) of the reference's get_dataloader
    (train.py:115-128); `sampler` may be a torch DistributedSampler over the dataset (its set_epoch is honoured,
    as the trainer calls it, utils/trainer.py:210-211). The flip probability and normalisation come from the
    dataset's ImageTransform (none -> no flip, ToTensor only)."""

    def __init__(self, dataset, batch_size, shuffle=True, sampler=None, drop_last=True, device=None, seed=0):
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.dataset, self.batch_size, self.shuffle, self.sampler = dataset, int(batch_size), shuffle, sampler
        self.drop_last, self.device, self.seed = drop_last, torch.device(device), int(seed)
        if sampler is not None and shuffle:
            raise ValueError("sampler option is mutually exclusive with shuffle")
        imgs = np.ascontiguousarray(dataset.images, dtype=np.uint8)
        if imgs.ndim != 4 or imgs.shape[3] > 4:
            raise ValueError(f"bank must be [N, H, W, C<=4] uint8, got {imgs.shape}")
        self.bank = torch.from_numpy(imgs).to(self.device)           # resident for the loader's lifetime
        self.conditional = bool(getattr(dataset, "conditional", False))
        lab = getattr(dataset, "labels", None)
        if self.conditional:
            lab = np.zeros(len(imgs), np.int64) if lab is None else lab
            self.labels = torch.from_numpy(np.asarray(lab, dtype=np.int64)).to(self.device)
        tr = getattr(dataset, "transform", None)
        C = imgs.shape[3]
        self.mean = tr.mean if tr is not None else [0.0] * C
        self.std = tr.std if tr is not None else [1.0] * C
        self.flip_p = tr.flip_p if tr is not None else 0.0
        if len(self.mean) != C or len(self.std) != C:
            raise ValueError(f"Normalize has {len(self.mean)} channels, the images {C}")
        # index order exactly as DataLoader produces it (same samplers, same generator draws)
        self._index_loader = DataLoader(_Range(len(imgs)), batch_size=self.batch_size,
                                        shuffle=shuffle if sampler is None else False, sampler=sampler,
                                        drop_last=drop_last, num_workers=0)
        self.epoch = 0

    def __len__(self):
        return len(self._index_loader)

    def set_epoch(self, epoch):
        self.epoch = int(epoch)

    def epoch_indices(self):
        """The epoch's batches of dataset indices (host), drawn as the reference's DataLoader draws them."""
        return [b.to(torch.int64) for b in self._index_loader]

    def __iter__(self):
        batches = self.epoch_indices()
        if isinstance(self.sampler, DistributedSampler):
            self.epoch = self.sampler.epoch
        ep = self.epoch
        if self.sampler is None:
            # advance when the epoch STARTS: an iteration cut short (early break, an exception) must not make the
            # next epoch reuse this epoch's flips
            self.epoch += 1
        if not batches:
            return
        flat = torch.cat(batches)
        n = len(self.dataset)
        if flat.numel() and (int(flat.min()) < 0 or int(flat.max()) >= n):
            raise IndexError("sampler produced an index outside the dataset")
        idx = flat.to(torch.int32).to(self.device, non_blocking=True)
        fseed = epoch_seed(self.seed, ep)
        # flip-hash positions: the rank's slice of the epoch (distributed) so ranks draw independent flips
        pos = self.sampler.rank * self.sampler.num_samples if isinstance(self.sampler, DistributedSampler) else 0
        pos_base = pos
        for b in batches:
            B = b.numel()
            sl = idx[pos - pos_base:pos - pos_base + B]
            y = torch.empty(B, dtype=torch.int64, device=self.device) if self.conditional else None
            x = load_batch(self.bank, sl, self.mean, self.std, flip_seed=fseed, flip_p=self.flip_p, pos0=pos,
                           labels=self.labels if self.conditional else None, labels_out=y)
            pos += B
            yield (x, y) if self.conditional else x


def get_dataloader(config, dataset, rank=0, world_size=1, train=True, device=None):
    """train.py:115-128 (get_dataloader) on the device loader: DistributedSampler when world_size > 1 and
    training, shuffle when training, drop_last when training."""
    if world_size > 1 and train:
        sampler, shuffle = DistributedSampler(dataset, num_replicas=world_size, rank=rank, shuffle=True), False
    else:
        sampler, shuffle = None, train
    return DeviceLoader(dataset, config["batch_size"], shuffle=shuffle, sampler=sampler, drop_last=train,
                        device=device, seed=int(config.get("seed", 0)))


def get_dataset(config, train=True):
    """train.py:84-104 (get_dataset)."""
    from ..utils.helpers import resolve_image_size
    from .base_dataset import CustomImageDataset, DiffusionDataset
    name = config["dataset"].lower()
    size = resolve_image_size(config["image_size"])
    if name == "custom":
        return CustomImageDataset(root=config["data_root"],
                                  transform=CustomImageDataset.get_default_transform(size, "rgb", train=train),
                                  conditional=config.get("conditional", False), label_file=config.get("label_file"),
                                  use_subdirs=config.get("use_subdirs", False))
    return DiffusionDataset(dataset_name=name, root=config["data_root"], train=train,
                            transform=DiffusionDataset.get_default_transform(size, name, train=train), download=True,
                            conditional=config.get("conditional", False))
