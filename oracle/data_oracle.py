"""CPU ORACLE — test infrastructure only. Never imported by the product path.

Restatement of the reference's per-sample training transform (datasets/base_dataset.py:100-133,
datasets/custom_dataset.py:150-170): RandomHorizontalFlip -> ToTensor -> Normalize. Those ops live in torchvision
(requirements.txt: `torchvision`, unpinned; absent in this image), so this follows torchvision's published
algorithm, 0.15-0.20 `transforms.functional`:
  hflip        PIL `img.transpose(FLIP_LEFT_RIGHT)`               -> columns reversed
  to_tensor    `torch.from_numpy(np.array(pic)).view(h, w, c).permute(2, 0, 1).contiguous().to(float32).div(255)`
  normalize    `tensor.sub_(mean[:, None, None]).div_(std[:, None, None])` (mean/std as float32 tensors)
evaluated here with the same torch CPU ops, so the values are the reference's bit for bit. The flip DECISION of
the device loader is its own counter hash (datasets/loader.py docstring); `flip_hash` restates it.
"""
import numpy as np
import torch


def to_tensor_normalize(img_hwc_u8: np.ndarray, mean, std, flip: bool = False) -> torch.Tensor:
    a = np.asarray(img_hwc_u8, dtype=np.uint8)
    if a.ndim == 2:
        a = a[:, :, None]
    if flip:
        a = a[:, ::-1]
    t = torch.from_numpy(np.ascontiguousarray(a)).permute(2, 0, 1).contiguous().to(torch.float32).div(255)
    m = torch.as_tensor(mean, dtype=torch.float32)
    s = torch.as_tensor(std, dtype=torch.float32)
    return t.sub_(m[:, None, None]).div_(s[:, None, None])


def load_batch(bank: np.ndarray, idx, mean, std, flips) -> torch.Tensor:
    """Batch of the device loader: out[b] = to_tensor_normalize(bank[idx[b]], flip=flips[b]), NCHW fp32."""
    return torch.stack([to_tensor_normalize(bank[int(i)], mean, std, bool(f)) for i, f in zip(idx, flips)])


def hash_u32(x, seed):
    """csrc/dmc_common.h hash_u32 in numpy uint32 arithmetic."""
    with np.errstate(over="ignore"):
        x = (np.asarray(x, dtype=np.uint32) ^ np.uint32(seed)).astype(np.uint32)
        x = (x * np.uint32(0x9E3779B1)).astype(np.uint32); x ^= x >> np.uint32(16)
        x = (x * np.uint32(0x85EBCA6B)).astype(np.uint32); x ^= x >> np.uint32(13)
        x = (x * np.uint32(0xC2B2AE35)).astype(np.uint32); x ^= x >> np.uint32(16)
    return x


def flip_hash(pos0: int, B: int, seed: int, p: float) -> np.ndarray:
    """dmc_load_batch's flip draw: hash(pos0 + b, seed) < p * 2^32."""
    thresh = min(int(round(p * 4294967296.0)), 0xFFFFFFFF)
    if thresh == 0:
        return np.zeros(B, dtype=bool)
    pos = (np.arange(B, dtype=np.int64) + pos0).astype(np.uint32)
    return hash_u32(pos, seed & 0xFFFFFFFF) < np.uint32(thresh)
