"""Device-resident data path (datasets/base_dataset.py:96-133, train.py:107-128 of the reference).

CPU tests: the dataset file readers, the host Resize/CenterCrop arithmetic, the oracle's op sequence, and that the
loader draws its epoch order exactly as torch's DataLoader does. GPU tests: dmc_load_batch bit-exact against the
oracle (oracle/data_oracle.py), and whole epochs through DeviceLoader."""
import gzip
import pickle
import struct

import numpy as np
import pytest
import torch
from torch.utils.data import DataLoader, DistributedSampler

from oracle import data_oracle as O
from diffusion_models_collection_amd.datasets import DiffusionDataset, ImageTransform, from_arrays
from diffusion_models_collection_amd.datasets.base_dataset import _SafeUnpickler

DEV = "cuda"


def _cifar_bin(path, data_chw, labels, label_bytes=1):
    rec = np.zeros((len(labels), label_bytes + 3072), np.uint8)
    rec[:, label_bytes - 1] = labels
    if label_bytes == 2:
        rec[:, 0] = 7   # coarse label, ignored
    rec[:, label_bytes:] = data_chw.reshape(len(labels), -1)
    rec.tofile(path)


def test_cifar10_binary_reader(tmp_path):
    rng = np.random.default_rng(0)
    d = tmp_path / "cifar-10-batches-bin"
    d.mkdir()
    chw, lab = [], []
    for i in range(1, 6):
        x = rng.integers(0, 256, (4, 3, 32, 32), dtype=np.uint8)
        y = rng.integers(0, 10, 4)
        _cifar_bin(d / f"data_batch_{i}.bin", x, y)
        chw.append(x), lab.append(y)
    _cifar_bin(d / "test_batch.bin", chw[0][:2], lab[0][:2])
    ds = DiffusionDataset("CIFAR10", root=str(tmp_path), train=True, conditional=True,
                          transform=DiffusionDataset.get_default_transform((32, 32), "cifar10", True))
    assert len(ds) == 20 and ds.images.shape == (20, 32, 32, 3)
    np.testing.assert_array_equal(ds.images, np.concatenate(chw).transpose(0, 2, 3, 1))
    np.testing.assert_array_equal(ds.labels, np.concatenate(lab))
    img, y = ds[3]
    assert img.shape == (3, 32, 32) and y == int(np.concatenate(lab)[3])
    assert len(DiffusionDataset("cifar10", root=str(tmp_path), train=False)) == 2


def test_cifar100_binary_and_python_layouts(tmp_path):
    rng = np.random.default_rng(1)
    x = rng.integers(0, 256, (5, 3, 32, 32), dtype=np.uint8)
    y = rng.integers(0, 100, 5)
    (tmp_path / "cifar-100-binary").mkdir()
    _cifar_bin(tmp_path / "cifar-100-binary" / "train.bin", x, y, label_bytes=2)
    ds = DiffusionDataset("cifar100", root=str(tmp_path))
    np.testing.assert_array_equal(ds.labels, y)            # fine label, not the coarse byte
    np.testing.assert_array_equal(ds.images, x.transpose(0, 2, 3, 1))
    # python layout (torchvision's download) through the restricted unpickler
    p2 = tmp_path / "p2"
    (p2 / "cifar-100-python").mkdir(parents=True)
    with open(p2 / "cifar-100-python" / "train", "wb") as f:
        pickle.dump({b"data": x.reshape(5, -1), b"fine_labels": list(map(int, y)), b"coarse_labels": [0] * 5}, f)
    ds2 = DiffusionDataset("cifar100", root=str(p2))
    np.testing.assert_array_equal(ds2.images, ds.images)
    np.testing.assert_array_equal(ds2.labels, ds.labels)


def test_safe_unpickler_refuses_code(tmp_path):
    class Evil:
        def __reduce__(self):
            return (print, ("pwned",))
    blob = pickle.dumps({b"data": Evil()})
    import io
    with pytest.raises(pickle.UnpicklingError):
        _SafeUnpickler(io.BytesIO(blob), encoding="bytes").load()


def _idx(path, arr, gz=False):
    hdr = struct.pack(">HBB", 0, 8, arr.ndim) + struct.pack(">" + "I" * arr.ndim, *arr.shape)
    data = hdr + arr.astype(np.uint8).tobytes()
    (gzip.open if gz else open)(path, "wb").write(data)


@pytest.mark.parametrize("name,gz", [("mnist", False), ("fashionmnist", True)])
def test_mnist_idx_reader(tmp_path, name, gz):
    rng = np.random.default_rng(2)
    raw = tmp_path / ("MNIST" if name == "mnist" else "FashionMNIST") / "raw"
    raw.mkdir(parents=True)
    x = rng.integers(0, 256, (6, 28, 28), dtype=np.uint8)
    y = rng.integers(0, 10, 6).astype(np.uint8)
    sfx = ".gz" if gz else ""
    _idx(raw / f"train-images-idx3-ubyte{sfx}", x, gz)
    _idx(raw / f"train-labels-idx1-ubyte{sfx}", y, gz)
    tr = DiffusionDataset.get_default_transform(28, name, True)
    assert tr.flip_p == 0.0 and tr.mean == [0.5]           # grayscale: no flip (base_dataset.py:111-116)
    ds = DiffusionDataset(name, root=str(tmp_path), transform=tr)
    assert ds.images.shape == (6, 28, 28, 1)
    np.testing.assert_array_equal(ds.images[..., 0], x)
    ref = O.to_tensor_normalize(x[2], [0.5], [0.5])
    assert torch.equal(ds[2], ref)


def test_missing_dataset_and_unknown_name(tmp_path):
    with pytest.raises(FileNotFoundError):
        DiffusionDataset("cifar10", root=str(tmp_path))
    with pytest.raises(ValueError, match="not supported"):
        DiffusionDataset("imagenet", root=str(tmp_path))


def test_resize_center_crop_arithmetic():
    """torchvision Resize(int) (shorter side, int(size*long/short)) + CenterCrop(round((h-th)/2)) on PIL."""
    from PIL import Image
    rng = np.random.default_rng(3)
    a = rng.integers(0, 256, (50, 40, 3), dtype=np.uint8)     # h=50, w=40
    tr = ImageTransform(32, True, 0.0, [0.5] * 3, [0.5] * 3)
    out = tr.prepare(a)
    im = Image.fromarray(a).resize((32, 40), Image.BILINEAR)  # w<=h: (32, int(32*50/40)=40)
    ref = np.asarray(im)[4:36, 0:32]                          # top = round((40-32)/2) = 4
    np.testing.assert_array_equal(out, ref)
    same = rng.integers(0, 256, (32, 32, 3), dtype=np.uint8)
    np.testing.assert_array_equal(tr.prepare(same), same)     # already at size: untouched


def test_oracle_op_sequence_is_float32_ieee():
    """((u / 255) - m) / s with float32 IEEE ops, the values the device kernel must reproduce."""
    u = np.arange(256, dtype=np.uint8).reshape(16, 16, 1)
    t = O.to_tensor_normalize(u, [0.5], [0.5]).numpy()[0]
    ref = ((u[..., 0].astype(np.float32) / np.float32(255)) - np.float32(0.5)) / np.float32(0.5)
    assert np.array_equal(t, ref)
    assert t.min() == -1.0 and t.max() == 1.0


def _index_batches_reference(n, bs, shuffle, sampler, drop_last, seed):
    torch.manual_seed(seed)
    dl = DataLoader(torch.utils.data.TensorDataset(torch.arange(n)), batch_size=bs, shuffle=shuffle, sampler=sampler,
                    drop_last=drop_last, num_workers=0)
    return [b[0] for b in dl]


@pytest.mark.parametrize("shuffle,drop_last", [(True, True), (False, False), (True, False)])
def test_loader_epoch_order_matches_dataloader(shuffle, drop_last):
    from diffusion_models_collection_amd.datasets.loader import DeviceLoader
    ds = from_arrays(np.zeros((103, 4, 4, 3), np.uint8))
    ld = DeviceLoader(ds, 16, shuffle=shuffle, drop_last=drop_last, device="cpu")
    for seed in (0, 5):
        ref = _index_batches_reference(103, 16, shuffle, None, drop_last, seed)
        torch.manual_seed(seed)
        got = ld.epoch_indices()
        assert len(got) == len(ref) == len(ld)
        for g, r in zip(got, ref):
            assert torch.equal(g, r)


def test_loader_distributed_order_matches_dataloader():
    from diffusion_models_collection_amd.datasets.loader import DeviceLoader, get_dataloader
    ds = from_arrays(np.zeros((50, 4, 4, 3), np.uint8))
    seen = []
    for rank in range(2):
        ld = get_dataloader({"batch_size": 8}, ds, rank=rank, world_size=2, train=True, device="cpu")
        assert isinstance(ld, DeviceLoader) and isinstance(ld.sampler, DistributedSampler)
        for epoch in (0, 3):
            ld.sampler.set_epoch(epoch)
            s_ref = DistributedSampler(ds, num_replicas=2, rank=rank, shuffle=True)
            s_ref.set_epoch(epoch)
            ref = _index_batches_reference(50, 8, False, s_ref, True, 0)
            got = ld.epoch_indices()
            assert [g.tolist() for g in got] == [r.tolist() for r in ref]
            if epoch == 0:
                seen += [i for g in got for i in g.tolist()]
    assert len(set(seen)) == 48     # 2 ranks x 3 full batches of 8, disjoint


def test_device_loader_refuses_host_bank():
    from diffusion_models_collection_amd.datasets.loader import DeviceLoader
    ld = DeviceLoader(from_arrays(np.zeros((4, 4, 4, 3), np.uint8)), 2, device="cpu")
    with pytest.raises(RuntimeError, match="device memory"):
        next(iter(ld))


# ---------------------------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("C,H,W", [(3, 32, 32), (1, 28, 28), (3, 64, 64), (3, 5, 7)])
def test_load_batch_bitexact(C, H, W):
    from diffusion_models_collection_amd.datasets.loader import load_batch
    rng = np.random.default_rng(C * 100 + H)
    N, B = 37, 19
    bank = rng.integers(0, 256, (N, H, W, C), dtype=np.uint8)
    idx = rng.integers(0, N, B).astype(np.int32)
    mean = [0.5, 0.4914, 0.4822][:C]
    std = [0.5, 0.247, 0.2435][:C]
    flips = rng.integers(0, 2, B).astype(np.uint8)
    labels = torch.from_numpy(rng.integers(0, 10, N)).to(DEV)
    bank_d = torch.from_numpy(bank).to(DEV)
    y = torch.empty(B, dtype=torch.int64, device=DEV)
    out = load_batch(bank_d, torch.from_numpy(idx).to(DEV), mean, std, flips=torch.from_numpy(flips).to(DEV),
                     labels=labels, labels_out=y)
    ref = O.load_batch(bank, idx, mean, std, flips)
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), ref)
    assert torch.equal(y.cpu(), labels.cpu()[torch.from_numpy(idx).long()])
    # hash flips (p = 0.5): the device draw equals the host restatement
    out2 = load_batch(bank_d, torch.from_numpy(idx).to(DEV), mean, std, flip_seed=1234, flip_p=0.5, pos0=77)
    ref2 = O.load_batch(bank, idx, mean, std, O.flip_hash(77, B, 1234, 0.5))
    assert torch.equal(out2.cpu(), ref2)
    # p = 0: no flips
    out3 = load_batch(bank_d, torch.from_numpy(idx).to(DEV), mean, std, flip_seed=1234, flip_p=0.0)
    assert torch.equal(out3.cpu(), O.load_batch(bank, idx, mean, std, np.zeros(B, bool)))


@pytest.mark.gpu
def test_load_batch_edge_cases():
    from diffusion_models_collection_amd import _lib as L
    from diffusion_models_collection_amd.datasets.loader import load_batch
    bank = torch.zeros(3, 4, 4, 3, dtype=torch.uint8, device=DEV)
    e = load_batch(bank, torch.zeros(0, dtype=torch.int32, device=DEV), [0.5] * 3, [0.5] * 3)   # empty batch
    assert e.shape == (0, 3, 4, 4)
    with pytest.raises(L.DMCError):
        load_batch(bank, torch.zeros(2, dtype=torch.int64, device=DEV), [0.5] * 3, [0.5] * 3)     # wrong idx dtype
    with pytest.raises(L.DMCError, match="zero"):
        load_batch(bank, torch.zeros(2, dtype=torch.int32, device=DEV), [0.5] * 3, [0.5, 0.0, 0.5])
    # flip statistics of the hash draw: p = 0.5 over 20k positions
    f = O.flip_hash(0, 20000, 99, 0.5)
    assert abs(f.mean() - 0.5) < 0.02


@pytest.mark.gpu
def test_device_loader_epoch_matches_oracle():
    from diffusion_models_collection_amd.datasets.loader import DeviceLoader, epoch_seed
    rng = np.random.default_rng(7)
    imgs = rng.integers(0, 256, (70, 32, 32, 3), dtype=np.uint8)
    tr = DiffusionDataset.get_default_transform(32, "cifar10", train=True)
    ds = from_arrays(imgs, labels=rng.integers(0, 10, 70), conditional=True, transform=tr)
    ld = DeviceLoader(ds, 16, shuffle=True, drop_last=True, seed=3)
    for epoch in range(2):
        torch.manual_seed(11 + epoch)
        order = ld.epoch_indices()
        torch.manual_seed(11 + epoch)
        e = ld.epoch
        batches = list(ld)
        assert len(batches) == 4
        pos = 0
        for (x, y), ix in zip(batches, order):
            flips = O.flip_hash(pos, len(ix), epoch_seed(3, e), 0.5)
            ref = O.load_batch(imgs, ix.numpy(), tr.mean, tr.std, flips)
            assert torch.equal(x.cpu(), ref)
            assert torch.equal(y.cpu(), torch.from_numpy(ds.labels[ix.numpy()]))
            pos += len(ix)


@pytest.mark.gpu
def test_trainer_epoch_on_device_loader_matches_oracle_batches(tmp_path, monkeypatch):
    """DiffusionTrainer.train_epoch fed by DeviceLoader == the same trainer fed the oracle's batches (same order,
    same flips): the loader changes where the batch comes from, not what the step computes."""
    monkeypatch.setenv("DMC_GRAPH", "0")
    from diffusion_models_collection_amd.datasets.loader import DeviceLoader, epoch_seed
    from diffusion_models_collection_amd.diffusion import DDPM
    from diffusion_models_collection_amd.models import UNet
    from diffusion_models_collection_amd.utils.trainer import DiffusionTrainer
    cfg = dict(image_size=(16, 16), in_channels=3, model_channels=32, out_channels=3, num_res_blocks=1,
               attention_resolutions=(8,), dropout=0.0, channel_mult=(1, 2), use_attention=True)
    rng = np.random.default_rng(5)
    imgs = rng.integers(0, 256, (40, 16, 16, 3), dtype=np.uint8)
    tr_ = DiffusionDataset.get_default_transform(16, "cifar10", train=True)
    ds = from_arrays(imgs, transform=tr_)

    def run(loader):
        torch.manual_seed(0)
        m = UNet(**cfg).to(DEV)
        opt = torch.optim.AdamW(m.parameters(), lr=2e-4, weight_decay=1e-4)
        conf = {"epochs": 1, "save_dir": str(tmp_path / "c"), "sample_dir": str(tmp_path / "s"), "loss_type": "l2",
                "use_ema": True, "ema_decay": 0.9, "model_type": "unet", "model_params": cfg}
        t = DiffusionTrainer(m, DDPM(device=DEV), loader, opt, None, device=DEV, config=conf)
        torch.manual_seed(1)
        loss = t.train_epoch(1)
        return loss, torch.cat([p.detach().flatten() for p in m.parameters()]).cpu()

    ld = DeviceLoader(ds, 8, shuffle=True, drop_last=True, seed=9)
    torch.manual_seed(1)
    order = ld.epoch_indices()
    l_dev, p_dev = run(ld)
    pos, ref_batches = 0, []
    for ix in order:
        fl = O.flip_hash(pos, len(ix), epoch_seed(9, 1), 0.5)   # train_epoch(1) sets the loader's epoch to 1
        ref_batches.append(O.load_batch(imgs, ix.numpy(), tr_.mean, tr_.std, fl))
        pos += len(ix)
    l_ref, p_ref = run(ref_batches)
    assert np.isfinite(l_dev) and l_dev == l_ref
    assert torch.equal(p_dev, p_ref)


def test_custom_image_dataset_subdirs_and_json(tmp_path):
    """datasets/custom_dataset.py semantics: class subdirectories -> labels in sorted-name order; a JSON label file
    -> labels remapped to consecutive indices; images decoded once through Resize + CenterCrop."""
    from PIL import Image
    from diffusion_models_collection_amd.datasets import CustomImageDataset
    rng = np.random.default_rng(4)
    for cls in ("zebra", "ant"):
        (tmp_path / cls).mkdir()
        for i in range(3):
            Image.fromarray(rng.integers(0, 256, (40, 48, 3), dtype=np.uint8)).save(tmp_path / cls / f"{i}.png")
    tr = CustomImageDataset.get_default_transform(32, "rgb", train=True)
    ds = CustomImageDataset(str(tmp_path), transform=tr, conditional=True, use_subdirs=True)
    assert len(ds) == 6 and ds.images.shape == (6, 32, 32, 3)
    assert ds.class_to_idx == {"ant": 0, "zebra": 1} and ds.num_classes == 2
    assert sorted(ds.labels.tolist()) == [0, 0, 0, 1, 1, 1]
    img, y = ds[0]
    assert img.shape == (3, 32, 32) and y in (0, 1)
    flat = tmp_path / "flat"
    flat.mkdir()
    for i in range(2):
        Image.fromarray(rng.integers(0, 256, (32, 32, 3), dtype=np.uint8)).save(flat / f"im{i}.png")
    (tmp_path / "labels.json").write_text('{"im0.png": 7, "im1.png": 3}')
    dj = CustomImageDataset(str(flat), conditional=True, label_file=str(tmp_path / "labels.json"))
    assert sorted(dj.labels.tolist()) == [0, 1] and dj.class_to_idx == {3: 0, 7: 1}
    with pytest.raises(ValueError, match="requires either"):
        CustomImageDataset(str(flat), conditional=True)


def test_get_dataset_from_config(tmp_path):
    """train.py:84-104 get_dataset on the reference's config keys (dataset, data_root, image_size, conditional)."""
    from diffusion_models_collection_amd.datasets.loader import get_dataset
    d = tmp_path / "cifar-10-batches-bin"
    d.mkdir()
    rng = np.random.default_rng(6)
    for name in [f"data_batch_{i}.bin" for i in range(1, 6)] + ["test_batch.bin"]:
        _cifar_bin(d / name, rng.integers(0, 256, (2, 3, 32, 32), dtype=np.uint8), rng.integers(0, 10, 2))
    ds = get_dataset({"dataset": "cifar10", "data_root": str(tmp_path), "image_size": 32, "conditional": True})
    assert len(ds) == 10 and ds.conditional and ds.transform.flip_p == 0.5
    dt = get_dataset({"dataset": "cifar10", "data_root": str(tmp_path), "image_size": (32, 32)}, train=False)
    assert len(dt) == 2 and dt.transform.flip_p == 0.0
