"""Datasets: partitioning, on-device synthetic batches, and offline loaders.

Reference (/root/reference/src/data.py):
* ``DataPartitioner`` — ``randperm(len)`` under the global seed, ``total_dev`` disjoint partitions
  of ``batches_per_dev * batch_size`` samples, partition index ``node_id*node_dev + worker_id``
  (data.py:26-41,58-68). Kept with identical semantics.
* MNIST / ImageFolder loaders via torchvision with downloads (data.py:71-127). torchvision is not
  installed and there is no network, so this module reads the on-disk formats directly: MNIST idx
  files, CIFAR-10 binary batches, and ImageFolder trees (PIL), each optional.
* ``random_data_generator`` — CPU ``rand_like``/``randint_like`` per step from a real template
  batch (data.py:129-132; ~130 ms/step on the reference's hardware). Replaced by
  :class:`SyntheticBatches`, which generates each batch directly in HBM with the native Philox
  kernel (csrc/kernels/synthetic.hip) and needs no dataset on disk.
"""
from __future__ import annotations

import os
import struct
from pathlib import Path
from typing import Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .ops import _ext

PER_WORKER_BATCH_SIZE = 128


class Partition(torch.utils.data.Dataset):
    """Index view over a dataset (reference data.py:10-23)."""

    def __init__(self, data, index: Sequence[int]):
        self.data = data
        self.index = index

    def __len__(self):
        return len(self.index)

    def __getitem__(self, i):
        return self.data[int(self.index[i])]


class DataPartitioner:
    """``total_dev`` disjoint, equally sized partitions (reference data.py:26-41)."""

    def __init__(self, data, total_dev: int, batch_size: int, seed: int = 1234):
        self.data = data
        n = len(data)
        batches_per_dev = n // total_dev // batch_size
        part_len = batches_per_dev * batch_size
        g = torch.Generator().manual_seed(seed)
        idx = torch.randperm(n, generator=g)
        self.partitions: List[torch.Tensor] = [idx[i * part_len:(i + 1) * part_len] for i in range(total_dev)]

    def use(self, partition: int) -> Partition:
        return Partition(self.data, self.partitions[partition])


class EpochSampler(torch.utils.data.Sampler):
    """Shuffled order drawn from (seed, epoch) alone, with a start offset.

    The reference shuffles with ``DataLoader(shuffle=True)`` (data.py:67), whose order depends on the
    global RNG state at the moment each epoch starts, so a run cannot be resumed mid-epoch on the same
    sequence. Here epoch e's permutation is a pure function of (seed, e): a resumed run at global
    batch k sets epoch k // batches_per_epoch and starts k % batches_per_epoch batches into it,
    without loading or decoding the skipped samples."""

    def __init__(self, n: int, seed: int = 1234):
        self.n, self.seed = n, seed
        self.epoch, self.start = 0, 0

    def set_epoch(self, epoch: int, start: int = 0) -> None:
        self.epoch, self.start = int(epoch), int(start)

    def order(self, epoch: int) -> List[int]:
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + epoch)
        return torch.randperm(self.n, generator=g).tolist()

    def __iter__(self):
        return iter(self.order(self.epoch)[self.start:])

    def __len__(self):
        return self.n - self.start


def resume_position(start_step: int, batches_per_epoch: int) -> Tuple[int, int]:
    """(epoch, batches to skip inside it) of global batch ``start_step``."""
    if batches_per_epoch <= 0:
        return 0, 0
    return start_step // batches_per_epoch, start_step % batches_per_epoch


def get_partition_loader(dataset, node_id: int, worker_id: int, node_dev: int, total_dev: int,
                         batch_size: int = PER_WORKER_BATCH_SIZE, num_workers: int = 2, seed: int = 1234):
    part = DataPartitioner(dataset, total_dev, batch_size, seed).use(node_id * node_dev + worker_id)
    sampler = EpochSampler(len(part), seed + node_id * node_dev + worker_id)
    # own generator: the loader's per-iterator worker seed must not be drawn from the global RNG, or every
    # epoch start (and a resume's first iterator) would shift the model's dropout stream
    loader = torch.utils.data.DataLoader(part, batch_size=batch_size, sampler=sampler, num_workers=num_workers,
                                         drop_last=True, generator=torch.Generator().manual_seed(seed))
    loader.epoch_sampler = sampler
    return loader


# ------------------------------------------------------------------------------------------------
# Offline dataset readers (no torchvision, no downloads)
# ------------------------------------------------------------------------------------------------
class TensorDataset(torch.utils.data.Dataset):
    def __init__(self, x: torch.Tensor, y: torch.Tensor):
        self.x, self.y = x, y

    def __len__(self):
        return self.x.shape[0]

    def __getitem__(self, i):
        return self.x[i], self.y[i]


def _read_idx(path: Path) -> np.ndarray:
    with open(path, "rb") as f:
        magic = struct.unpack(">I", f.read(4))[0]
        ndim = magic & 0xFF
        dims = struct.unpack(">" + "I" * ndim, f.read(4 * ndim))
        return np.frombuffer(f.read(), dtype=np.uint8).reshape(dims)


def load_mnist(root: str, train: bool = True) -> TensorDataset:
    """MNIST from idx files under ``root/mnist/MNIST/raw`` (torchvision layout) or ``root/mnist``."""
    stem = "train" if train else "t10k"
    for d in (Path(root) / "mnist" / "MNIST" / "raw", Path(root) / "mnist", Path(root)):
        img, lab = d / f"{stem}-images-idx3-ubyte", d / f"{stem}-labels-idx1-ubyte"
        if img.exists() and lab.exists():
            x = torch.from_numpy(_read_idx(img).astype(np.float32) / 255.0).unsqueeze(1)
            x = (x - 0.1307) / 0.3081  # reference normalisation (data.py:78-79)
            y = torch.from_numpy(_read_idx(lab).astype(np.int64))
            return TensorDataset(x, y)
    raise FileNotFoundError(f"MNIST idx files not found under {root}")


def load_cifar10(root: str, train: bool = True) -> TensorDataset:
    """CIFAR-10 binary batches (``cifar-10-batches-bin``); never unpickles anything."""
    d = Path(root) / "cifar-10-batches-bin"
    files = [d / f"data_batch_{i}.bin" for i in range(1, 6)] if train else [d / "test_batch.bin"]
    if not all(f.exists() for f in files):
        raise FileNotFoundError(f"CIFAR-10 binary batches not found under {d}")
    raw = np.concatenate([np.fromfile(f, dtype=np.uint8).reshape(-1, 3073) for f in files])
    y = torch.from_numpy(raw[:, 0].astype(np.int64))
    x = torch.from_numpy(raw[:, 1:].reshape(-1, 3, 32, 32).astype(np.float32) / 255.0)
    mean = torch.tensor([0.4914, 0.4822, 0.4465]).view(1, 3, 1, 1)
    std = torch.tensor([0.2470, 0.2435, 0.2616]).view(1, 3, 1, 1)
    return TensorDataset((x - mean) / std, y)


class ImageFolder(torch.utils.data.Dataset):
    """``root/<class>/<image>`` tree; Resize(256) -> CenterCrop(224) -> normalise (data.py:116-125)."""

    EXT = (".jpg", ".jpeg", ".png", ".bmp", ".ppm", ".webp")

    def __init__(self, root: str):
        self.root = Path(root)
        self.classes = sorted(p.name for p in self.root.iterdir() if p.is_dir())
        self.samples = [(str(f), ci) for ci, c in enumerate(self.classes) for f in sorted((self.root / c).rglob("*"))
                        if f.suffix.lower() in self.EXT]
        self.mean = torch.tensor([0.485, 0.456, 0.406]).view(3, 1, 1)
        self.std = torch.tensor([0.229, 0.224, 0.225]).view(3, 1, 1)

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, i):
        from PIL import Image

        path, label = self.samples[i]
        img = Image.open(path).convert("RGB")
        w, h = img.size
        s = 256 / min(w, h)
        img = img.resize((max(1, round(w * s)), max(1, round(h * s))), Image.BILINEAR)
        w, h = img.size
        left, top = (w - 224) // 2, (h - 224) // 2
        img = img.crop((left, top, left + 224, top + 224))
        x = torch.from_numpy(np.asarray(img, dtype=np.float32) / 255.0).permute(2, 0, 1)
        return (x - self.mean) / self.std, label


def load_dataset(kind: str, root: str):
    if kind == "mnist":
        return load_mnist(root)
    if kind == "cifar10":
        return load_cifar10(root)
    if kind == "imagenet":
        return ImageFolder(os.path.join(root, "ImageFolder"))
    raise ValueError(f"unknown dataset kind {kind!r}")


# ------------------------------------------------------------------------------------------------
# Synthetic batches
# ------------------------------------------------------------------------------------------------
class SyntheticBatches:
    """Uniform [0,1) images + uniform labels, generated on the training device every step.

    ``per_rank_seed``: by default each rank draws a different stream (seed + rank), which is what
    data parallelism actually sees; set ``identical=True`` to reproduce the reference, where every
    rank seeds 1234 and draws bit-identical batches.
    """

    def __init__(self, batch_size: int, shape: Tuple[int, int, int], num_classes: int, device,
                 dtype: torch.dtype = torch.float32, seed: int = 1234, rank: int = 0, identical: bool = False,
                 channels_last: bool = False, regenerate: bool = True, device_step: bool = False):
        self.batch_size = batch_size
        self.shape = tuple(shape)
        self.num_classes = num_classes
        self.device = torch.device(device)
        self.dtype = dtype
        self.seed = seed if identical else seed + 7919 * rank
        self.channels_last = channels_last and len(shape) == 3
        self.regenerate = regenerate
        self.step = 0
        n, (c, h, w) = batch_size, self.shape
        if self.channels_last:
            self._x = torch.empty((n, h, w, c), device=self.device, dtype=dtype).permute(0, 3, 1, 2)
        else:
            self._x = torch.empty((n, c, h, w), device=self.device, dtype=dtype)
        self._y = torch.empty((n,), device=self.device, dtype=torch.long)
        self._native = self.device.type == "cuda" and _ext.available()
        if self.device.type == "cuda" and not self._native:
            _ext.require()  # fail loudly on a GPU box without the extension
        # device_step: the stream position lives in a device counter advanced by a kernel, so the
        # generation can be captured in a HIP graph and still draw a new batch on every replay
        self._step_dev = (torch.zeros((1,), dtype=torch.long, device=self.device)
                          if device_step and self._native else None)
        self._fill()
        if self._step_dev is not None:
            self._step_dev.zero_()  # same stream positions as the host-stepped generator

    def _fill(self):
        if self._native:
            C = _ext.require()
            flat = self._x if not self.channels_last else self._x.permute(0, 2, 3, 1)
            per_x, per_y = (flat.numel() + 3) // 4, self.batch_size
            if self._step_dev is not None:
                C.uniform_(flat, self.seed, 0, 0.0, 1.0, self._step_dev, per_x)
                C.randint_(self._y, self.num_classes, self.seed, 0, self._step_dev, per_y)
                self._step_dev.add_(1)
            else:
                C.uniform_(flat, self.seed, self.step * per_x, 0.0, 1.0)
                C.randint_(self._y, self.num_classes, self.seed, self.step * per_y)
        else:
            # one generator per step position, so the stream is seekable (checkpoint resume)
            g = torch.Generator().manual_seed(self.seed + 1_000_003 * self.step)
            self._x.copy_(torch.rand(self._x.shape, generator=g).to(self.dtype))
            self._y.copy_(torch.randint(0, self.num_classes, self._y.shape, generator=g))

    def seek(self, step: int) -> None:
        """Continue the stream at batch ``step`` (a resumed run draws the batches it has not seen)."""
        self.step = int(step)
        if self._step_dev is not None:
            self._step_dev.fill_(self.step)

    def next(self) -> Tuple[torch.Tensor, torch.Tensor]:
        if self.regenerate:
            self._fill()
        self.step += 1
        return self._x, self._y

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        while True:
            yield self.next()


def random_data_generator(data_pair):
    """Reference-compatible generator (data.py:129-132): CPU tensors shaped like a template."""
    data, target = data_pair
    while True:
        yield torch.rand_like(data), torch.randint_like(target, high=int(target.max()) + 1)
