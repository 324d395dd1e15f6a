"""MNIST data module (reference ``data/mnist.py:1-55``, SURVEY #28).

Reads the standard IDX files (``train-images-idx3-ubyte[.gz]`` …) from ``<data_dir>/MNIST/raw``
or ``<data_dir>``; no download (offline).  ``synthetic=True`` (or ``synthetic='auto'`` with the
files absent) generates class-structured 28×28 images.  Transforms as the reference:
[RandomCrop], scale to [0, 1], Normalize(0.5, 0.5), channels-last.  The train split holds
out ``val_split`` images for validation (pl_bolts semantics), the test split is MNIST test.
Defect D7 fixed: ``image_shape`` reflects ``random_crop``.
"""
from __future__ import annotations

import gzip
import os
import struct
from typing import Optional, Union

import torch

from .registry import register_datamodule
from .synthetic import SyntheticImages


def _read_idx(path: str) -> torch.Tensor:
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rb") as f:
        data = f.read()
    magic = struct.unpack(">I", data[:4])[0]
    nd = magic & 0xFF
    dims = struct.unpack(">" + "I" * nd, data[4:4 + 4 * nd])
    return torch.frombuffer(bytearray(data[4 + 4 * nd:]), dtype=torch.uint8).reshape(dims)


def _find(root: str, stem: str) -> Optional[str]:
    for d in (os.path.join(root, "MNIST", "raw"), root):
        for ext in ("", ".gz"):
            p = os.path.join(d, stem + ext)
            if os.path.exists(p):
                return p
    return None


class _Transformed(torch.utils.data.Dataset):
    def __init__(self, images: torch.Tensor, labels: torch.Tensor, crop: Optional[int], normalize: bool,
                 channels_last: bool, train: bool):
        self.images, self.labels = images, labels
        self.crop, self.normalize, self.cl, self.train = crop, normalize, channels_last, train

    def __len__(self):
        return len(self.labels)

    def __getitem__(self, i):
        x = self.images[i].float() / 255.0  # (H, W)
        if self.crop:
            h, w = x.shape
            if self.train:
                top = int(torch.randint(0, h - self.crop + 1, (1,)))
                left = int(torch.randint(0, w - self.crop + 1, (1,)))
            else:
                top, left = (h - self.crop) // 2, (w - self.crop) // 2
            x = x[top:top + self.crop, left:left + self.crop]
        if self.normalize:
            x = (x - 0.5) / 0.5
        x = x.unsqueeze(-1) if self.cl else x.unsqueeze(0)
        return x, int(self.labels[i])


@register_datamodule
class MNISTDataModule:
    name = "mnist"

    def __init__(self, channels_last: bool = True, random_crop: Optional[int] = None, data_dir: Optional[str] = ".cache",
                 val_split: Union[int, float] = 10000, num_workers: int = 3, normalize: bool = True, pin_memory: bool = False,
                 batch_size: int = 32, seed: int = 42, shuffle: bool = True, drop_last: bool = False,
                 synthetic: Union[bool, str] = "auto", synthetic_size: int = 60000):
        self.hparams = dict(channels_last=channels_last, random_crop=random_crop, data_dir=data_dir, val_split=val_split,
                            num_workers=num_workers, normalize=normalize, pin_memory=pin_memory, batch_size=batch_size,
                            seed=seed, synthetic=synthetic)
        self.channels_last, self.random_crop = channels_last, random_crop
        self.data_dir = data_dir or "."
        self.val_split, self.num_workers, self.normalize = val_split, num_workers, normalize
        self.pin_memory, self.batch_size, self.seed = pin_memory, batch_size, seed
        self.shuffle, self.drop_last = shuffle, drop_last
        self.synthetic, self.synthetic_size = synthetic, synthetic_size
        self.num_classes = 10
        side = random_crop or 28
        self._image_shape = (side, side, 1) if channels_last else (1, side, side)
        self.ds_train = self.ds_val = self.ds_test = None

    @property
    def image_shape(self):
        return self._image_shape

    @property
    def dims(self):
        return (1, self._image_shape[0], self._image_shape[1]) if self.channels_last else self._image_shape

    def _use_synthetic(self) -> bool:
        if self.synthetic == "auto":
            return _find(self.data_dir, "train-images-idx3-ubyte") is None
        return bool(self.synthetic)

    def prepare_data(self):
        if not self._use_synthetic() and _find(self.data_dir, "train-images-idx3-ubyte") is None:
            raise FileNotFoundError(f"MNIST IDX files not found under {self.data_dir} (offline; use --data.synthetic=true)")

    def setup(self, stage: Optional[str] = None):
        if self._use_synthetic():
            n = self.synthetic_size
            full = SyntheticImages(n, (28, 28, 1), 10, seed=self.seed)
            imgs = torch.stack([((full[i][0][..., 0] * 0.5 + 0.5) * 255).round().to(torch.uint8) for i in range(n)])
            labs = torch.tensor([full[i][1] for i in range(n)])
            timgs, tlabs = imgs[: max(1, n // 6)], labs[: max(1, n // 6)]
        else:
            imgs = _read_idx(_find(self.data_dir, "train-images-idx3-ubyte"))
            labs = _read_idx(_find(self.data_dir, "train-labels-idx1-ubyte")).long()
            timgs = _read_idx(_find(self.data_dir, "t10k-images-idx3-ubyte"))
            tlabs = _read_idx(_find(self.data_dir, "t10k-labels-idx1-ubyte")).long()
        n = len(labs)
        nval = int(self.val_split * n) if isinstance(self.val_split, float) else min(int(self.val_split), n // 2)
        g = torch.Generator().manual_seed(self.seed)
        perm = torch.randperm(n, generator=g)
        tr, va = perm[: n - nval], perm[n - nval:]
        mk = lambda i, l, train: _Transformed(i, l, self.random_crop, self.normalize, self.channels_last, train)
        self.ds_train = mk(imgs[tr], labs[tr], True)
        self.ds_val = mk(imgs[va], labs[va], False)
        self.ds_test = mk(timgs, tlabs, False)

    def _dl(self, ds, shuffle):
        return torch.utils.data.DataLoader(ds, batch_size=self.batch_size, shuffle=shuffle, num_workers=self.num_workers,
                                           pin_memory=self.pin_memory, drop_last=self.drop_last,
                                           persistent_workers=self.num_workers > 0)

    def train_dataloader(self):
        return self._dl(self.ds_train, self.shuffle)

    def val_dataloader(self):
        return self._dl(self.ds_val, False)

    def test_dataloader(self):
        return self._dl(self.ds_test, False)


@register_datamodule
class SyntheticImageDataModule:
    """ImageNet-shape (224×224×3 by default) synthetic classification data (BASELINE config 4)."""

    def __init__(self, image_shape=(224, 224, 3), num_classes: int = 1000, size: int = 10000, batch_size: int = 32,
                 num_workers: int = 2, pin_memory: bool = False, seed: int = 0):
        self.hparams = dict(image_shape=list(image_shape), num_classes=num_classes, size=size, batch_size=batch_size)
        self._image_shape = tuple(image_shape)
        self.num_classes = num_classes
        self.size, self.batch_size, self.num_workers, self.pin_memory, self.seed = size, batch_size, num_workers, pin_memory, seed

    @property
    def image_shape(self):
        return self._image_shape

    def prepare_data(self):
        pass

    def setup(self, stage=None):
        self.ds_train = SyntheticImages(self.size, self._image_shape, self.num_classes, seed=self.seed)
        self.ds_val = SyntheticImages(max(64, self.size // 10), self._image_shape, self.num_classes, seed=self.seed + 1)

    def _dl(self, ds, shuffle):
        return torch.utils.data.DataLoader(ds, batch_size=self.batch_size, shuffle=shuffle, num_workers=self.num_workers,
                                           pin_memory=self.pin_memory)

    def train_dataloader(self):
        return self._dl(self.ds_train, True)

    def val_dataloader(self):
        return self._dl(self.ds_val, False)

    def test_dataloader(self):
        return self._dl(self.ds_val, False)
