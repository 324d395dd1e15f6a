"""IMDB data module (reference ``data/imdb.py:1-126``, SURVEY #27).

Real mode reads ``<data_dir>/IMDB/aclImdb/{train,test}/{neg,pos}/*.txt`` (glob order, labels
neg=0 / pos=1) — the torchtext download the reference performs is not available offline, so
``prepare_data`` only checks that the directory exists.  A WordPiece tokenizer is trained and
saved to ``<data_dir>/imdb-tokenizer-<vocab>.json`` when missing (``Replace('<br />', ' ')``
+ NFD/Lowercase/StripAccents, like the reference).  Validation uses the IMDB *test* split.

Tokenizer: the reference ships its trained WordPiece tokenizer as
``.cache/imdb-tokenizer-10003.json`` (vocab 10003, [PAD]/[UNK]/[MASK] = 0/1/2; reference
``data/imdb.py:82,96-106`` loads it from ``<data_dir>`` or trains one).  The same vocabulary
ships here as package data (``data/assets/imdb-tokenizer-10003.json``, Apache-2.0, a data
artifact of the reference): a real-data run at vocab 10003 with no tokenizer in ``<data_dir>``
installs it there instead of training a new one, so default runs use the reference's token ids.
An existing ``<data_dir>/imdb-tokenizer-<vocab>.json`` or ``tokenizer_path=`` is loaded as is
and never retrained.

``synthetic=True`` generates token sequences of the same shape (and a matching tokenizer)
so every task runs without the dataset: ``synthetic_structure="topic"`` (default) mixes Zipf,
per-document topic and Markov-successor tokens (label = topic parity, so both MLM and
classifier have something to learn); ``"markov"`` / ``"unigram"`` are simpler variants.  ``pad_to_max=True`` pads every batch to
``max_seq_len`` instead of the longest sequence: padded positions are masked (keys) or never
selected (MLM), so results are identical, and static shapes let the step be graph-captured.
"""
from __future__ import annotations

import glob
import os
from typing import List, Optional

import torch

from ..utils.tokenizer import PAD_TOKEN, create_tokenizer, load_tokenizer, save_tokenizer, train_tokenizer
from .registry import register_datamodule
from .synthetic import SyntheticText

os.environ.setdefault("TOKENIZERS_PARALLELISM", "false")


def load_split(root: str, split: str):
    if split not in ("train", "test"):
        raise ValueError(f"invalid split: {split}")
    xs, ys = [], []
    for i, label in enumerate(["neg", "pos"]):
        for name in glob.glob(os.path.join(root, f"IMDB/aclImdb/{split}/{label}", "*.txt")):
            with open(name, encoding="utf-8") as f:
                xs.append(f.read())
                ys.append(i)
    return xs, ys


class IMDBDataset(torch.utils.data.Dataset):
    def __init__(self, root: str, split: str):
        self.raw_x, self.raw_y = load_split(root, split)

    def __len__(self):
        return len(self.raw_x)

    def __getitem__(self, i):
        return self.raw_y[i], self.raw_x[i]


class Collator:
    def __init__(self, tokenizer, max_seq_len: int, pad_to_max: bool = False):
        self.pad_id = tokenizer.token_to_id(PAD_TOKEN)
        self.tokenizer = tokenizer
        self.max_seq_len = max_seq_len
        if pad_to_max:
            tokenizer.enable_padding(pad_id=self.pad_id, pad_token=PAD_TOKEN, length=max_seq_len)
        else:
            tokenizer.enable_padding(pad_id=self.pad_id, pad_token=PAD_TOKEN)
        tokenizer.enable_truncation(max_length=max_seq_len)

    def collate(self, batch):
        ys, xs = zip(*batch)
        ids = torch.tensor([e.ids for e in self.tokenizer.encode_batch(list(xs))])
        return torch.tensor(ys), ids, ids == self.pad_id

    def encode(self, samples: List[str]):
        return self.collate([(0, s) for s in samples])[1:]


def shipped_tokenizer(vocab_size: int = 10003) -> str:
    """Path of the packaged reference tokenizer for ``vocab_size`` (exists for 10003 only)."""
    return os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets", f"imdb-tokenizer-{vocab_size}.json")


@register_datamodule
class IMDBDataModule:
    def __init__(self, data_dir: str = ".cache", vocab_size: int = 10003, max_seq_len: int = 512, batch_size: int = 64,
                 num_workers: int = 3, pin_memory: bool = False, synthetic: bool = False, synthetic_size: int = 25000,
                 pad_to_max: bool = False, seed: int = 0, synthetic_structure: str = "topic",
                 tokenizer_path: Optional[str] = None):
        self.hparams = dict(data_dir=data_dir, vocab_size=vocab_size, max_seq_len=max_seq_len, batch_size=batch_size,
                            num_workers=num_workers, pin_memory=pin_memory, synthetic=synthetic,
                            synthetic_size=synthetic_size, pad_to_max=pad_to_max, seed=seed,
                            synthetic_structure=synthetic_structure, tokenizer_path=tokenizer_path)
        self.data_dir = data_dir
        self.vocab_size = vocab_size
        self.max_seq_len = max_seq_len
        self.batch_size = batch_size
        self.num_workers = num_workers
        self.pin_memory = pin_memory
        self.synthetic = synthetic
        self.synthetic_size = synthetic_size
        self.pad_to_max = pad_to_max
        self.seed = seed
        self.synthetic_structure = synthetic_structure
        tag = "synthetic-" if synthetic else ""
        self.user_tokenizer = tokenizer_path is not None
        self.tokenizer_path = tokenizer_path or os.path.join(data_dir, f"imdb-{tag}tokenizer-{vocab_size}.json")
        self.tokenizer = None
        self.collator = None
        self.ds_train = self.ds_valid = None

    def _synthetic(self, split: str):
        n = self.synthetic_size if split == "train" else max(64, self.synthetic_size // 10)
        return SyntheticText(n, self.vocab_size, max(8, self.max_seq_len // 4), self.max_seq_len,
                             seed=self.seed + (0 if split == "train" else 1), structure=self.synthetic_structure)

    def prepare_data(self):
        if not self.synthetic and not os.path.isdir(os.path.join(self.data_dir, "IMDB", "aclImdb")):
            raise FileNotFoundError(
                f"IMDB not found under {self.data_dir}/IMDB/aclImdb (no network access to download it); "
                "place the extracted aclImdb directory there or use --data.synthetic=true")
        if self.user_tokenizer and not os.path.exists(self.tokenizer_path):
            raise FileNotFoundError(f"tokenizer_path={self.tokenizer_path} does not exist")
        if not os.path.exists(self.tokenizer_path):
            os.makedirs(self.data_dir, exist_ok=True)
            if not self.synthetic and os.path.exists(shipped_tokenizer(self.vocab_size)):
                import shutil

                shutil.copyfile(shipped_tokenizer(self.vocab_size), self.tokenizer_path)  # the reference vocabulary
                return
            if self.synthetic:
                ds = self._synthetic("train")
                text = (ds[i][1] for i in range(min(len(ds), 2000)))
                tok = create_tokenizer()
            else:
                from tokenizers.normalizers import Replace

                text, _ = load_split(self.data_dir, "train")
                tok = create_tokenizer(Replace("<br />", " "))
            train_tokenizer(tok, data=text, vocab_size=self.vocab_size)
            save_tokenizer(tok, self.tokenizer_path)

    def setup(self, stage: Optional[str] = None):
        self.tokenizer = load_tokenizer(self.tokenizer_path)
        if self.tokenizer.get_vocab_size() > self.vocab_size:  # ids past the embedding table
            raise ValueError(f"{self.tokenizer_path} has {self.tokenizer.get_vocab_size()} tokens, more than "
                             f"vocab_size={self.vocab_size}")
        self.collator = Collator(self.tokenizer, self.max_seq_len, pad_to_max=self.pad_to_max)
        if self.synthetic:
            self.ds_train, self.ds_valid = self._synthetic("train"), self._synthetic("test")
        else:
            self.ds_train = IMDBDataset(self.data_dir, "train")
            self.ds_valid = IMDBDataset(self.data_dir, "test")

    def _dl(self, ds, shuffle):
        return torch.utils.data.DataLoader(ds, batch_size=self.batch_size, shuffle=shuffle,
                                           collate_fn=self.collator.collate, num_workers=self.num_workers,
                                           pin_memory=self.pin_memory, persistent_workers=self.num_workers > 0)

    def train_dataloader(self):
        return self._dl(self.ds_train, True)

    def val_dataloader(self):
        return self._dl(self.ds_valid, False)

    def test_dataloader(self):
        return self._dl(self.ds_valid, False)
