"""WordPiece tokenizer helpers (host-side data prep).

Parity: reference ``perceiver/tokenizer.py:1-40`` — same special tokens/ids
(PAD=0, UNK=1, MASK=2), same normalizer chain (extra normalizers, then
NFD → Lowercase → StripAccents), Whitespace pre-tokenizer and WordPiece
decoder, and the same JSON on-disk format (HF ``tokenizers``).  Tokenization
is CPU work feeding the GPU step; it is not a kernel target.
"""
from __future__ import annotations

from typing import Iterable

PAD_TOKEN = "[PAD]"
PAD_TOKEN_ID = 0
UNK_TOKEN = "[UNK]"
UNK_TOKEN_ID = 1
MASK_TOKEN = "[MASK]"
MASK_TOKEN_ID = 2

SPECIAL_TOKENS = [PAD_TOKEN, UNK_TOKEN, MASK_TOKEN]


def _tk():
    import tokenizers  # imported lazily: only the data path needs it

    return tokenizers


def create_tokenizer(*normalizers):
    tk = _tk()
    from tokenizers.models import WordPiece
    from tokenizers.normalizers import NFD, Lowercase, StripAccents, Sequence
    from tokenizers.pre_tokenizers import Whitespace

    tok = tk.Tokenizer(WordPiece(unk_token=UNK_TOKEN))
    tok.normalizer = Sequence(list(normalizers) + [NFD(), Lowercase(), StripAccents()])
    tok.pre_tokenizer = Whitespace()
    tok.decoder = tk.decoders.WordPiece()
    return tok


def train_tokenizer(tokenizer, data: Iterable[str], vocab_size: int):
    from tokenizers.trainers import WordPieceTrainer

    tokenizer.train_from_iterator(data, WordPieceTrainer(vocab_size=vocab_size, special_tokens=SPECIAL_TOKENS))


def save_tokenizer(tokenizer, path: str):
    tokenizer.save(path)


def load_tokenizer(path: str):
    return _tk().Tokenizer.from_file(path)
