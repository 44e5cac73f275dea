"""Character corpus: vocabulary, encoding, TBPTT batching and offline sharding.

Behavioural parity with the reference data layer (C1-C5 of SURVEY.md §2.1):

* vocab = characters sorted by descending count, ties in first-occurrence order
  (``collections.Counter`` + stable sort, utils.py:7-17);
* ``TextLoader`` truncates to ``num_batches*B*T`` tokens, builds ``y = x`` shifted left with
  wrap-around ``y[-1] = x[0]`` and splits ``x.reshape(B, -1)`` along time into ``[B, T]``
  batches, so row ``b`` of batch ``k`` continues row ``b`` of batch ``k-1`` (utils.py:62-90) --
  the property that makes carrying the final RNN state across batches valid;
* the sharder builds the vocab over the full corpus and writes ``data-<i>.npy``
  (data_splitter.py:8-36).

Deliberate fixes: tokens are stored as int32 everywhere (A-9); a worker
given a ``tensor_file`` never overwrites it (A-6); sharding uses ``np.array_split`` so any
number of parts works (A-8), with ``exact=True`` reproducing ``np.split`` byte-for-byte.
"""
from __future__ import annotations

import codecs
import collections
import os
from typing import Dict, Optional, Sequence, Tuple

import numpy as np

from . import safe_pickle

# tinyshakespeare unigram statistics (data/tinyshakespeare/input.txt, 1,115,394 chars): used to
# generate Shakespeare-shaped synthetic corpora for benchmarks without touching the network.
SHAKESPEARE_CHARS = " etoahsrni\nldumy,wfcgIbp:.AvkT'EONRSLC;WUHMB?G!D-FYPKVjqxzJQZX3&$"
SHAKESPEARE_COUNTS = [
    169892, 94611, 67009, 65798, 55507, 51310, 49696, 48889, 48529, 45537, 40000, 33339, 31358,
    26584, 22243, 20448, 19846, 17585, 15770, 15623, 13356, 11832, 11321, 10808, 10316, 7885, 7819,
    7793, 7088, 7015, 6187, 6041, 5481, 5079, 4869, 4523, 3876, 3820, 3628, 3530, 3313, 3068, 2840,
    2761, 2462, 2399, 2172, 2089, 1897, 1797, 1718, 1641, 1584, 798, 628, 609, 529, 356, 320, 231,
    198, 112, 27, 3, 1]


def build_vocab(text: str) -> Tuple[Tuple[str, ...], Dict[str, int]]:
    counter = collections.Counter(text)
    pairs = sorted(counter.items(), key=lambda kv: -kv[1])  # stable: ties keep first occurrence
    chars = tuple(c for c, _ in pairs)
    return chars, {c: i for i, c in enumerate(chars)}


def read_text(path: str, encoding: str = "utf-8") -> str:
    with codecs.open(path, "r", encoding=encoding) as f:
        return f.read()


def encode(text: str, vocab: Dict[str, int]) -> np.ndarray:
    """Vectorised char -> id encoding (int32)."""
    if not text:
        return np.zeros(0, dtype=np.int32)
    cps = np.frombuffer(text.encode("utf-32-le"), dtype=np.uint32)
    max_cp = int(cps.max())
    table = np.full(max(max_cp + 1, 1), -1, dtype=np.int32)
    for ch, i in vocab.items():
        cp = ord(ch)
        if cp <= max_cp:
            table[cp] = i
    out = table[cps]
    if (out < 0).any():
        bad = {chr(int(c)) for c in cps[out < 0][:10]}
        raise KeyError(f"characters not in vocabulary: {sorted(bad)!r}")
    return out


def decode(ids: Sequence[int], chars: Sequence[str]) -> str:
    return "".join(chars[int(i)] for i in ids)


def create_vocab_file(input_file: str, vocab_file: str, encoding: str = "utf-8") -> dict:
    """Reference-compatible (utils.py:7-17): writes the pickled ``chars`` tuple."""
    data = read_text(input_file, encoding)
    chars, vocab = build_vocab(data)
    safe_pickle.dump(chars, vocab_file)
    return {"vocab": vocab, "chars": chars, "vocab_size": len(chars), "data": data}


def load_vocab_file(vocab_file: str) -> Tuple[Tuple[str, ...], Dict[str, int]]:
    chars = tuple(safe_pickle.load(vocab_file))
    return chars, {c: i for i, c in enumerate(chars)}


def make_batches(tensor: np.ndarray, batch_size: int, seq_length: int):
    """utils.py:62-82 semantics; returns (x_batches, y_batches, num_batches, truncated)."""
    num_batches = int(tensor.size // (batch_size * seq_length))
    if num_batches == 0:
        raise ValueError("Not enough data. Make seq_length and batch_size small.")
    t = np.ascontiguousarray(tensor[: num_batches * batch_size * seq_length]).astype(np.int32)
    x = t
    y = np.copy(t)
    y[:-1] = x[1:]
    y[-1] = x[0]
    xb = np.split(x.reshape(batch_size, -1), num_batches, 1)
    yb = np.split(y.reshape(batch_size, -1), num_batches, 1)
    return xb, yb, num_batches, t


class TextLoader:
    """Drop-in for the reference ``TextLoader`` (utils.py:19-90).

    Attributes: ``vocab_size``, ``chars``, ``vocab``, ``num_batches``, ``tensor``,
    ``x_batches``, ``y_batches``, ``pointer``; methods ``next_batch()``,
    ``reset_batch_pointer()``.
    """

    def __init__(self, data_dir: str, batch_size: int, seq_length: int, encoding: str = "utf-8",
                 tensor_file: Optional[str] = None, verbose: bool = True):
        self.data_dir = data_dir
        self.batch_size = batch_size
        self.seq_length = seq_length
        self.encoding = encoding
        input_file = os.path.join(data_dir, "input.txt")
        vocab_file = os.path.join(data_dir, "vocab.pkl")
        if tensor_file is not None:
            # worker shard: never (re)written here (fixes A-6)
            if not os.path.exists(tensor_file):
                raise FileNotFoundError(f"tensor file {tensor_file} does not exist "
                                        "(create shards with data_splitter.py)")
            if os.path.exists(vocab_file):
                self.chars, self.vocab = load_vocab_file(vocab_file)
            else:
                if verbose:
                    print("reading text file")
                res = create_vocab_file(input_file, vocab_file, encoding)
                self.chars, self.vocab = res["chars"], res["vocab"]
            if verbose:
                print("loading preprocessed files")
            self.tensor = np.load(tensor_file).astype(np.int32)
        else:
            tensor_file = os.path.join(data_dir, "data.npy")
            if not (os.path.exists(vocab_file) and os.path.exists(tensor_file)):
                if verbose:
                    print("reading text file")
                self.preprocess(input_file, vocab_file, tensor_file)
            else:
                if verbose:
                    print("loading preprocessed files")
                self.chars, self.vocab = load_vocab_file(vocab_file)
                self.tensor = np.load(tensor_file).astype(np.int32)
        self.vocab_size = len(self.chars)
        self.create_batches()
        self.reset_batch_pointer()

    def preprocess(self, input_file: str, vocab_file: str, tensor_file: str) -> None:
        res = create_vocab_file(input_file, vocab_file, encoding=self.encoding)
        self.chars, self.vocab = res["chars"], res["vocab"]
        self.tensor = encode(res["data"], self.vocab)
        np.save(tensor_file, self.tensor)

    def create_batches(self) -> None:
        self.x_batches, self.y_batches, self.num_batches, self.tensor = make_batches(
            self.tensor, self.batch_size, self.seq_length)

    def next_batch(self):
        x, y = self.x_batches[self.pointer], self.y_batches[self.pointer]
        self.pointer += 1
        return x, y

    def reset_batch_pointer(self) -> None:
        self.pointer = 0


class ArrayLoader(TextLoader):
    """A TextLoader over an in-memory token array (synthetic corpora, in-process shards)."""

    def __init__(self, tensor: np.ndarray, chars: Sequence[str], batch_size: int, seq_length: int):
        self.data_dir = None
        self.batch_size = batch_size
        self.seq_length = seq_length
        self.encoding = "utf-8"
        self.chars = tuple(chars)
        self.vocab = {c: i for i, c in enumerate(self.chars)}
        self.vocab_size = len(self.chars)
        self.tensor = np.asarray(tensor, dtype=np.int32)
        self.create_batches()
        self.reset_batch_pointer()


def shard(tensor: np.ndarray, num_parts: int, exact: bool = False):
    """Split a token array into ``num_parts`` contiguous shards.

    ``exact=True`` reproduces the reference's ``np.split`` (raises unless the length divides);
    the default ``np.array_split`` works for any part count (A-8).
    """
    if num_parts < 1:
        raise ValueError("num_parts must be >= 1")
    return np.split(tensor, num_parts) if exact else np.array_split(tensor, num_parts)


def synthetic_tokens(n: int, vocab_size: int = 65, seed: int = 0) -> np.ndarray:
    """Shakespeare-shaped synthetic token stream: ids drawn from the tinyshakespeare unigram
    distribution (for vocab_size > 65 the tail is filled with a Zipf-like decay)."""
    rng = np.random.default_rng(seed)
    counts = np.asarray(SHAKESPEARE_COUNTS[:vocab_size], dtype=np.float64)
    if vocab_size > len(counts):
        extra = 1.0 / np.arange(2, vocab_size - len(counts) + 2, dtype=np.float64)
        counts = np.concatenate([counts, extra * counts[-1]])
    p = counts / counts.sum()
    return rng.choice(vocab_size, size=n, p=p).astype(np.int32)


def synthetic_chars(vocab_size: int = 65) -> Tuple[str, ...]:
    if vocab_size <= len(SHAKESPEARE_CHARS):
        return tuple(SHAKESPEARE_CHARS[:vocab_size])
    extra = [chr(0x100 + i) for i in range(vocab_size - len(SHAKESPEARE_CHARS))]
    return tuple(SHAKESPEARE_CHARS) + tuple(extra)
