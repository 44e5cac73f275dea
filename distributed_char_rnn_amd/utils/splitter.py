"""Offline corpus sharding CLI (reference: data_splitter.py:8-36).

Builds the vocabulary over the FULL corpus (shared by every worker, README.md:19), encodes it and
writes ``<out_dir>/data-<i>.npy``.  ``np.array_split`` is used so 4 or 8 workers work on
tinyshakespeare (the reference's ``np.split`` raises unless the length divides, A-8); with an
exact division the shards are identical to the reference's (``--exact`` enforces that mode).
Shards are int32 (the checked-in reference shards are int32 too).
"""
from __future__ import annotations

import os
import sys

import numpy as np

from . import data as data_mod
from .config import splitter_parser


def split_corpus(data_dir: str, num_parts: int, out_dir: str = "sharded_data",
                 exact: bool = False, verbose: bool = True):
    inp = os.path.join(data_dir, "input.txt")
    vocab_file = os.path.join(data_dir, "vocab.pkl")
    os.makedirs(out_dir, exist_ok=True)
    if verbose:
        print("building vocabulary...")
    res = data_mod.create_vocab_file(inp, vocab_file)
    if verbose:
        print("sharding file...")
    tensor = data_mod.encode(res["data"], res["vocab"])
    parts = data_mod.shard(tensor, num_parts, exact=exact)
    paths = []
    for i, t in enumerate(parts):
        if verbose:
            print("writing shard %d.." % i, end="\r")
        p = os.path.join(out_dir, "data-%d.npy" % i)
        np.save(p, t.astype(np.int32))
        paths.append(p)
    if verbose:
        print("\ndone")
    return paths


def main(argv=None) -> int:
    a = splitter_parser().parse_args(argv)
    split_corpus(a.data_dir, a.num_parts, a.out_dir, exact=a.exact)
    return 0


if __name__ == "__main__":
    sys.exit(main())
