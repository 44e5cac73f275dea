"""Checkpoint directory layout compatible with the reference's ``save_dir``.

Reference artefacts (train.py:109-115, 145, 209-217; TF Saver V2 [TF-ext]):

* ``config.pkl``       pickled ``argparse.Namespace`` of all flags (+ ``vocab_size``)
* ``chars_vocab.pkl``  pickled ``(chars, vocab)``
* ``checkpoint``       text index: ``model_checkpoint_path: "model.ckpt-N"`` +
                       ``all_model_checkpoint_paths: ...`` lines (max_to_keep = 5)
* ``model.ckpt-N.index`` / ``model.ckpt-N.data-00000-of-00001`` per saved step.

We keep every filename and the TF variable names/layouts (``rnnlm/multi_rnn_cell/cell_l/
lstm_cell/kernel`` [D+H, 4H] in i,j,f,o order, ``<var>/Adam``, ``<var>/Adam_1``,
``beta1_power``, ``beta2_power``, ``global_step``, ``Variable`` = the lr variable), and the
bundle itself is TF's V2 tensor-bundle format (``utils/tf_bundle.py``: SSTable ``.index`` of
BundleEntryProtos + raw ``.data`` shard), so checkpoints move both ways between this framework
and a TF 1.x run of the reference (decision recorded in SURVEY.md §5.4).  ``DCR_CKPT_FORMAT=json``
writes the older self-describing JSON container instead (``.index`` = JSON name ->
dtype/shape/offset/crc32); reading detects either.  Nothing in a bundle is pickled, so loading
executes nothing.  Extra entries (``dcr/epoch``, ``dcr/batch_pointer``, optional TBPTT state)
make resume exact; TF ignores keys it has no variable for.
"""
from __future__ import annotations

import json
import os
import re
import zlib
from typing import Dict, List, Optional

import numpy as np
import torch

from . import tf_bundle

FORMAT = "dcr-bundle-v1"
_DT = {"float32": np.float32, "float64": np.float64, "int64": np.int64, "int32": np.int32,
       "float16": np.float16, "uint16": np.uint16}


def _to_numpy(t) -> np.ndarray:
    if isinstance(t, torch.Tensor):
        t = t.detach().cpu()
        if t.dtype == torch.bfloat16:
            t = t.float()
        return t.numpy()
    return np.asarray(t)


def write_bundle(prefix: str, tensors: Dict[str, object], fmt: Optional[str] = None) -> None:
    fmt = fmt or os.environ.get("DCR_CKPT_FORMAT", "tf")
    if fmt == "tf":
        tf_bundle.write_bundle(prefix, {k: _to_numpy(v) for k, v in tensors.items()})
        return
    index = {"format": FORMAT, "tensors": {}}
    data_path = prefix + ".data-00000-of-00001"
    tmp = data_path + ".tmp"
    off = 0
    with open(tmp, "wb") as f:
        for name in sorted(tensors):
            a = np.require(_to_numpy(tensors[name]), requirements="C")  # keeps 0-d scalars
            if a.dtype.name not in _DT:
                a = a.astype(np.float32)
            b = a.astype(a.dtype.newbyteorder("<"), copy=False).tobytes()
            pad = (-off) % 64
            if pad:
                f.write(b"\0" * pad)
                off += pad
            f.write(b)
            index["tensors"][name] = {"dtype": a.dtype.name, "shape": list(a.shape),
                                      "offset": off, "nbytes": len(b),
                                      "crc32": zlib.crc32(b) & 0xFFFFFFFF}
            off += len(b)
    os.replace(tmp, data_path)
    itmp = prefix + ".index.tmp"
    with open(itmp, "w") as f:
        json.dump(index, f, indent=1, sort_keys=True)
    os.replace(itmp, prefix + ".index")


def read_bundle(prefix: str, verify: bool = True) -> Dict[str, np.ndarray]:
    if tf_bundle.is_tf_bundle(prefix):
        return tf_bundle.read_bundle(prefix, verify)
    with open(prefix + ".index") as f:
        index = json.load(f)
    if index.get("format") != FORMAT:
        raise ValueError(f"{prefix}.index: unknown checkpoint format {index.get('format')!r}")
    out = {}
    with open(prefix + ".data-00000-of-00001", "rb") as f:
        for name, e in index["tensors"].items():
            f.seek(e["offset"])
            b = f.read(e["nbytes"])
            if verify and (zlib.crc32(b) & 0xFFFFFFFF) != e["crc32"]:
                raise IOError(f"checksum mismatch for {name} in {prefix}")
            out[name] = np.frombuffer(b, dtype=np.dtype(_DT[e["dtype"]]).newbyteorder("<")) \
                .reshape(e["shape"]).copy()
    return out


def _state_file(save_dir: str) -> str:
    return os.path.join(save_dir, "checkpoint")


def get_checkpoint_state(save_dir: str) -> Optional[dict]:
    """Parses the TF-style ``checkpoint`` text file; paths are resolved relative to save_dir."""
    p = _state_file(save_dir)
    if not os.path.exists(p):
        return None
    model, allp = None, []
    with open(p) as f:
        for line in f:
            m = re.match(r'\s*(model_checkpoint_path|all_model_checkpoint_paths):\s*"(.*)"', line)
            if not m:
                continue
            path = m.group(2)
            if not os.path.isabs(path):
                path = os.path.join(save_dir, path)
            if m.group(1) == "model_checkpoint_path":
                model = path
            else:
                allp.append(path)
    if model is None:
        return None
    return {"model_checkpoint_path": model, "all_model_checkpoint_paths": allp}


def latest_checkpoint(save_dir: str) -> Optional[str]:
    st = get_checkpoint_state(save_dir)
    if st and os.path.exists(st["model_checkpoint_path"] + ".index"):
        return st["model_checkpoint_path"]
    # fall back to scanning (e.g. a hand-copied directory without the index file)
    best = None
    if os.path.isdir(save_dir):
        for fn in os.listdir(save_dir):
            m = re.match(r"model\.ckpt-(\d+)\.index$", fn)
            if m and (best is None or int(m.group(1)) > best[0]):
                best = (int(m.group(1)), os.path.join(save_dir, fn[: -len(".index")]))
    return best[1] if best else None


class Saver:
    """``tf.train.Saver(max_to_keep=5)`` equivalent for our bundle format."""

    def __init__(self, max_to_keep: int = 5):
        self.max_to_keep = max_to_keep

    def save(self, save_dir: str, tensors: Dict[str, object], global_step: int,
             basename: str = "model.ckpt") -> str:
        os.makedirs(save_dir, exist_ok=True)
        prefix = os.path.join(save_dir, f"{basename}-{int(global_step)}")
        write_bundle(prefix, tensors)
        st = get_checkpoint_state(save_dir) or {"all_model_checkpoint_paths": []}
        paths: List[str] = [p for p in st["all_model_checkpoint_paths"]
                            if os.path.abspath(p) != os.path.abspath(prefix)]
        paths.append(prefix)
        while self.max_to_keep and len(paths) > self.max_to_keep:
            old = paths.pop(0)
            for suf in (".index", ".data-00000-of-00001"):
                try:
                    os.remove(old + suf)
                except FileNotFoundError:
                    pass
        rel = lambda p: os.path.relpath(p, save_dir)  # noqa: E731
        tmp = _state_file(save_dir) + ".tmp"
        with open(tmp, "w") as f:
            f.write(f'model_checkpoint_path: "{rel(prefix)}"\n')
            for p in paths:
                f.write(f'all_model_checkpoint_paths: "{rel(p)}"\n')
        os.replace(tmp, _state_file(save_dir))
        return prefix

    @staticmethod
    def restore(prefix: str) -> Dict[str, np.ndarray]:
        return read_bundle(prefix)
