"""Minimal TensorBoard event-file writer (no TensorFlow / tensorboard dependency).

The reference writes ``tf.summary`` scalars (``train_loss``) and histograms (``logits``,
``loss``) to ``log_dir/<YYYY-mm-dd-HH-MM-SS>`` (model.py:100-103, train.py:140-143, 199-202).
This module emits the same kind of file: TFRecord framing (length + masked CRC32C) of
``tensorflow.Event`` protos hand-encoded in protobuf wire format, readable by
``tensorboard --logdir``.
"""
from __future__ import annotations

import os
import socket
import struct
import time
from typing import Optional

import numpy as np

# ---------------------------------------------------------------- CRC32C (Castagnoli)
_POLY = 0x82F63B78
_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ _POLY if _c & 1 else _c >> 1
    _TABLE.append(_c)


def crc32c(data: bytes) -> int:
    crc = 0xFFFFFFFF
    t = _TABLE
    for b in data:
        crc = t[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def masked_crc(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


# ---------------------------------------------------------------- protobuf wire helpers
def _varint(v: int) -> bytes:
    out = bytearray()
    v &= (1 << 64) - 1
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field: int, wt: int) -> bytes:
    return _varint((field << 3) | wt)


def _ld(field: int, payload: bytes) -> bytes:
    return _key(field, 2) + _varint(len(payload)) + payload


def _double(field: int, v: float) -> bytes:
    return _key(field, 1) + struct.pack("<d", float(v))


def _float(field: int, v: float) -> bytes:
    return _key(field, 5) + struct.pack("<f", float(v))


def _packed_doubles(field: int, vs) -> bytes:
    return _ld(field, b"".join(struct.pack("<d", float(x)) for x in vs))


def _event(step: int, summary: Optional[bytes] = None, file_version: Optional[str] = None,
           wall_time: Optional[float] = None) -> bytes:
    ev = _double(1, time.time() if wall_time is None else wall_time) + _key(2, 0) + _varint(step)
    if file_version is not None:
        ev += _ld(3, file_version.encode())
    if summary is not None:
        ev += _ld(5, summary)
    return ev


def _histo(values: np.ndarray, bins: int = 30) -> bytes:
    v = np.asarray(values, dtype=np.float64).ravel()
    if v.size == 0:
        v = np.zeros(1)
    lo, hi = float(v.min()), float(v.max())
    if hi <= lo:
        hi = lo + 1e-6
    counts, edges = np.histogram(v, bins=bins, range=(lo, hi))
    return (_double(1, lo) + _double(2, hi) + _double(3, v.size) + _double(4, v.sum())
            + _double(5, float((v * v).sum())) + _packed_doubles(6, edges[1:])
            + _packed_doubles(7, counts))


class EventWriter:
    def __init__(self, logdir: str):
        os.makedirs(logdir, exist_ok=True)
        fn = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}"
        self.path = os.path.join(logdir, fn)
        self._f = open(self.path, "wb")
        self._write(_event(0, file_version="brain.Event:2"))

    def _write(self, rec: bytes) -> None:
        hdr = struct.pack("<Q", len(rec))
        self._f.write(hdr + struct.pack("<I", masked_crc(hdr)) + rec
                      + struct.pack("<I", masked_crc(rec)))

    def scalar(self, tag: str, value: float, step: int) -> None:
        val = _ld(1, tag.encode()) + _float(2, value)
        self._write(_event(step, summary=_ld(1, val)))

    def histogram(self, tag: str, values, step: int) -> None:
        val = _ld(1, tag.encode()) + _ld(5, _histo(values))
        self._write(_event(step, summary=_ld(1, val)))

    def flush(self) -> None:
        self._f.flush()

    def close(self) -> None:
        if not self._f.closed:
            self._f.close()


def read_records(path: str):
    """Yield raw record payloads (used by tests to validate framing)."""
    with open(path, "rb") as f:
        while True:
            hdr = f.read(8)
            if len(hdr) < 8:
                return
            (n,) = struct.unpack("<Q", hdr)
            (hc,) = struct.unpack("<I", f.read(4))
            if hc != masked_crc(hdr):
                raise IOError("bad length crc")
            rec = f.read(n)
            (rc,) = struct.unpack("<I", f.read(4))
            if rc != masked_crc(rec):
                raise IOError("bad record crc")
            yield rec
