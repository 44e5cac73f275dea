"""TensorFlow V2 checkpoint bundle (``model.ckpt-N.index`` + ``.data-00000-of-00001``) writer
and reader, without TensorFlow.

The reference saves with ``tf.train.Saver`` (train.py:145, 209-217): TF's tensor-bundle format
[TF-ext].  Writing and reading that format here lets checkpoints move both ways between this
framework and a TF 1.x run of the reference: ``--init_from`` / ``sample.py`` accept a reference
``save_dir``, and ``tf.train.Saver.restore`` can read what ``train.py`` here writes (variable
names and layouts are TF's, models/params.py).

Format (TF ``core/util/tensor_bundle``, on-disk table = the LevelDB SSTable layout):

* ``.data-00000-of-00001``: the raw little-endian bytes of every tensor, back to back.
* ``.index``: an SSTable whose keys are tensor names (sorted bytewise) and whose values are
  serialized protos: key ``""`` -> ``BundleHeaderProto{num_shards=1, endianness=LITTLE,
  version{producer=1}}``; every other key -> ``BundleEntryProto{dtype, shape, shard_id=0,
  offset, size, crc32c (masked CRC-32C of the bytes)}``.
  SSTable = data blocks (prefix-compressed entries, a restart point every 16 entries, uint32
  restart array, block trailer = compression byte 0 + masked CRC-32C) + an empty metaindex
  block + an index block (last key of each data block -> BlockHandle) + a 48-byte footer
  (two BlockHandles, zero padding, magic 0xdb4775248b80fb57).

Protos are hand-encoded (field numbers from tensor_bundle.proto / tensor_shape.proto /
versions.proto); nothing in the file is executed when it is read.  Snappy-compressed blocks
(not used by TF bundles) are rejected.
"""
from __future__ import annotations

import os
import struct
from typing import Dict, Iterator, List, Tuple

import numpy as np

from .tfevents import crc32c, masked_crc

MAGIC = 0xDB4775248B80FB57
RESTART_INTERVAL = 16
BLOCK_SIZE = 4096
# tensorflow/core/framework/types.proto DataType
_NP2DT = {np.dtype(np.float32): 1, np.dtype(np.float64): 2, np.dtype(np.int32): 3,
          np.dtype(np.uint8): 4, np.dtype(np.int16): 5, np.dtype(np.int8): 6,
          np.dtype(np.int64): 9, np.dtype(np.bool_): 10, np.dtype(np.uint16): 17,
          np.dtype(np.float16): 19, np.dtype(np.uint32): 22, np.dtype(np.uint64): 23}
_DT2NP = {v: k for k, v in _NP2DT.items()}
DT_BFLOAT16 = 14


# ------------------------------------------------------------------------------ protobuf wire
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


def _read_varint(buf: bytes, pos: int) -> Tuple[int, int]:
    shift = v = 0
    while True:
        b = buf[pos]
        pos += 1
        v |= (b & 0x7F) << shift
        if not b & 0x80:
            return v, pos
        shift += 7
        if shift > 63:
            raise ValueError("varint too long")


def _field_varint(no: int, v: int) -> bytes:
    return _varint(no << 3) + _varint(v)


def _field_bytes(no: int, b: bytes) -> bytes:
    return _varint((no << 3) | 2) + _varint(len(b)) + b


def _field_fixed32(no: int, v: int) -> bytes:
    return _varint((no << 3) | 5) + struct.pack("<I", v & 0xFFFFFFFF)


def _parse(buf: bytes) -> Dict[int, list]:
    """Minimal protobuf parser: field number -> list of raw values (ints or bytes)."""
    out: Dict[int, list] = {}
    pos = 0
    while pos < len(buf):
        key, pos = _read_varint(buf, pos)
        no, wt = key >> 3, key & 7
        if wt == 0:
            v, pos = _read_varint(buf, pos)
        elif wt == 1:
            v = struct.unpack_from("<Q", buf, pos)[0]
            pos += 8
        elif wt == 2:
            n, pos = _read_varint(buf, pos)
            v = bytes(buf[pos: pos + n])
            pos += n
        elif wt == 5:
            v = struct.unpack_from("<I", buf, pos)[0]
            pos += 4
        else:
            raise ValueError(f"unsupported protobuf wire type {wt}")
        out.setdefault(no, []).append(v)
    return out


def _header_proto() -> bytes:
    # num_shards = 1; endianness = LITTLE (0, the proto3 default: not written);
    # version.producer = kTensorBundleVersion (1)
    return _field_varint(1, 1) + _field_bytes(3, _field_varint(1, 1))


def _entry_proto(dtype: int, shape, offset: int, size: int, crc: int) -> bytes:
    dims = b"".join(_field_bytes(2, _field_varint(1, int(d))) for d in shape)
    out = _field_varint(1, dtype) + _field_bytes(2, dims)
    # shard_id = 0 is the proto3 default and not written (TF omits it too)
    if offset:
        out += _field_varint(4, offset)
    out += _field_varint(5, size) + _field_fixed32(6, crc)
    return out


def _masked(c: int) -> int:
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def _unmask(m: int) -> int:
    r = (m - 0xA282EAD8) & 0xFFFFFFFF
    return ((r >> 17) | (r << 15)) & 0xFFFFFFFF


# ------------------------------------------------------------------------------ SSTable
class _BlockBuilder:
    def __init__(self):
        self.buf = bytearray()
        self.restarts = [0]
        self.count = 0
        self.last = b""

    def add(self, key: bytes, value: bytes):
        shared = 0
        if self.count < RESTART_INTERVAL:
            n = min(len(self.last), len(key))
            while shared < n and self.last[shared] == key[shared]:
                shared += 1
        else:
            self.restarts.append(len(self.buf))
            self.count = 0
        self.buf += _varint(shared) + _varint(len(key) - shared) + _varint(len(value))
        self.buf += key[shared:] + value
        self.last = key
        self.count += 1

    def finish(self) -> bytes:
        return bytes(self.buf) + b"".join(struct.pack("<I", r) for r in self.restarts) + \
            struct.pack("<I", len(self.restarts))

    def size(self) -> int:
        return len(self.buf) + 4 * len(self.restarts) + 4


def _write_block(f, contents: bytes) -> Tuple[int, int]:
    off = f.tell()
    f.write(contents)
    trailer = b"\x00"  # kNoCompression
    f.write(trailer + struct.pack("<I", masked_crc(contents + trailer)))
    return off, len(contents)


def _handle(off: int, size: int) -> bytes:
    return _varint(off) + _varint(size)


def write_table(path: str, items: List[Tuple[bytes, bytes]]) -> None:
    """Write sorted (key, value) pairs as an uncompressed SSTable."""
    keys = [k for k, _ in items]
    if keys != sorted(keys) or len(set(keys)) != len(keys):
        raise ValueError("SSTable keys must be unique and sorted")
    with open(path, "wb") as f:
        index = _BlockBuilder()
        block = _BlockBuilder()
        for k, v in items:
            block.add(k, v)
            if block.size() >= BLOCK_SIZE:
                off, n = _write_block(f, block.finish())
                index.add(block.last, _handle(off, n))
                block = _BlockBuilder()
        if block.count or not items:
            off, n = _write_block(f, block.finish())
            index.add(block.last, _handle(off, n))
        meta_off, meta_n = _write_block(f, _BlockBuilder().finish())
        idx_off, idx_n = _write_block(f, index.finish())
        footer = _handle(meta_off, meta_n) + _handle(idx_off, idx_n)
        footer += b"\x00" * (40 - len(footer)) + struct.pack("<Q", MAGIC)
        f.write(footer)


def _read_block(data: bytes, off: int, size: int, verify: bool) -> bytes:
    contents = data[off: off + size]
    ctype = data[off + size]
    if verify:
        want = struct.unpack_from("<I", data, off + size + 1)[0]
        if _unmask(want) != crc32c(contents + bytes([ctype])):
            raise IOError("SSTable block checksum mismatch")
    if ctype != 0:
        raise ValueError(f"compressed SSTable block (type {ctype}) is not supported")
    return contents


def _block_entries(block: bytes) -> Iterator[Tuple[bytes, bytes]]:
    nrest = struct.unpack_from("<I", block, len(block) - 4)[0]
    end = len(block) - 4 - 4 * nrest
    pos, last = 0, b""
    while pos < end:
        shared, pos = _read_varint(block, pos)
        nonshared, pos = _read_varint(block, pos)
        vlen, pos = _read_varint(block, pos)
        key = last[:shared] + block[pos: pos + nonshared]
        pos += nonshared
        yield key, block[pos: pos + vlen]
        pos += vlen
        last = key


def read_table(path: str, verify: bool = True) -> List[Tuple[bytes, bytes]]:
    with open(path, "rb") as f:
        data = f.read()
    if len(data) < 48 or struct.unpack_from("<Q", data, len(data) - 8)[0] != MAGIC:
        raise ValueError(f"{path}: not an SSTable (bad magic)")
    footer = data[-48:-8]
    pos = 0
    _, pos = _read_varint(footer, pos)  # metaindex handle (unused)
    _, pos = _read_varint(footer, pos)
    idx_off, pos = _read_varint(footer, pos)
    idx_n, pos = _read_varint(footer, pos)
    out = []
    for _, h in _block_entries(_read_block(data, idx_off, idx_n, verify)):
        off, p = _read_varint(h, 0)
        n, _ = _read_varint(h, p)
        out.extend(_block_entries(_read_block(data, off, n, verify)))
    return out


# ------------------------------------------------------------------------------ bundles
def is_tf_bundle(prefix: str) -> bool:
    try:
        with open(prefix + ".index", "rb") as f:
            f.seek(-8, os.SEEK_END)
            return struct.unpack("<Q", f.read(8))[0] == MAGIC
    except (OSError, struct.error):
        return False


def write_bundle(prefix: str, tensors: Dict[str, np.ndarray]) -> None:
    """Write ``tensors`` (name -> numpy array) as a TF V2 bundle (one data shard)."""
    data_path = prefix + ".data-00000-of-00001"
    entries = []
    off = 0
    with open(data_path + ".tmp", "wb") as f:
        for name in sorted(tensors, key=lambda s: s.encode()):
            a = np.require(np.asarray(tensors[name]), requirements="C")
            if a.dtype not in _NP2DT:
                a = a.astype(np.float32)
            b = a.astype(a.dtype.newbyteorder("<"), copy=False).tobytes()
            f.write(b)
            entries.append((name.encode(), _entry_proto(_NP2DT[a.dtype], a.shape, off, len(b),
                                                        _masked(crc32c(b)))))
            off += len(b)
    items = [(b"", _header_proto())] + entries
    write_table(prefix + ".index.tmp", items)
    os.replace(data_path + ".tmp", data_path)
    os.replace(prefix + ".index.tmp", prefix + ".index")


def read_bundle(prefix: str, verify: bool = True) -> Dict[str, np.ndarray]:
    items = read_table(prefix + ".index", verify)
    if not items or items[0][0] != b"":
        raise ValueError(f"{prefix}.index: no BundleHeaderProto")
    hdr = _parse(items[0][1])
    if hdr.get(1, [1])[0] != 1:
        raise ValueError(f"{prefix}: {hdr[1][0]} data shards are not supported")
    if hdr.get(2, [0])[0] != 0:
        raise ValueError(f"{prefix}: big-endian bundle")
    out = {}
    with open(prefix + ".data-00000-of-00001", "rb") as f:
        for key, val in items[1:]:
            e = _parse(val)
            if 7 in e:
                raise ValueError(f"{key!r}: sliced (partitioned) variables are not supported")
            dt = e.get(1, [0])[0]
            shape = [_parse(d).get(1, [0])[0] for d in _parse(e[2][0]).get(2, [])] if 2 in e else []
            off, size = e.get(4, [0])[0], e.get(5, [0])[0]
            f.seek(off)
            b = f.read(size)
            if verify and 6 in e and _unmask(e[6][0]) != crc32c(b):
                raise IOError(f"checksum mismatch for {key!r} in {prefix}")
            if dt == DT_BFLOAT16:
                u = np.frombuffer(b, dtype="<u2").astype(np.uint32) << 16
                a = u.view(np.float32)
            elif dt in _DT2NP:
                a = np.frombuffer(b, dtype=_DT2NP[dt].newbyteorder("<"))
            else:
                raise ValueError(f"{key!r}: unsupported TF dtype {dt}")
            out[key.decode()] = a.reshape(shape).copy()
    return out
