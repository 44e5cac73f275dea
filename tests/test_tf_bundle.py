"""TF V2 tensor-bundle checkpoints (utils/tf_bundle.py): SSTable structure, BundleEntryProto
fields, CRCs and round trips, plus the Saver writing them by default.  Reference: the reference
saves with tf.train.Saver (train.py:145, 209-217); TF itself is not importable here, so these
tests check the on-disk structure against the format spec (LevelDB table + tensor_bundle.proto)
and round trips; reading a real TF-written checkpoint is parity unpinned (no fixture ships in
the reference tree)."""
import os
import struct

import numpy as np
import pytest

from distributed_char_rnn_amd.utils import checkpoint as ckpt
from distributed_char_rnn_amd.utils import tf_bundle as tb


def _tensors():
    rng = np.random.default_rng(0)
    return {
        "rnnlm/multi_rnn_cell/cell_0/lstm_cell/kernel": rng.standard_normal((16, 32), dtype=np.float32),
        "rnnlm/multi_rnn_cell/cell_0/lstm_cell/bias": np.zeros(32, np.float32),
        "rnnlm/softmax_w": rng.standard_normal((8, 5)).astype(np.float32),
        "embedding": rng.standard_normal((5, 8)).astype(np.float32),
        "global_step": np.array(1234, np.int64),
        "Variable": np.array(0.002, np.float32),
        "beta1_power": np.array(0.9 ** 3, np.float32),
        "dcr/batch_pointer": np.array(7, np.int64),
        "ints": np.arange(6, dtype=np.int32).reshape(2, 3),
        "half": np.linspace(0, 1, 7).astype(np.float16),
    }


def test_round_trip_and_dtypes(tmp_path):
    t = _tensors()
    prefix = str(tmp_path / "model.ckpt-3")
    tb.write_bundle(prefix, t)
    assert tb.is_tf_bundle(prefix)
    r = tb.read_bundle(prefix)
    assert set(r) == set(t)
    for k in t:
        assert r[k].dtype == t[k].dtype and r[k].shape == t[k].shape, k
        np.testing.assert_array_equal(r[k], t[k])


def test_sstable_layout(tmp_path):
    prefix = str(tmp_path / "b")
    t = {f"v{i:03d}": np.full((3,), i, np.float32) for i in range(100)}  # several blocks
    tb.write_bundle(prefix, t)
    raw = open(prefix + ".index", "rb").read()
    assert struct.unpack("<Q", raw[-8:])[0] == 0xDB4775248B80FB57
    items = tb.read_table(prefix + ".index")
    keys = [k for k, _ in items]
    assert keys[0] == b"" and keys == sorted(keys) and len(keys) == 101
    hdr = tb._parse(items[0][1])
    assert hdr[1] == [1]                      # num_shards
    assert tb._parse(hdr[3][0])[1] == [1]     # version.producer
    e = tb._parse(dict(items)[b"v042"])
    assert e[1] == [1]                        # DT_FLOAT
    assert tb._parse(tb._parse(e[2][0])[2][0])[1] == [3]  # shape [3]
    assert e[5] == [12]                       # size in bytes
    data = open(prefix + ".data-00000-of-00001", "rb").read()
    off = e[4][0]
    assert tb._unmask(e[6][0]) == tb.crc32c(data[off: off + 12])
    assert np.frombuffer(data[off: off + 12], "<f4").tolist() == [42.0] * 3


def test_corruption_detected(tmp_path):
    prefix = str(tmp_path / "c")
    tb.write_bundle(prefix, {"x": np.arange(10, dtype=np.float32)})
    p = prefix + ".data-00000-of-00001"
    b = bytearray(open(p, "rb").read())
    b[5] ^= 0xFF
    open(p, "wb").write(bytes(b))
    with pytest.raises(IOError):
        tb.read_bundle(prefix)


def test_bfloat16_entries_read_as_float(tmp_path):
    """TF may store bf16 variables (DT_BFLOAT16 = 14): read back as float32."""
    prefix = str(tmp_path / "bf")
    vals = np.array([1.0, -2.5, 0.15625], np.float32)
    u16 = (vals.view(np.uint32) >> 16).astype("<u2").tobytes()
    with open(prefix + ".data-00000-of-00001", "wb") as f:
        f.write(u16)
    entry = tb._entry_proto(tb.DT_BFLOAT16, (3,), 0, len(u16), tb._masked(tb.crc32c(u16)))
    tb.write_table(prefix + ".index", [(b"", tb._header_proto()), (b"w", entry)])
    np.testing.assert_array_equal(tb.read_bundle(prefix)["w"], vals)


def test_saver_writes_tf_bundles_and_reads_json_ones(tmp_path, monkeypatch):
    t = _tensors()
    saver = ckpt.Saver(max_to_keep=2)
    for step in (0, 5, 9):
        saver.save(str(tmp_path), t, step)
    latest = ckpt.latest_checkpoint(str(tmp_path))
    assert latest.endswith("model.ckpt-9") and tb.is_tf_bundle(latest)
    assert not os.path.exists(str(tmp_path / "model.ckpt-0.index"))  # max_to_keep
    np.testing.assert_array_equal(ckpt.Saver.restore(latest)["global_step"], t["global_step"])
    monkeypatch.setenv("DCR_CKPT_FORMAT", "json")
    saver.save(str(tmp_path), t, 12)
    p12 = ckpt.latest_checkpoint(str(tmp_path))
    assert not tb.is_tf_bundle(p12)
    np.testing.assert_array_equal(ckpt.Saver.restore(p12)["ints"], t["ints"])
