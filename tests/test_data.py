"""Data layer parity with the reference (utils.py, data_splitter.py): vocab order, encoding,
TBPTT batch layout (row-contiguous streams, wrap-around target), sharding."""
import os

import numpy as np
import pytest

from distributed_char_rnn_amd.utils import data as D
from distributed_char_rnn_amd.utils import safe_pickle
from distributed_char_rnn_amd.utils.splitter import split_corpus

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CORPUS = os.path.join(ROOT, "data", "tinyshakespeare", "input.txt")
REF_SHARDS = "/root/reference/sharded_data"


def test_vocab_order_frequency_then_first_occurrence():
    chars, vocab = D.build_vocab("abbcccaZZ")
    # counts: c3 b2 a2 Z2 ; ties keep first occurrence (a before b before Z)
    assert chars == ("c", "a", "b", "Z")
    assert vocab == {"c": 0, "a": 1, "b": 2, "Z": 3}


@pytest.mark.skipif(not os.path.exists(CORPUS), reason="corpus missing")
def test_tinyshakespeare_vocab_matches_survey():
    text = D.read_text(CORPUS)
    chars, _ = D.build_vocab(text)
    assert len(text) == 1115394
    assert "".join(chars) == D.SHAKESPEARE_CHARS


def test_encode_decode_roundtrip():
    text = "hello world\nünïcode"
    chars, vocab = D.build_vocab(text)
    ids = D.encode(text, vocab)
    assert ids.dtype == np.int32
    assert D.decode(ids, chars) == text
    with pytest.raises(KeyError):
        D.encode("q", vocab)


def test_batches_match_reference_semantics():
    t = np.arange(12, dtype=np.int32)
    xb, yb, nb, _ = D.make_batches(t, 2, 3)
    assert nb == 2
    np.testing.assert_array_equal(xb[0], [[0, 1, 2], [6, 7, 8]])
    np.testing.assert_array_equal(xb[1], [[3, 4, 5], [9, 10, 11]])
    np.testing.assert_array_equal(yb[0], [[1, 2, 3], [7, 8, 9]])
    np.testing.assert_array_equal(yb[1], [[4, 5, 6], [10, 11, 0]])  # wrap-around y[-1] = x[0]


def test_batches_truncate_and_error():
    xb, _, nb, tt = D.make_batches(np.arange(13, dtype=np.int32), 2, 3)
    assert nb == 2 and tt.size == 12
    with pytest.raises(ValueError):
        D.make_batches(np.arange(5, dtype=np.int32), 2, 3)


def test_text_loader_preprocess_then_load(tmp_path):
    d = tmp_path / "c"
    d.mkdir()
    (d / "input.txt").write_text("the quick brown fox jumps over the lazy dog " * 20)
    a = D.TextLoader(str(d), 4, 5, verbose=False)
    assert (d / "vocab.pkl").exists() and (d / "data.npy").exists()
    b = D.TextLoader(str(d), 4, 5, verbose=False)  # second time: load path
    assert a.chars == b.chars and a.num_batches == b.num_batches
    x, y = a.next_batch()
    assert x.shape == (4, 5) and a.pointer == 1
    a.reset_batch_pointer()
    assert a.pointer == 0
    assert tuple(safe_pickle.load(str(d / "vocab.pkl"))) == a.chars


def test_tensor_file_is_never_overwritten(tmp_path):
    d = tmp_path / "c"
    d.mkdir()
    (d / "input.txt").write_text("abcabcabcabc" * 10)
    shard = tmp_path / "shard.npy"
    np.save(shard, np.zeros(40, dtype=np.int32))
    before = shard.read_bytes()
    ld = D.TextLoader(str(d), 2, 4, tensor_file=str(shard), verbose=False)
    assert shard.read_bytes() == before  # A-6 fixed
    assert ld.num_batches == 5


def test_shard_any_parts():
    t = np.arange(1115394)
    for n in (1, 2, 3, 4, 7, 8):
        parts = D.shard(t, n)
        assert sum(len(p) for p in parts) == t.size and len(parts) == n
    with pytest.raises(ValueError):
        D.shard(t, 4, exact=True)  # the reference's np.split limitation


@pytest.mark.skipif(not (os.path.exists(CORPUS) and os.path.isdir(REF_SHARDS)),
                    reason="reference shards not mounted")
def test_splitter_reproduces_reference_shards(tmp_path):
    d = tmp_path / "ts"
    d.mkdir()
    (d / "input.txt").write_bytes(open(CORPUS, "rb").read())
    paths = split_corpus(str(d), 2, str(tmp_path / "out"), exact=True, verbose=False)
    for i, p in enumerate(paths):
        ours = np.load(p)
        ref = np.load(os.path.join(REF_SHARDS, f"data-{i}.npy"))  # allow_pickle=False default
        np.testing.assert_array_equal(ours, ref)


def test_synthetic_tokens_distribution():
    t = D.synthetic_tokens(200000, 65, seed=0)
    assert t.min() >= 0 and t.max() < 65
    freq = np.bincount(t, minlength=65) / t.size
    assert freq[0] > 0.12  # ' ' is the most frequent char (~15%)
    assert len(D.synthetic_chars(65)) == 65 and len(D.synthetic_chars(100)) == 100


def test_safe_unpickler_refuses_code(tmp_path):
    import pickle

    class Evil:
        def __reduce__(self):
            return (os.system, ("true",))

    p = tmp_path / "evil.pkl"
    p.write_bytes(pickle.dumps(Evil()))
    with pytest.raises(pickle.UnpicklingError):
        safe_pickle.load(str(p))
    import argparse

    ns = argparse.Namespace(model="lstm", rnn_size=3)
    safe_pickle.dump(ns, str(tmp_path / "ok.pkl"))
    assert safe_pickle.load(str(tmp_path / "ok.pkl")) == ns
