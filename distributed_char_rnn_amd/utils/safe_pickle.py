"""Restricted (non-executing) pickle IO for the reference-compatible metadata files.

The reference persists ``config.pkl`` (a pickled ``argparse.Namespace``, train.py:112-113),
``chars_vocab.pkl`` (``(chars, vocab)``, train.py:114-115) and ``vocab.pkl`` (the ``chars``
tuple, utils.py:15-16).  We keep those filenames and payload shapes for drop-in compatibility,
but every load goes through :class:`SafeUnpickler`, which resolves only plain containers,
scalars and ``argparse.Namespace`` -- nothing in the file can execute code.
"""
from __future__ import annotations

import argparse
import io
import pickle

_ALLOWED = {
    ("builtins", "tuple"), ("builtins", "list"), ("builtins", "dict"), ("builtins", "set"),
    ("builtins", "frozenset"), ("builtins", "str"), ("builtins", "int"), ("builtins", "float"),
    ("builtins", "bool"), ("builtins", "bytes"), ("builtins", "NoneType"),
    ("argparse", "Namespace"), ("collections", "OrderedDict"),
    # python2-era pickles (six.moves.cPickle under py2)
    ("__builtin__", "unicode"), ("__builtin__", "tuple"), ("__builtin__", "dict"),
}


class SafeUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if (module, name) in _ALLOWED:
            if module == "argparse":
                return argparse.Namespace
            if module == "collections":
                import collections

                return collections.OrderedDict
            if module == "__builtin__":
                return {"unicode": str, "tuple": tuple, "dict": dict}[name]
            import builtins

            return getattr(builtins, name)
        raise pickle.UnpicklingError(f"refusing to unpickle {module}.{name}")


def load(path: str):
    with open(path, "rb") as f:
        return SafeUnpickler(f).load()


def loads(data: bytes):
    return SafeUnpickler(io.BytesIO(data)).load()


def dump(obj, path: str) -> None:
    """Atomic write (tmp + rename) so concurrent readers never see a torn file."""
    import os

    tmp = f"{path}.tmp.{os.getpid()}"
    with open(tmp, "wb") as f:
        pickle.dump(obj, f, protocol=2)
    os.replace(tmp, path)
