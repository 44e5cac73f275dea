"""Loader for the in-tree gfx950 kernel library ``distributed_char_rnn_amd/_C.so``.

The library registers its ops under ``torch.ops.dcr``.  On a GPU the native path is
mandatory: :func:`ops` raises if the library is missing or fails to load, so a GPU run can
never silently fall back to eager PyTorch.  CPU code paths (tests, gloo plumbing) use the
pure-PyTorch reference implementations in ``ops/reference.py`` instead and never call this.
"""
from __future__ import annotations

import os
import threading

import torch

# DCR_NATIVE_LIB selects another build of the library (same-box A/B runs: scripts/ab_bench.sh)
_LIB = os.environ.get("DCR_NATIVE_LIB") or os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_C.so")
_lock = threading.Lock()
_loaded = False
_err: str | None = None


def library_path() -> str:
    return _LIB


BUILD_INFO: dict = {}


def _in_tree() -> bool:
    return not os.environ.get("DCR_NATIVE_LIB")


def try_load(build_if_missing: bool = False) -> bool:
    """Load the library once; returns True on success.  The in-tree library must match the
    sources next to it (``_build.source_hash`` vs its ``.srchash`` sidecar): a stale one is
    rebuilt first when building is allowed, and refused otherwise."""
    global _loaded, _err
    with _lock:
        if _loaded:
            return True
        from .. import _build

        if _in_tree() and os.path.isdir(_build.CSRC):
            want, have = _build.source_hash(), _build.recorded_hash(_LIB)
            BUILD_INFO.update(source_hash=want, library_hash=have)
            if os.path.exists(_LIB) and have != want:
                if not build_if_missing:
                    _err = (f"{_LIB} was built from other sources (hash {have} != {want}); "
                            "rebuild with python -m distributed_char_rnn_amd._build")
                    return False
                print(f"[dcr] native library stale (built from {have}, sources {want}): "
                      "rebuilding", flush=True)
                _build.build()
                BUILD_INFO.update(library_hash=_build.recorded_hash(_LIB), rebuilt=True)
        if not os.path.exists(_LIB) and build_if_missing:
            _build.build()
            BUILD_INFO.update(library_hash=_build.recorded_hash(_LIB), rebuilt=True)
        if not os.path.exists(_LIB):
            _err = f"native library not built: {_LIB} (run python -m distributed_char_rnn_amd._build)"
            return False
        try:
            torch.ops.load_library(_LIB)
        except Exception as e:  # pragma: no cover - depends on the box
            _err = f"failed to load {_LIB}: {e}"
            return False
        _loaded = True
        return True


def available() -> bool:
    return try_load()


def ops():
    """Return ``torch.ops.dcr``; raise loudly if the native library is unavailable."""
    if not try_load(build_if_missing=os.environ.get("DCR_AUTOBUILD", "1") == "1"):
        raise RuntimeError(_err or "native library unavailable")
    return torch.ops.dcr
