"""``CharRNN``: the model facade used by the trainer, sampler and benchmark.

Equivalent of the reference ``Model`` (model.py:8-140) minus the TF graph: parameters live in a
:class:`ParamStore` (flat fp32 buffers, TF names) and execution is delegated to a backend:

* ``native``    -- gfx950 HIP kernels (engine/native/): fused recurrent cell
                   kernels, fused softmax-CE, embedding-projection gather/segment-sum, etc.
                   Mandatory on GPU; raises if the native library is missing.
* ``native32``  -- ``dtype="fp32"`` on a GPU: the oracle's step with every recurrent cell step
                   on the fp32-operand HIP kernels (engine/native/fp32.py).
* ``reference`` -- pure PyTorch autograd with TF cell semantics (models/reference.py); the
                   CPU path and the numerical oracle.

``Model.__init__`` in the reference mutates the caller's args to B = T = 1 for inference
(model.py:11-13); here inference simply calls :meth:`step_logits` with any batch.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from .params import ModelConfig, ParamStore
from .reference import ReferenceBackend, State, zero_state


def _as_ids(x, device: torch.device) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        return x.to(device=device, dtype=torch.int32, non_blocking=True)
    t = torch.from_numpy(np.ascontiguousarray(x, dtype=np.int32))
    if device.type == "cuda":
        t = t.pin_memory()
    return t.to(device, non_blocking=True)


class CharRNN:
    def __init__(self, cfg: ModelConfig, device="cpu", seed: Optional[int] = 0,
                 backend: str = "auto", dtype: str = "auto", rank: int = 0):
        """``seed`` initialises the parameters (identical on every data-parallel rank);
        ``rank`` only decorrelates the ranks' dropout masks."""
        self.cfg = cfg
        self.device = torch.device(device)
        self.store = ParamStore(cfg, self.device, seed)
        if backend == "auto":
            # fp32 on the GPU: the native fp32-operand recurrence (engine/native/fp32.py) for
            # LSTM / GRU / BasicRNN; the default native kernels compute with bf16 operands
            backend = "native" if (self.device.type == "cuda" and dtype != "fp32") else "reference"
            if self.device.type == "cuda" and dtype == "fp32":
                from ..engine.native import fp32 as f32mod

                if f32mod.supported(cfg):
                    backend = "native32"
                else:
                    import warnings

                    warnings.warn(f"dtype fp32 with {cfg.model} / rnn_size {cfg.rnn_size}: no "
                                  "fp32 native kernels; running the PyTorch autograd path")
            if backend == "native" and cfg.rnn_size % 32 != 0 and cfg.model == "nas":
                import warnings

                warnings.warn(f"NAS with rnn_size={cfg.rnn_size} (not a multiple of 32): "
                              "running the PyTorch autograd path on the GPU")
                backend = "reference"
        self.backend_name = backend
        if backend == "native" and cfg.rnn_size % 32 != 0:
            # the MFMA kernels tile H by 32 / 128: run a zero-padded model (engine/native/padded.py)
            from ..engine.native.padded import PaddedNativeBackend

            self.backend = PaddedNativeBackend(self.store, dtype=dtype, seed=seed or 0, rank=rank)
        elif backend == "native":
            from ..engine.native import NativeBackend

            self.backend = NativeBackend(self.store, dtype=dtype, seed=seed or 0, rank=rank)
        elif backend == "native32":
            from ..engine.native.fp32 import NativeFp32Backend

            self.backend = NativeFp32Backend(self.store, seed=(seed or 0) + 7919 * rank)
        elif backend == "reference":
            self.backend = ReferenceBackend(self.store, seed=(seed or 0) + 7919 * rank)
        else:
            raise ValueError(f"unknown backend {backend}")

    def zero_state(self, batch: int) -> State:
        return zero_state(self.cfg, batch, self.device)

    def train_step(self, x, y, state: State, grad_sync=None, want_extras: bool = False):
        """One TBPTT step: forward, loss, backward into ``store.grad``.  ``grad_sync.ready``
        is called as gradient ranges become final.  Returns (cost tensor, final_state,
        extras)."""
        xi, yi = _as_ids(x, self.device), _as_ids(y, self.device)
        # a disabled sync (one rank) gets no callback: the backend then defers its gradient
        # sums to one launch at the end of the step instead of flushing per bucket
        cb = (grad_sync.ready if grad_sync is not None and getattr(grad_sync, "enabled", True)
              else None)
        return self.backend.train_step(xi, yi, state, cb, want_extras=want_extras)

    def step_logits(self, x_t, state: State):
        return self.backend.step_logits(_as_ids(x_t, self.device), state)

    def eval_loss(self, x, y, state: State):
        return self.backend.eval_loss(_as_ids(x, self.device), _as_ids(y, self.device), state)

    def error_word(self) -> Optional[torch.Tensor]:
        """The native backend's device error word (persistent-kernel spin timeouts), for
        ``TFAdam(guard=...)``; None on the reference backend."""
        return getattr(self.backend, "err", None)

    def poll_errors(self) -> None:
        """Non-blocking error-word poll (raises a few steps after a persistent-kernel timeout
        without a device sync); the backend's own poll runs inside train_step unless
        ``defer_err_poll`` is set (data parallelism: the trainer calls this after the exchange)."""
        poll = getattr(self.backend, "_poll_errors", None)
        if poll is not None:
            poll()

    def check_errors(self) -> None:
        """Raise if a persistent kernel timed out (synchronises the device)."""
        check = getattr(self.backend, "check_errors", None)
        if check is not None:
            check()

    @property
    def drop_step(self) -> int:
        """Dropout mask counter of the native backend (checkpointed for --resume_exact)."""
        be = getattr(self.backend, "inner", self.backend)
        return int(getattr(be, "_drop_step", 0))

    @drop_step.setter
    def drop_step(self, v: int) -> None:
        be = getattr(self.backend, "inner", self.backend)
        if hasattr(be, "_drop_step"):
            be._drop_step = int(v)

    def bind_optimizer(self, opt) -> None:
        """Let the backend run ``opt``'s update as its fused step-tail launch when it can
        (native LSTM / BasicRNN: Adam + the bf16 weight layouts in one pass, csrc/tail.hip)."""
        hook = getattr(self.backend, "bind_optimizer", None)
        if hook is not None:
            hook(opt)

    def params_changed(self):
        """Call after parameters were modified outside the optimizer (restore/broadcast)."""
        self.store.version += 1
        hook = getattr(self.backend, "params_changed", None)
        if hook is not None:
            hook()
