"""Native execution of models whose ``rnn_size`` is not a multiple of the kernels' tiles.

The reference accepts any ``--rnn_size`` (model.py:30; the default is 128 but e.g. 100 is a
valid choice).  The MFMA kernels tile the hidden dimension by 32 (per-step kernels) and 128
(persistent kernels), so such a model runs as a zero-padded model of ``Hp`` units: every
weight row / column / bias entry of a padding unit is zero, its initial state is zero, and then
its pre-activations are 0, its cell state stays 0 and its output h = o·tanh(0) = 0 (LSTM; GRU:
h = u·0 + (1-u)·tanh(0) = 0; BasicRNN: tanh(0) = 0) -- so it never influences a real unit, and
all of its gradients are zero.  Forward values, the loss and the real gradients are exactly
those of the unpadded model (up to summation order); TF's clip norm is unaffected.

Per step this costs one index-scatter of the parameters into the padded store (only when
they changed), one index-gather of the gradients back, and the state pad / unpad copies."""
from __future__ import annotations

from dataclasses import replace

import torch

from ...models.params import ParamStore, cell_specs
from .backend import NativeBackend


def padded_size(H: int) -> int:
    """Hidden size the kernels run: a multiple of 128 (persistent kernels) up to 1024, else of
    32 (per-step / library kernels)."""
    q = 128 if H <= 1024 else 32
    return -(-H // q) * q


def _block_map(n: int, H: int, Hp: int) -> torch.Tensor:
    """Index map of a dimension made of n // H blocks of H units into blocks of Hp units."""
    i = torch.arange(n)
    return (i // H) * Hp + i % H


def _index_map(store: ParamStore, pstore: ParamStore) -> torch.Tensor:
    """Flat offset in the padded store of every element of every real parameter (in the real
    store's flat order over its specs; alignment gaps excluded)."""
    H, Hp = store.cfg.rnn_size, pstore.cfg.rnn_size
    cells = {sp.name for layer in range(store.cfg.num_layers)
             for sp in cell_specs(store.cfg, layer)}
    parts = []
    for s in store.specs:
        ps = pstore.by_name[s.name]
        if len(s.shape) == 1:
            rows = _block_map(s.shape[0], H, Hp) if s.name in cells else torch.arange(s.shape[0])
            parts.append(ps.offset + rows)
            continue
        R, C = s.shape
        if s.name == "embedding":           # [V, H]
            rmap, cmap = torch.arange(R), _block_map(C, H, Hp)
        elif s.name == "rnnlm/softmax_w":   # [H, V]
            rmap, cmap = _block_map(R, H, Hp), torch.arange(C)
        else:                               # cell kernels [D + H, k H]
            rmap, cmap = _block_map(R, H, Hp), _block_map(C, H, Hp)
        parts.append(ps.offset + (rmap[:, None] * ps.shape[1] + cmap[None, :]).reshape(-1))
    return torch.cat(parts)


def _real_offsets(store: ParamStore) -> torch.Tensor:
    return torch.cat([s.offset + torch.arange(s.numel) for s in store.specs])


class PaddedNativeBackend:
    """Drop-in for :class:`NativeBackend` (same methods) over a zero-padded private model."""

    def __init__(self, store: ParamStore, dtype: str = "auto", seed: int = 0, rank: int = 0):
        if store.cfg.model == "nas":
            raise ValueError("NAS cells need rnn_size % 32 == 0 on the GPU path")
        self.store = store
        self.cfg = store.cfg
        self.H = store.cfg.rnn_size
        self.Hp = padded_size(self.H)
        pcfg = replace(store.cfg, rnn_size=self.Hp)
        self.pstore = ParamStore(pcfg, store.device, seed=None)
        self.pstore.flat.zero_()
        self.inner = NativeBackend(self.pstore, dtype=dtype, seed=seed, rank=rank)
        dev = store.device
        self._dst = _index_map(store, self.pstore).to(dev)   # padded offsets
        self._src = _real_offsets(store).to(dev)             # real offsets
        self._synced = None

    # -- parameters / gradients -----------------------------------------------------------
    def _sync_params(self):
        v = getattr(self.store, "version", 0)
        if self._synced == v:
            return
        self.pstore.flat.index_copy_(0, self._dst, self.store.flat.index_select(0, self._src))
        self.pstore.version += 1
        self.inner.params_changed()
        self._synced = v

    def params_changed(self):
        self._synced = None

    def _gather_grads(self):
        self.store.grad.index_copy_(0, self._src, self.pstore.grad.index_select(0, self._dst))
        self.store.norm_slot_view().copy_(self.pstore.norm_slot_view())

    # -- state ----------------------------------------------------------------------------
    def _pad_state(self, state):
        out = []
        for layer in state:
            comps = []
            for t in layer:
                p = torch.zeros(t.shape[0], self.Hp, dtype=torch.float32, device=t.device)
                p[:, : self.H].copy_(t)
                comps.append(p)
            out.append(tuple(comps))
        return out

    def _unpad_state(self, state):
        return [tuple(t[:, : self.H].contiguous() for t in layer) for layer in state]

    # -- the backend interface --------------------------------------------------------------
    def train_step(self, x, y, state, on_ready=None, want_extras: bool = False):
        self._sync_params()
        loss, new_state, extras = self.inner.train_step(x, y, self._pad_state(state), None,
                                                        want_extras=want_extras)
        self._gather_grads()
        if on_ready is not None:  # padded offsets do not map to the real buckets: all at once
            on_ready(None)
        return loss, self._unpad_state(new_state), extras

    def step_logits(self, x_t, state):
        self._sync_params()
        lg, st = self.inner.step_logits(x_t, self._pad_state(state))
        return lg, self._unpad_state(st)

    def eval_loss(self, x, y, state):
        self._sync_params()
        loss, st = self.inner.eval_loss(x, y, self._pad_state(state))
        return loss, self._unpad_state(st)

    def sample_sequence(self, *args, **kwargs):
        self._sync_params()
        return self.inner.sample_sequence(*args, **kwargs)

    def check_errors(self):
        self.inner.check_errors()

    @property
    def err(self):
        return self.inner.err

    @property
    def last_dropout_masks(self):
        return self.inner.last_dropout_masks

    def _persist_plan(self, *args, **kwargs):
        return self.inner._persist_plan(*args, **kwargs)
