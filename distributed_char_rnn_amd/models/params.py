"""Parameter specification and flat parameter/gradient storage.

Variable names, shapes and initialisers follow the reference graph (model.py:15-54, TF 1.8
cell classes [TF-ext]) so checkpoints keep the reference's naming and layouts:

====================  ==========================================================  ============
cell                  variables (per layer ``l``; ``D`` = input depth, ``H`` = rnn_size)  init
====================  ==========================================================  ============
lstm (LSTMCell)       ``.../cell_l/lstm_cell/kernel`` [D+H, 4H] (gates i,j,f,o),    glorot
                      ``.../lstm_cell/bias`` [4H]  (forget bias +1.0 added at run time) zeros
gru (GRUCell)         ``gru_cell/gates/kernel`` [D+H, 2H] (r,u) / ``gates/bias``    glorot / 1
                      ``gru_cell/candidate/kernel`` [D+H, H] / ``candidate/bias``   glorot / 0
rnn (BasicRNNCell)    ``basic_rnn_cell/kernel`` [D+H, H] / ``bias`` [H]             glorot / 0
nas (NASCell)         ``nas_cell/kernel`` [D, 8H], ``nas_cell/recurrent_kernel``   glorot
                      [H, 8H] (no biases: use_biases=False)
head                  ``rnnlm/softmax_w`` [H, V], ``rnnlm/softmax_b`` [V],         glorot
                      ``embedding`` [V, H]
====================  ==========================================================  ============

(``...`` = ``rnnlm/multi_rnn_cell``.)  TF's default ``get_variable`` initialiser is
glorot-uniform, including for the 1-D ``softmax_b`` (fan_in = fan_out = V).

All trainable tensors live in ONE flat fp32 buffer (and a matching flat gradient buffer), laid
out in *reverse backward-availability order* -- softmax head first, then the top layer down to
layer 0, then the embedding -- so gradient all-reduce buckets are contiguous slices that become
ready in order during BPTT (see parallel/grad_sync.py).  Every tensor starts on a 64-element
boundary so fp32 and bf16 views are 16-byte aligned for vector loads.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch

CELL_SCOPES = {"lstm": "lstm_cell", "gru": "gru_cell", "rnn": "basic_rnn_cell", "nas": "nas_cell"}
ALIGN = 64
SHARD_ALIGN = 64 * 64  # world sizes dividing 64 get 64-element-aligned shards


@dataclass(frozen=True)
class ModelConfig:
    model: str = "lstm"
    vocab_size: int = 65
    rnn_size: int = 128
    num_layers: int = 2
    input_keep_prob: float = 1.0
    output_keep_prob: float = 1.0
    # What the global-norm clip measures for the embedding gradient: "tf" = TF 1.x semantics,
    # the IndexedSlices values (one [H] row per token, before duplicates are summed;
    # model.py:55,91-92 [TF-ext]); "dense" = the norm of the summed [V, H] gradient.
    clip_norm: str = "tf"

    def __post_init__(self):
        if self.model not in CELL_SCOPES:
            raise ValueError(f"model type not supported: {self.model}")
        if self.clip_norm not in ("tf", "dense"):
            raise ValueError(f"clip_norm must be 'tf' or 'dense', got {self.clip_norm!r}")

    @property
    def gates(self) -> int:
        """Gate columns per unit of the recurrent GEMM."""
        return {"lstm": 4, "gru": 2, "rnn": 1, "nas": 8}[self.model]

    @property
    def state_arity(self) -> int:
        return 2 if self.model in ("lstm", "nas") else 1


@dataclass
class ParamSpec:
    name: str
    shape: Tuple[int, ...]
    init: str  # glorot | zeros | ones
    offset: int = 0

    @property
    def numel(self) -> int:
        n = 1
        for s in self.shape:
            n *= s
        return n


def cell_specs(cfg: ModelConfig, layer: int) -> List[ParamSpec]:
    H = cfg.rnn_size
    D = H  # embedding dim == rnn_size (model.py:54), so every layer's input depth is H
    scope = f"rnnlm/multi_rnn_cell/cell_{layer}/{CELL_SCOPES[cfg.model]}"
    if cfg.model == "lstm":
        return [ParamSpec(f"{scope}/kernel", (D + H, 4 * H), "glorot"),
                ParamSpec(f"{scope}/bias", (4 * H,), "zeros")]
    if cfg.model == "gru":
        return [ParamSpec(f"{scope}/gates/kernel", (D + H, 2 * H), "glorot"),
                ParamSpec(f"{scope}/gates/bias", (2 * H,), "ones"),
                ParamSpec(f"{scope}/candidate/kernel", (D + H, H), "glorot"),
                ParamSpec(f"{scope}/candidate/bias", (H,), "zeros")]
    if cfg.model == "rnn":
        return [ParamSpec(f"{scope}/kernel", (D + H, H), "glorot"),
                ParamSpec(f"{scope}/bias", (H,), "zeros")]
    return [ParamSpec(f"{scope}/kernel", (D, 8 * H), "glorot"),
            ParamSpec(f"{scope}/recurrent_kernel", (H, 8 * H), "glorot")]


def model_specs(cfg: ModelConfig) -> List[ParamSpec]:
    H, V = cfg.rnn_size, cfg.vocab_size
    specs = [ParamSpec("rnnlm/softmax_w", (H, V), "glorot"),
             ParamSpec("rnnlm/softmax_b", (V,), "glorot")]
    for layer in reversed(range(cfg.num_layers)):
        specs += cell_specs(cfg, layer)
    specs.append(ParamSpec("embedding", (V, H), "glorot"))
    off = 0
    for s in specs:
        s.offset = off
        off += (s.numel + ALIGN - 1) // ALIGN * ALIGN
    return specs


def glorot_limit(shape: Tuple[int, ...]) -> float:
    if len(shape) == 1:
        fan_in = fan_out = shape[0]
    else:
        fan_in, fan_out = shape[-2], shape[-1]
    return math.sqrt(6.0 / (fan_in + fan_out))


class ParamStore:
    """Flat fp32 parameters + gradients with named views (TF variable names)."""

    def __init__(self, cfg: ModelConfig, device="cpu", seed: Optional[int] = 0):
        self.cfg = cfg
        self.specs = model_specs(cfg)
        last = self.specs[-1]
        # After the last tensor (the embedding): one aligned block whose first element is the
        # "norm slot" -- the per-token sum of squares of the embedding gradient that TF's
        # clip_by_global_norm sees (ModelConfig.clip_norm == "tf").  It lives in the gradient
        # buffer so data-parallel all-reduce sums it with everything else for free; the
        # optimizer never updates it.
        self.norm_slot = last.offset + (last.numel + ALIGN - 1) // ALIGN * ALIGN
        # total size a multiple of SHARD_ALIGN: the sharded data-parallel optimizer
        # (parallel/zero.py) splits the flat buffers into world equal, 64-element-aligned shards
        self.numel = -(-(self.norm_slot + ALIGN) // SHARD_ALIGN) * SHARD_ALIGN
        self.device = torch.device(device)
        self.flat = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros_like(self.flat)
        self.by_name: Dict[str, ParamSpec] = {s.name: s for s in self.specs}
        self.version = 0  # bumped whenever `flat` changes (optimizer step, restore, broadcast)
        self.initialize(seed)

    # -- views ---------------------------------------------------------------------------
    def view(self, name: str, buf: Optional[torch.Tensor] = None) -> torch.Tensor:
        s = self.by_name[name]
        b = self.flat if buf is None else buf
        return b.narrow(0, s.offset, s.numel).view(s.shape)

    def gview(self, name: str) -> torch.Tensor:
        return self.view(name, self.grad)

    def names(self) -> List[str]:
        return [s.name for s in self.specs]

    def norm_terms(self) -> Tuple[int, bool]:
        """(n_norm, use_slot): the clip norm is sum(grad[:n_norm]^2) (+ grad[norm_slot] when
        use_slot).  In "tf" mode the dense embedding gradient (the last tensor) is replaced
        by the per-token term in the slot."""
        if self.cfg.clip_norm == "tf":
            return self.by_name["embedding"].offset, True
        return self.norm_slot, False

    def norm_slot_view(self, buf: Optional[torch.Tensor] = None) -> torch.Tensor:
        b = self.grad if buf is None else buf
        return b.narrow(0, self.norm_slot, 1)

    def layer_names(self, layer: int) -> List[str]:
        return [s.name for s in cell_specs(self.cfg, layer)]

    def layer_range(self, layer: int) -> Tuple[int, int]:
        """[start, end) of one layer's parameters in the flat buffer."""
        names = self.layer_names(layer)
        lo = min(self.by_name[n].offset for n in names)
        hi = max(self.by_name[n].offset + self.by_name[n].numel for n in names)
        return lo, hi

    # -- init ----------------------------------------------------------------------------
    def initialize(self, seed: Optional[int] = 0) -> None:
        g = torch.Generator(device="cpu")
        if seed is not None:
            g.manual_seed(int(seed))
        host = torch.zeros(self.numel, dtype=torch.float32)
        for s in self.specs:
            v = host.narrow(0, s.offset, s.numel)
            if s.init == "glorot":
                lim = glorot_limit(s.shape)
                v.uniform_(-lim, lim, generator=g)
            elif s.init == "ones":
                v.fill_(1.0)
            else:
                v.zero_()
        self.flat.copy_(host)
        self.version = getattr(self, "version", 0) + 1

    def state_dict(self) -> Dict[str, torch.Tensor]:
        return {s.name: self.view(s.name).detach().cpu().clone() for s in self.specs}

    def load_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True) -> None:
        for s in self.specs:
            if s.name not in sd:
                if strict:
                    raise KeyError(f"missing variable {s.name}")
                continue
            t = torch.as_tensor(sd[s.name])
            if tuple(t.shape) != s.shape:
                raise ValueError(f"{s.name}: shape {tuple(t.shape)} != {s.shape}")
            self.view(s.name).copy_(t.to(self.flat.dtype))
        self.version += 1
