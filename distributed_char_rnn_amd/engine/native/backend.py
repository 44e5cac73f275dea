"""``NativeBackend``: one stateful-TBPTT training step on the gfx950 kernels of csrc/.

Replaces the reference's TF graph execution of one ``Session.run([summaries, cost,
final_state, train_op])`` (train.py:199) -- T x L unrolled cell chains forward, tf.gradients
backward -- with an explicit, hand-scheduled forward/backward:

forward, per layer l (time-major rows n = t*B + b):
  * layer 0 without dropout: Zx_0 = (E·W_x0 + b0)[ids] is gathered from a [V, G·H] table
    inside the recurrent kernel (V = 65 rows instead of B·T rows); otherwise Zx = X_l·W_x + b
    is one library GEMM over all T steps, or fused into the recurrent kernel;
  * the recurrence: two-layer wavefront kernels (lstm2_persist.hip) for LSTM layer pairs,
    weights-resident single-layer kernels (lstm_persist.hip, gru_persist.hip), or the fused
    per-step kernels (rnn_step.hip) -- chosen per step shape by ``plan.make_plan``;
head: fused logits + softmax-CE + dlogits + d softmax_b + dtop (head.hip);
backward, top layer first: BPTT kernels (dZ per step, bias partials fused), weight gradients
as split-K library GEMMs, gradient ranges reported ready for the bucketed all-reduce.

All weights are refreshed from the fp32 master buffer into bf16 kernel layouts once per
optimizer step (layouts.py).  Modules: plan (knobs, kernel choice), layouts, buffers, forward,
backward, libstep (large-H library path), inference (logits, eval, sampling).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Tuple

import torch

from ...models.params import ParamStore
from ...ops import native
from .backward import BackwardMixin
from .buffers import BuffersMixin
from .forward import ForwardMixin
from .inference import InferenceMixin
from .layouts import LayerWeights, LayoutsMixin
from .libstep import LibStepMixin
from .plan import Knobs

CELL_ID = {"lstm": 0, "gru": 1, "rnn": 3, "nas": 4}

# launches whose grid must be co-resident on the whole chip (hand-offs between workgroups)
PERSISTENT_OPS = ("lstm2_persist_fwd", "lstm2_persist_bwd", "lstm_persist_fwd",
                  "lstm_persist_bwd", "gru_persist_fwd", "gru_persist_bwd", "generate")


class SharedGpuOps:
    """``DCR_GPU_SHARE=<lock file>``: several processes (data-parallel ranks) share one GPU and
    still run the persistent kernels.  Two co-residency-dependent grids of different processes
    must never overlap (each would wait on workgroups the other keeps off the chip), so every
    persistent launch takes an inter-process file lock, runs, and is synchronised before the
    lock is released; everything else runs concurrently (a persistent grid beside another
    process's ordinary kernels only waits for their CUs).  The step's tail launches then use
    the atomic tile queue (layouts.tail_dynamic).  For multi-process tests on one GPU
    (tests/test_gpu_dp2.py): one rank per GPU needs none of this."""

    def __init__(self, ops, path: str):
        self._ops = ops
        self._path = path
        self._fd = None

    def __getattr__(self, name):
        fn = getattr(self._ops, name)
        if name not in PERSISTENT_OPS:
            return fn

        def locked(*args, **kwargs):
            import fcntl

            if self._fd is None:
                self._fd = open(self._path, "a+")
            fcntl.flock(self._fd, fcntl.LOCK_EX)
            try:
                out = fn(*args, **kwargs)
                torch.cuda.synchronize()
                return out
            finally:
                fcntl.flock(self._fd, fcntl.LOCK_UN)
        return locked


class NativeBackend(LayoutsMixin, BuffersMixin, ForwardMixin, BackwardMixin, LibStepMixin,
                    InferenceMixin):
    def __init__(self, store: ParamStore, dtype: str = "auto", seed: int = 0,
                 knobs: Optional[Knobs] = None, rank: int = 0):
        if dtype not in ("auto", "bf16"):
            raise ValueError("the native GPU path computes in bf16 (use --dtype bf16/auto)")
        self.ops = native.ops()
        share = os.environ.get("DCR_GPU_SHARE")
        self.gpu_shared = bool(share)
        if share:
            self.ops = SharedGpuOps(self.ops, share)
        self.store = store
        self.cfg = store.cfg
        self.dev = store.device
        self.cell = CELL_ID[self.cfg.model]
        self.H = self.cfg.rnn_size
        self.V = self.cfg.vocab_size
        self.L = self.cfg.num_layers
        if self.H % 32 != 0:
            raise ValueError("the GPU path needs rnn_size % 32 == 0")
        self.GW = {"lstm": 4, "gru": 3, "rnn": 1, "nas": 8}[self.cfg.model] * self.H
        self.knobs = knobs if knobs is not None else Knobs.from_env()
        self.spin_limit = self.knobs.spin_limit
        self.side_overlap = self.knobs.on("side")
        self.dew_mode = self.knobs.dbg("dew", "gemm")
        if self.dew_mode not in ("gemm", "segsum", "fused"):
            raise ValueError(f"DCR_DEBUG dew={self.dew_mode!r}: gemm | segsum | fused")
        # fused softmax head (csrc/head.hip): logits + CE + dlogits + d softmax_b + dtop
        self.fused_head = self.knobs.on("fused_head") and bool(self.ops.head_supported(self.V,
                                                                                          self.H))
        # fused wide-vocabulary head (csrc/head_wide.hip): logits + CE + bf16 dlogits + d softmax_b
        # without the fp32 logits round trip, for the vocabularies the narrow head does not cover
        self.wide_head = (not self.fused_head and self.knobs.on("wide_head")
                          and bool(self.ops.head_wide_supported(self.V, self.H)))
        # TF clip-norm semantics for the embedding gradient (models/params.py: clip_norm)
        self.tf_norm = self.cfg.clip_norm == "tf"
        self._wver = None
        self._w: List[LayerWeights] = []
        self._table_dirty = False
        self._head = None
        self._bufs: Dict[Tuple[int, int, bool], dict] = {}
        self.err = torch.zeros(1, dtype=torch.int32, device=self.dev)
        self._err_host: Optional[torch.Tensor] = None
        # data parallelism: the trainer polls the error word itself after the gradient exchange
        # has folded every rank's word into each rank's own (GradSync.finish / ShardedStep), so
        # all ranks see a timeout -- and raise -- on the same step
        self.defer_err_poll = False
        self._side = None
        self._side_used = False
        self._steps = 0
        self.capturing = False  # a hipGraph capture of train_step is in progress (graph_step.py)
        self._npart: Optional[torch.Tensor] = None
        # dropout masks: every data-parallel rank draws its own (the reference's workers each
        # had their own TF RNG), from the shared seed mixed with the rank; the step counter is
        # checkpointed (``drop_step``) so --resume_exact continues the mask sequence
        self._drop_seed = (int(seed) * 0x9E3779B1 + 0x5EED + int(rank) * 0x632BE5AB) & ((1 << 62) - 1)
        self._drop_step = 0
        self._sorted_ids = None  # wide vocabulary: (sorted ids, permutation) of this step
        self._dm_bufs: Dict[Tuple[int, int], dict] = {}
        self.last_dropout_masks: Optional[dict] = None
        # the fused step tail (csrc/tail.hip, engine/native/tail.py): bf16 mirror of the flat
        # parameters (layouts.py), the fused-Adam task table, and the global sum of squares the
        # step's FINALIZE launch left for the update (valid until the optimizer consumes it)
        self._mirror: Optional[torch.Tensor] = None
        self._adam_tab = None
        self._adam_ws = None
        self._adam_sq = None
        self._tail_total: Optional[torch.Tensor] = None
        self._tail_total_ok = False
        self._tn_ws = None  # token-norm kernel partials + ticket
        self._gen_ver = None  # weight version of the generator's softmax_wᵀ copy

    def check_errors(self):
        """Raise if a persistent kernel hit its spin timeout (forces a device sync).  The word
        is cleared so the caller may recover (e.g. restore a checkpoint and continue)."""
        v = int(self.err.item())
        if v:
            self.err.zero_()
            if self._err_host is not None:
                self._err_host.zero_()
            # (under data parallelism the word also carries the fold of every rank's word as
            # float bits -- non-zero iff any rank's kernel timed out: a code >= 0x3F800000
            # may come from a peer)
            who = " (this or a peer rank)" if v >= 0x3F800000 or v < 0 else ""
            raise RuntimeError(f"persistent recurrent kernel timed out (code {v}{who}); the "
                               "optimizer skipped the step's update.  Another process sharing "
                               "this GPU can cause this (one rank per GPU); "
                               "DCR_RECURRENCE=step selects the per-step kernels")
