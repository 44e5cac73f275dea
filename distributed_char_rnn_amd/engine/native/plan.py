"""Execution plan of the native backend: which kernels run a training / inference step at
(B, T), and the environment knobs that may steer that choice.

Public knobs (docs/DESIGN.md "Knobs"); everything else is chosen from measurements:

=================  ==========================================================================
DCR_RECURRENCE     ``auto`` (default): two-layer wavefront kernels for LSTM layer pairs, single-
                   layer persistent kernels otherwise, per-step kernels where no persistent
                   grid fits; ``single``: no layer-pair wavefronts; ``step``: the fused per-step
                   kernels only (no persistent grids, e.g. several processes on one GPU);
                   ``library``: library GEMM + epilogue kernel per step (large-H LSTM path)
DCR_PAIR_G         batch groups per workgroup of the wavefront kernels (0 = smallest that fits)
DCR_MODE           ``auto`` | ``exclusive`` | ``overlap``: whether anything (RCCL buckets,
                   side-stream GEMMs) may run beside a persistent BPTT grid
DCR_SPIN_LIMIT     bound of every hand-off spin (a timeout sets the error word instead of hanging)
DCR_DEBUG          ``key=value,...`` diagnostic overrides for tests and same-box A/B runs
                   (DEBUG_KEYS below; the C++ launchers read ``gru_ub``, ``step_nbt``,
                   ``wide``, ``wgarr``, ``xcdloc``, ``wide_pf``)
=================  ==========================================================================
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Dict, Mapping, Optional

PERSIST_MIN_T = 8  # shortest sequence that takes the persistent (weights-resident) kernels
# lstm_persist_occupancy flags (csrc/lstm_persist.hip PF_*)
PF_FUSED, PF_DIAG, PF_EXCL = 1, 2, 4

RECURRENCES = ("auto", "single", "step", "library")
MODES = ("auto", "exclusive", "overlap")
DEBUG_KEYS = {
    "persist_min_t": "shortest T that takes the persistent kernels (default 8)",
    "pair_bwd": "0: paired forward, single-layer BPTT",
    "wide": "0: the 16-unit x 32-row pair BPTT instead of the 32 x 16 one (C++ launcher)",
    "wgarr": "0: one hand-off counter add per epilogue wave in the pair kernels (C++ launcher)",
    "xcdloc": "0: write-through (sc1) hand-offs + atomic counters everywhere, never the "
              "XCD-resident form (plain payload, L2 flags) on single-XCD columns (C++ launcher)",
    "wide_pf": "wide BPTT epilogue-operand loads: 0 before the poll, 1 after the payload, 2 "
               "one tick ahead, 3 / 4 poller-wave variants, 5 1 + the row-major dZ copy "
               "deferred behind the next payload + the dtop stash inside the drain, all "
               "unconditional (exact waitcnt), 6 (default) 1 + the dtop stash inside the MFMA "
               "phase (C++)",
    "fused_head": "0: library logits GEMM + CE kernel instead of the fused head",
    "bwd_rs": "1: the reduce-scatter pair BPTT (lstm2_bwd_rs.hip) instead of the all-gather "
              "one (lstm2_bwd_wide.hip); default 0 (measured slower)",
    "tail_wide": "0: the wide-vocabulary head's step keeps the plain Adam + prep layout "
                 "refresh instead of the fused Adam (csrc/tail.hip phase 1)",
    "gru_bpart": "0: GRU bias gradients as column sums of the row-major dZ (a colsum launch per "
                 "layer) instead of the persistent BPTT kernel's partials",
    "graph_refresh": "1: a captured step (--graph) refreshes every weight layout in its prep "
                     "launch even when the fused Adam keeps them current",
    "gru_adam": "0: the GRU step keeps the plain Adam + prep layout refresh instead of the "
                "fused Adam (csrc/tail.hip phase 1)",
    "x0_prep": "0: the wide-vocabulary backward gathers its bf16 embedding rows X0 = E[ids] in "
               "a launch of its own instead of a GATHER task of the step-start prep launch",
    "fin_wide": "0: the wide-vocabulary head's deferred sums as a prep-launch flush (+ a "
                "sum-of-squares launch for the norm) instead of the tail FINALIZE (default 1)",
    "dew": "layer-0 embedding-table gradient: gemm (one-hot MFMA GEMM, default) | segsum | fused",
    "side": "0: no side-stream weight GEMMs in overlap mode",
    "xfuse": "0: no fused input projection in the single-layer persistent forward",
    "exclusive": "0: never pick the one-workgroup-per-CU single-layer BPTT variant",
    "wide_xent": "0: no one-read CE kernel for wide vocabularies",
    "wide_head": "0: library logits GEMM + one-read CE instead of the fused wide-vocabulary head",
    "seg_sort": "0: unsorted atomic embedding gradient for wide vocabularies",
    "lib_graph": "0: eager library-step loops (no hipGraph replay)",
    "bigstep": "large-H LSTM steps: 0 library GEMM + epilogue kernel, 1 (default) the fused MFMA "
               "step kernels (csrc/lstm_gemm_step.hip) where measured faster, 2 fused always",
    "bigstep_s": "n: force n split-K slices in the fused large-H step kernels",
    "bigstep_cfg": "id: force tile configuration id of the fused large-H step kernels (C++)",
    "sample_graph": "0: eager sampling loop (no hipGraph replay)",
    "generate": "0: sampling as the replayed per-character step graph instead of the "
                "single-launch generator (csrc/generate.hip)",
    "head_omask": "0: top output dropout applied to dtop by a separate pass, not the head",
    "xin": "0: library zx GEMM for a dense layer-l input instead of the G = 1 two-layer "
           "forward's in-kernel projection",
    "bits_embed": "0: layer 0's masked embedding rows by their own launch after the dropout bits "
                  "instead of inside the bits launch",
    "xdst": "0: layer l+1's masked input rows by a separate mask pass instead of the G = 1 "
            "two-layer dropout forward's in-kernel store",
    "pair_dw": "0: separate h buffers per layer of a wavefront pair (two weight GEMMs for the "
               "upper layer instead of one over the pair-interleaved h)",
    "gru_dwx": "0: GRU input-weight gradient as one [H, 3H] temporary + sum + two copies",
    "head_lds": "0: fused head streams softmax_wᵀ from L2 instead of staging it in LDS (C++)",
    "nt_bwd": "0: H > 1024: persistent forward (csrc/lstm_persist_nt.hip) but library-GEMM "
              "BPTT steps",
    "nt_poll": "w: hand-off poller on wave w in the H > 1024 persistent kernels (C++ launcher)",
    "nt_dma": "0: H > 1024 persistent forward at NT = 4 streams its h tiles through registers "
              "instead of LDS-DMA (C++ launcher)",
    "wgrad": "0: library split-K GEMMs for the weight gradients instead of the hand-written "
             "wgrad kernel (csrc/wgrad.hip)",
    "tokennorm": "0: TF token-norm term as a library GEMM to bf16 rows + a sumsq launch instead "
                 "of the fused MFMA kernel (csrc/tokennorm.hip)",
    "fwd_steady": "0: the two-layer forward's steady ticks on the generic tick body (run-time "
                  "edge conditions) instead of the constant-condition one (C++)",
    "table_nt": "0: wide-vocabulary gather table E·W_x0 + b0 as a library GEMM on bias rows "
                "instead of one gemm_nt launch with the bias in its epilogue",
    "dx_fused": "0: dropout route's embedding input gradient as a library GEMM + mask pass + "
                "sum-of-squares pass instead of the masked token-norm launch",
    "dws_wgrad": "0: softmax_w gradient (fused head) as a library GEMM instead of a zero-padded "
                 "[H x 256] problem of the wgrad launch",
    "id_sort": "0: library sort of the wide-vocabulary segment-sum ids instead of the counting "
               "sort (csrc/embed.hip id_sort)",
    "dtop_nt": "0: wide-vocabulary dtop = dlogits·softmax_wᵀ as a library GEMM instead of the "
               "token-norm pipeline's store form (csrc/tokennorm.hip gemm_nt)",
    "tail": "0: no fused step tail (csrc/tail.hip): prep-launch slab flush, library fp32 "
            "products, separate norm / Adam / weight-layout launches",
    "tail_queue": "1: tail launches take tiles from the atomic queue even on an unshared GPU",
    "tail_per": "N: tail workgroups per CU (C++, default 2)",
    "gen_dbg": "1: generator without the head, 2: head without h loads (C++, timing only)",
    "hw_fl": "0: wide head always on its generic kernels (runtime flags and counted-wait trees) "
             "instead of the training step's compile-time-flag kernels (C++)",
    "gnt_st": "5: gemm_nt (wide dtop) with a 5-stage ring (C++)",
    "tn_v": "token-norm GEMM: 3 (default) 8 waves, 4-stage ring; 5 the same with 5 stages; 4 four "
            "waves of 128 x 128 (C++)",
    "gru_ub": "1: 16-unit GRU workgroups (C++)",
    "gru_nt": "N: N batch tiles of 16 rows per GRU workgroup (C++)",
    "step_nbt": "1/2/4: batch tiles per per-step workgroup (C++)",
}


def _parse_debug(s: str) -> Dict[str, str]:
    out = {}
    for item in filter(None, (x.strip() for x in s.split(","))):
        k, sep, v = item.partition("=")
        if not sep:
            raise ValueError(f"DCR_DEBUG entry {item!r} is not key=value")
        if k not in DEBUG_KEYS:
            raise ValueError(f"unknown DCR_DEBUG key {k!r} (known: {', '.join(DEBUG_KEYS)})")
        out[k] = v
    return out


@dataclass(frozen=True)
class Knobs:
    recurrence: str = "auto"
    pair_g: int = 0
    mode: str = "auto"
    spin_limit: int = 1 << 22
    debug: Mapping[str, str] = field(default_factory=dict)

    @classmethod
    def from_env(cls, env: Optional[Mapping[str, str]] = None) -> "Knobs":
        env = os.environ if env is None else env
        rec = env.get("DCR_RECURRENCE", "auto")
        mode = env.get("DCR_MODE", "auto")
        if rec not in RECURRENCES:
            raise ValueError(f"DCR_RECURRENCE={rec!r}: one of {RECURRENCES}")
        if mode not in MODES:
            raise ValueError(f"DCR_MODE={mode!r}: one of {MODES}")
        return cls(recurrence=rec, pair_g=int(env.get("DCR_PAIR_G", "0")), mode=mode,
                   spin_limit=int(env.get("DCR_SPIN_LIMIT", str(1 << 22))),
                   debug=_parse_debug(env.get("DCR_DEBUG", "")))

    def dbg(self, key: str, default: str) -> str:
        return self.debug.get(key, default)

    def on(self, key: str) -> bool:
        """A debug switch that is on unless set to 0."""
        return self.debug.get(key, "1") != "0"

    @property
    def persistent(self) -> bool:
        return self.recurrence in ("auto", "single")


@dataclass
class ExecutionPlan:
    """Kernel choice for one (B, T, training) step shape.

    * ``pair`` / ``pair_bwd``: LSTM layers (0,1), (2,3), ... run as two-layer wavefronts
      (csrc/lstm2_persist.hip) with ``pair_g`` 32-row batch groups per workgroup over
      ``pair_nbg`` groups (the batch padded to 32-row groups);
    * ``persist``: the remaining LSTM layers run the single-layer persistent kernels
      (csrc/lstm_persist.hip), ``xfuse`` with the layer input projection fused in;
    * ``gru_persist``: the persistent GRU kernels (csrc/gru_persist.hip);
    * ``mode``: ``exclusive`` (nothing beside a persistent grid: weight GEMMs in stream order,
      all-reduce buckets released after the last BPTT launch) or ``overlap``; ``bwd_excl``: the
      one-workgroup-per-CU single-layer BPTT variant (all hand-off loads in flight).
    """
    persist: bool = False
    persist_bwd: bool = True
    xfuse: bool = False
    mode: str = "exclusive"
    bwd_excl: bool = False
    gru_persist: bool = False
    pair: bool = False
    pair_bwd: bool = False
    pair_g: int = 0
    pair_nbg: int = 0

    @property
    def persistent(self) -> bool:
        return self.persist or self.pair or self.gru_persist

    @property
    def pair_rows(self) -> int:
        """Rows of the wavefront BPTT's bias-gradient partials (two per workgroup column)."""
        return 2 * self.pair_nbg // max(self.pair_g, 1)


def make_plan(ops, cfg, knobs: Knobs, B: int, training: bool, T: int,
              side_overlap: bool) -> ExecutionPlan:
    """Residency plan of the persistent kernels at batch ``B``.

    Every workgroup of a persistent grid spins on its neighbours, so the whole grid must be
    co-resident.  ``lstm_persist_occupancy`` reports how many workgroups of the exact
    instantiation fit on one CU (registers + LDS).  The single-layer kernels run in one of two
    modes:

    * ``overlap``: RCCL buckets and the side-stream weight-gradient GEMMs run *beside* the BPTT
      kernels, so every BPTT grid must leave a spare workgroup slot on each CU
      (grid <= (occupancy - 1) * CUs);
    * ``exclusive``: nothing runs beside the persistent kernels, which allows the faster
      one-workgroup-per-CU BPTT variant.

    Exclusive is preferred whenever its BPTT variant fits: with the weight GEMMs split-K in
    stream order it measured 2.74-2.80 vs 3.03-3.06 ms/step for overlap (H=512, B=256, same
    box) -- a chip-filling GEMM beside the latency-bound recurrence slows both.  The wavefront
    kernels are one workgroup per CU and always exclusive.
    """
    plan = ExecutionPlan()
    H, o = cfg.rnn_size, ops
    if T < int(knobs.dbg("persist_min_t", str(PERSIST_MIN_T))) or not knobs.persistent:
        # a persistent grid first loads every weight slice into registers (~6 MB for the
        # 2-layer H=512 pair); for a handful of steps (sampling: T = 1) the per-step kernels,
        # which stream W_h from L2, are faster (scripts/bench_sample.py)
        return plan
    if cfg.model == "gru":
        # persistent GRU: the C++ side picks the unit block whose fwd and bwd grids are
        # co-resident; always exclusive (nothing beside it)
        plan.gru_persist = bool(o.gru_persist_ub(H, B))
        return plan
    if cfg.model != "lstm":
        return plan
    # two-layer wavefront kernels for layers (0,1), (2,3), ...: any batch (padded to 32-row
    # groups, G groups per workgroup), H in {128..512}
    if cfg.num_layers >= 2 and knobs.recurrence == "auto":
        G = int(o.lstm2_plan(H, B, knobs.pair_g))
        if G:
            plan.pair, plan.pair_g, plan.pair_nbg = True, G, int(o.lstm2_nbg(B, G))
            plan.pair_bwd = training and knobs.on("pair_bwd")
    if not bool(o.lstm_persist_supported(H, B)):
        return plan
    cus, grid = int(o.num_cus()), int(o.lstm_persist_grid(H, B))
    vdew = cfg.vocab_size if (training and cfg.vocab_size <= 128) else 0

    def fits(bwd, flags, margin=0):
        return all(grid <= (int(o.lstm_persist_occupancy(bwd, H, B, v, flags)) - margin) * cus
                   for v in {0, vdew})

    if not (fits(0, 0) and (not training or fits(1, 0))):
        return plan
    plan.persist = True
    # H > 1024 (lstm_persist_nt.hip), 4-layer LSTM-2048 T = 512 B = 64: 87.5 ms/step on the
    # library steps, 71.4 with the persistent forward only, 43.6 with both directions
    plan.persist_bwd = H <= 1024 or knobs.on("nt_bwd")
    plan.xfuse = knobs.on("xfuse") and bool(o.lstm_persist_xfuse_supported(H, B))
    if not training:
        return plan
    shared_ok = fits(1, 0, margin=1)
    excl_ok = fits(1, PF_EXCL) and knobs.on("exclusive")
    if knobs.mode == "overlap" and shared_ok:
        mode = "overlap"
    elif knobs.mode == "exclusive" or excl_ok:
        mode = "exclusive"
    else:
        mode = "overlap" if (shared_ok and side_overlap) else "exclusive"
    if plan.pair_bwd:
        mode = "exclusive"  # one workgroup per CU (register-bound): nothing runs beside it
    plan.mode = mode
    plan.bwd_excl = mode == "exclusive" and excl_ok
    return plan
