"""Native (gfx950 HIP) execution of one stateful-TBPTT training step.

Replaces the reference's TF graph execution of one ``Session.run([summaries, cost,
final_state, train_op])`` (train.py:199) -- T x L unrolled cell chains forward, tf.gradients
backward -- with an explicit, hand-scheduled forward/backward over the kernels in ``csrc/``:

forward, per layer l (time-major rows n = t*B + b):
  * Zx = X_l · W_x + b  -- one MFMA library GEMM over all T steps (hipBLASLt, fp32 out); for
    layer 0 without dropout the GEMM disappears: Zx_0 = (E·W_x0 + b0)[ids] is gathered from a
    [V, G·H] table inside the recurrent kernel (V = 65 rows instead of B·T rows);
  * ``dcr::rnn_fwd_seq``: the fused recurrent-GEMM + cell kernels, T launches from C++;
head: logits = O·W_s + b_s (GEMM), ``dcr::xent`` = fused softmax-CE forward + dlogits;
backward, top layer first:
  * dO = dlogits·W_sᵀ, dW_s = Oᵀ·dlogits, db_s = colsum  -> head bucket ready for all-reduce
  * ``dcr::rnn_bwd_seq``: fused recurrent-GEMM + cell-backward kernels (dZ per step)
  * dW_h = H_prevᵀ·dZ, dW_x = X_lᵀ·dZ, db = colsum(dZ), dX = dZ·W_xᵀ  -> layer bucket ready
  * layer 0 (gather mode): dEW = segsum(dZ_0 by id) [V, G·H]; dW_x0 = Eᵀ·dEW, db_0 = colsum(dEW),
    dE = dEW·W_x0ᵀ  (three tiny GEMMs instead of two [B·T]-sized ones)

All weights are refreshed from the fp32 master buffer into bf16 kernel layouts once per
optimizer step (W_hᵀ for the forward's A operand, W_h in TF layout for the backward's).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch

from ..models.params import ParamStore, cell_specs
from ..ops import native

CELL_ID = {"lstm": 0, "gru": 1, "rnn": 3, "nas": 4}
FORGET_BIAS = 1.0
PERSIST_MIN_T = 8  # shortest sequence that takes the persistent (weights-resident) kernels
SEG_LDS_MAX_V = 96  # csrc/embed.hip kSegLdsMaxV: larger vocabularies take the atomic scatter
# lstm_persist_occupancy flags (csrc/lstm_persist.hip PF_*)
PF_FUSED, PF_DIAG, PF_EXCL, PF_GRANULE = 1, 2, 4, 8
bf16 = torch.bfloat16
f32 = torch.float32


def _mm(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """bf16 x bf16 -> fp32 GEMM on the MFMA library path."""
    return torch.mm(a, b, out_dtype=f32)


_OUT_OK = [None]


def _mm_into(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor,
             bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """GEMM written straight into ``out`` (e.g. a gradient view of the flat buffer), avoiding
    a temporary + copy; falls back to copy if this torch build lacks the out= overload."""
    if _OUT_OK[0] is not False and out.is_contiguous():
        try:
            if bias is None:
                torch.mm(a, b, out_dtype=f32, out=out)
            else:
                torch.addmm(bias, a, b, out_dtype=f32, out=out)
            _OUT_OK[0] = True
            return out
        except (RuntimeError, TypeError):
            _OUT_OK[0] = False
    out.copy_(_mm(a, b) if bias is None else torch.addmm(bias, a, b, out_dtype=f32))
    return out


def _split_k(K: int, M: int, Nn: int) -> int:
    """Split factor for a token-reduction GEMM with a small [M, Nn] output: the library tiles
    such an output into a few dozen workgroups (the 512x2048, K=32768 weight gradient ran on 73
    of 256 CUs at 335 TFLOP/s), so the reduction is split into S batched slices instead
    (scripts/bench_gemms.py: 205 -> 97 us at S=8; the 512x65 head gradient 133 -> 27 us)."""
    if K < 8192 or -(-M // 128) * -(-Nn // 256) >= 128:
        return 1
    S = 8 if M * Nn >= (1 << 18) else 16
    while S > 1 and (K % S or K // S < 1024):
        S //= 2
    return S


def _mm_tn(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None,
           split: bool = True) -> torch.Tensor:
    """fp32 ``aᵀ·b`` for token-major bf16 operands ``a`` [K, M] and ``b`` [K, Nn] (weight
    gradients: K = T·B tokens), split-K over batched MFMA GEMMs + one fp32 sum when the output
    is too small to fill the chip.  ``split=False`` for GEMMs that run beside a persistent
    kernel on a side stream: there a chip-filling grid only steals the recurrence's CUs
    (measured: 256-workgroup split-K beside BPTT stretched both)."""
    K, M = a.shape
    Nn = b.shape[1]
    S = _split_k(K, M, Nn) if split else 1
    if S == 1:
        return _mm(a.t(), b) if out is None else _mm_into(a.t(), b, out)
    part = torch.bmm(a.unflatten(0, (S, K // S)).transpose(1, 2), b.unflatten(0, (S, K // S)),
                     out_dtype=f32)
    if out is None:
        return part.sum(0)
    torch.sum(part, 0, out=out)
    return out


def _put(dst: torch.Tensor, src: torch.Tensor):
    """dst.copy_(src) unless src already is dst's memory (results written in place)."""
    if not (src.data_ptr() == dst.data_ptr() and src.shape == dst.shape
            and src.stride() == dst.stride()):
        dst.copy_(src)


@dataclass
class LayerWeights:
    Wx: torch.Tensor            # [D, GW] bf16 input projection
    Wx32: Optional[torch.Tensor]  # [D, GW] fp32 (layer-0 table / dE)
    bias: torch.Tensor          # [GW] fp32 (zeros for NAS)
    Wh: torch.Tensor            # [H, GWr] bf16 TF layout (backward A operand); GRU: Wc_h
    WhT: torch.Tensor           # [GWr, H] bf16 (forward A operand); GRU: Wg_hᵀ
    W2: Optional[torch.Tensor] = None   # GRU: Wg_h [H, 2H]
    WxT: Optional[torch.Tensor] = None  # LSTM: W_xᵀ [4H, D] (fused-input persistent forward)
    WT2: Optional[torch.Tensor] = None  # GRU: Wc_hᵀ [H, H]


@dataclass
class LayerBufs:
    hbuf: torch.Tensor
    cbuf: Optional[torch.Tensor]
    h32: Optional[torch.Tensor]
    gates: Optional[torch.Tensor]
    pre: Optional[torch.Tensor]
    aux: Optional[torch.Tensor]
    rh: Optional[torch.Tensor]
    hlast32: torch.Tensor
    zx: Optional[torch.Tensor]
    dz: Optional[torch.Tensor]
    dzx: Optional[torch.Tensor]
    x_in: Optional[torch.Tensor] = None      # bf16 [N, D] layer input (dense mode)
    clast32: Optional[torch.Tensor] = None   # fp32 [B, H] final c (persistent LSTM)
    x_drop: Optional[torch.Tensor] = None    # bf16 [N, D] masked layer input (dropout)


class NativeBackend:
    def __init__(self, store: ParamStore, dtype: str = "auto", seed: int = 0):
        if dtype not in ("auto", "bf16"):
            raise ValueError("the native GPU path computes in bf16 (use --dtype bf16/auto)")
        self.ops = native.ops()
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
        self._wver = None
        self._w: List[LayerWeights] = []
        self._table_dirty = False
        self._head = None
        self._bufs: Dict[Tuple[int, int, bool], dict] = {}
        self.use_persist = os.environ.get("DCR_PERSIST", "1") != "0"
        self.persist_min_t = int(os.environ.get("DCR_PERSIST_MIN_T", str(PERSIST_MIN_T)))
        # two-layer wavefront forward (lstm2_persist.hip) for layers (0, 1)
        self.use_pair = os.environ.get("DCR_PAIR", "1") != "0"
        # two-layer wavefront BPTT (lstm2_persist.hip) for the same pairs
        self.use_pair_bwd = os.environ.get("DCR_PAIR_BWD", "1") != "0"
        # large-H weights-resident forward (lstm_big.hip) for 1024 < H <= 2048: opt-in.  Its
        # every-step all-to-all hand-off spans all 8 XCDs and the payload phase measured ~15 us
        # per step (scripts/big_stamps.py) vs 16.4 us for a whole per-step kernel, so the
        # per-step kernels stay the default there (open gap)
        self.use_big_fwd = os.environ.get("DCR_BIG_FWD", "0") == "1"
        self.spin_limit = int(os.environ.get("DCR_SPIN_LIMIT", str(1 << 22)))
        # forward hand-off form: "granule" (tagged data, R2) or "counter" (sc1 data + counter)
        self.handoff = os.environ.get("DCR_HANDOFF", "counter")
        # fused dtop (dZ_above·W_xᵀ inside the lower layer's BPTT): measured slower (4.22 vs
        # 3.47 ms/step: its extra dZ loads sit on the load-bound critical path), opt-in only
        self.fused_dtop = os.environ.get("DCR_FUSED_DTOP", "0") == "1"
        self.side_overlap = os.environ.get("DCR_SIDE", "1") == "1"
        # layer-0 embedding-table gradient dEW = onehot(ids)ᵀ·dZ0 [V, 4H]:
        #   "gemm"  split-K MFMA GEMM against a bf16 one-hot matrix after the BPTT;
        #   "fused" LDS atomics inside the BPTT epilogue;  "segsum" the segment-sum kernel
        self.dew_mode = os.environ.get("DCR_DEW", "gemm")
        self.fused_dew = self.dew_mode == "fused"
        # fused softmax head (csrc/head.hip): logits + CE + dlogits + d softmax_b + dtop
        self.fused_head = (os.environ.get("DCR_FUSED_HEAD", "1") != "0"
                           and bool(self.ops.head_supported(self.V, self.H)))
        self.err = torch.zeros(1, dtype=torch.int32, device=self.dev)
        self._err_host: Optional[torch.Tensor] = None
        self._side = None
        self._side_used = False
        self._steps = 0
        # TF clip-norm semantics for the embedding gradient (models/params.py: clip_norm)
        self.tf_norm = self.cfg.clip_norm == "tf"
        self._npart: Optional[torch.Tensor] = None
        self._tpart: Optional[torch.Tensor] = None
        self.tok_norm_fused = os.environ.get("DCR_TOK_NORM", "library") == "fused"
        self.libstep = os.environ.get("DCR_LIBSTEP", "auto")
        # per-step recurrent GEMM of the library-step path: "library" (hipBLASLt) or "native"
        # (csrc/step_gemm.hip split-K; correct, but its fp32 split slabs cost more than they
        # save: LSTM-2048 108.5 vs 96.0 ms at B = 64, 216 vs 199 at B = 256)
        self.step_gemm_mode = os.environ.get("DCR_STEP_GEMM", "library")
        self._drop_seed = int(seed) * 0x9E3779B1 + 0x5EED
        self._drop_step = 0
        self._dm_bufs: Dict[Tuple[int, int], dict] = {}
        self.last_dropout_masks: Optional[dict] = None

    # ------------------------------------------------------------------ weights
    def params_changed(self):
        self._wver = None

    def _alloc_weights(self):
        """bf16 (and padded / concatenated fp32) layouts of the master weights, allocated once
        and refreshed by ``_weight_tasks`` through the batched prep kernel."""
        s, H, D, dev = self.store, self.H, self.H, self.dev
        self._w, self._wtasks = [], []
        T = self._wtasks
        e = lambda *shape, dt=bf16: torch.empty(*shape, dtype=dt, device=dev)  # noqa: E731
        for layer in range(self.L):
            names = [sp.name for sp in cell_specs(self.cfg, layer)]
            if self.cfg.model in ("lstm", "rnn"):
                k, b = s.view(names[0]), s.view(names[1])
                GW = k.shape[1]
                lw = LayerWeights(Wx=e(D, GW), Wx32=k[:D], bias=b, Wh=e(H, GW), WhT=e(GW, H),
                                  WxT=e(GW, D) if (layer > 0 and self.cfg.model == "lstm")
                                  else None)
                T += [(k[D:], lw.Wh, 0), (k[D:], lw.WhT, 1), (k[:D], lw.Wx, 0)]
                if lw.WxT is not None:
                    T.append((k[:D], lw.WxT, 1))
            elif self.cfg.model == "gru":
                gk, gb, ck, cb = (s.view(n) for n in names)
                Wx32, bias = e(D, 3 * H, dt=f32), e(3 * H, dt=f32)
                lw = LayerWeights(Wx=e(D, 3 * H), Wx32=Wx32, bias=bias, Wh=e(H, H),
                                  WhT=e(2 * H, H), W2=e(H, 2 * H), WT2=e(H, H))
                T += [(gk[:D], Wx32[:, : 2 * H], 0), (ck[:D], Wx32[:, 2 * H:], 0),
                      (gk[:D], lw.Wx[:, : 2 * H], 0), (ck[:D], lw.Wx[:, 2 * H:], 0),
                      (gk[D:], lw.W2, 0), (gk[D:], lw.WhT, 1), (ck[D:], lw.Wh, 0),
                      (ck[D:], lw.WT2, 1), (gb.view(1, -1), bias[: 2 * H].view(1, -1), 0),
                      (cb.view(1, -1), bias[2 * H:].view(1, -1), 0)]
            else:  # nas
                kx, km = s.view(names[0]), s.view(names[1])
                lw = LayerWeights(Wx=e(D, 8 * H), Wx32=kx, bias=torch.zeros(8 * H, device=dev),
                                  Wh=e(H, 8 * H), WhT=e(8 * H, H))
                T += [(km, lw.Wh, 0), (km, lw.WhT, 1), (kx, lw.Wx, 0)]
            self._w.append(lw)
        Ws32 = s.view("rnnlm/softmax_w")
        self._head = dict(E=s.view("embedding"), Ws=e(H, self.V), bs=s.view("rnnlm/softmax_b"))
        T.append((Ws32, self._head["Ws"], 0))
        if self.fused_head:
            VP, VK = self.ops.head_pads(self.V)
            self._head["WsT"] = torch.zeros(VP, H, dtype=bf16, device=dev)   # pads stay zero
            self._head["Wsk"] = torch.zeros(H, VK, dtype=bf16, device=dev)
            T += [(Ws32, self._head["WsT"][: self.V], 1),
                  (Ws32, self._head["Wsk"][:, : self.V], 0)]

    def _prep(self) -> list:
        """Prep-kernel tasks that refresh the weight layouts after a parameter change (empty
        when the weights are current); the layer-0 ``E·W_x + b`` table is recomputed after
        they ran (``_run_prep``)."""
        ver = getattr(self.store, "version", 0)
        if not self._w:
            self._alloc_weights()
        elif self._wver == ver:
            return []
        self._wver = ver
        self._table_dirty = True
        return list(self._wtasks)

    def _run_prep(self, tasks: list):
        for i in range(0, len(tasks), 48):  # kPrepMaxTasks
            chunk = tasks[i: i + 48]
            self.ops.prep([t[0] for t in chunk], [t[1] for t in chunk], [t[2] for t in chunk])
        if self._table_dirty:
            w0 = self._w[0]
            if self.V > SEG_LDS_MAX_V:
                # wide vocabulary: the [V, H] x [H, GW] table product on bf16 MFMA operands
                # (the fp32 GEMM took 139 us per step at V = 8192), i.e. the same operand
                # precision as a bf16 layer-0 input projection; the bf16 E copy is also the
                # row source of the dense backward route's X0 gather
                Eb = self._head.get("Ebf")
                if Eb is None or Eb.shape != self._head["E"].shape:
                    Eb = self._head["Ebf"] = torch.empty_like(self._head["E"], dtype=bf16)
                Eb.copy_(self._head["E"])
                self._head["table"] = torch.addmm(w0.bias, Eb, w0.Wx, out_dtype=f32)
            else:
                self._head["table"] = torch.addmm(w0.bias, self._head["E"], w0.Wx32)  # [V, GW]
            self._table_dirty = False

    # ------------------------------------------------------------------ buffers
    def _buffers(self, B: int, T: int, training: bool) -> dict:
        key = (B, T, training)
        if key in self._bufs:
            return self._bufs[key]
        H, GW, dev, m = self.H, self.GW, self.dev, self.cfg.model
        N = B * T
        plan = self._persist_plan(B, training, T)
        Bp = max(B, 32 * plan["pair_nbg"])  # hand-off rings of the pair kernels: padded batch
        nrow = max(B // 16, 2 * plan["pair_nbg"] // max(plan["pair_g"], 1), 1)
        layers = []
        for layer in range(self.L):
            dense = layer > 0 or self._dropout(training)
            lb = LayerBufs(
                hbuf=torch.empty(T + 1, B, H, dtype=bf16, device=dev),
                cbuf=torch.empty(T + 1, B, H, dtype=f32, device=dev) if m in ("lstm", "nas") else None,
                h32=torch.empty(T + 1, B, H, dtype=f32, device=dev) if m == "gru" else None,
                gates=(torch.empty(T, B, GW, dtype=bf16, device=dev)
                       if m == "gru" or (m == "lstm" and training) else None),
                pre=torch.empty(T, B, GW, dtype=f32, device=dev) if m == "nas" else None,
                aux=torch.empty(T, B, H, dtype=f32, device=dev) if m == "nas" else None,
                rh=torch.empty(T, B, H, dtype=bf16, device=dev) if m == "gru" else None,
                hlast32=torch.empty(B, H, dtype=f32, device=dev),
                zx=torch.empty(T, B, GW, dtype=f32, device=dev) if (dense or m == "nas") else None,
                dz=torch.empty(T, B, GW, dtype=bf16, device=dev) if training else None,
                dzx=torch.empty(T, B, GW, dtype=bf16, device=dev) if (training and m == "nas") else None,
            )
            if training and self._dropout(True):
                lb.x_drop = torch.empty(N, H, dtype=bf16, device=dev)
            layers.append(lb)
        ws = max(self.ops.segsum_workspace(N, GW, self.V), self.ops.segsum_workspace(N, H, self.V),
                 self.ops.segsum_workspace(N, GW, 1), self.ops.segsum_workspace(N, self.V, 1), 1)
        bufs = dict(
            layers=layers,
            logits=torch.empty(N, self.V, dtype=f32, device=dev),
            dlogits=torch.empty(N, self.V, dtype=bf16, device=dev) if training else None,
            row_loss=torch.empty(N, dtype=f32, device=dev),
            xpart=torch.empty(self.ops.xent_num_partials(N), dtype=f32, device=dev),
            loss=torch.empty(1, dtype=f32, device=dev),
            dc=torch.empty(B, H, dtype=f32, device=dev),
            gpart=torch.empty(B, H, dtype=f32, device=dev) if m == "gru" else None,
            ws=torch.empty(ws, dtype=f32, device=dev),
            colsum=torch.empty(1, max(GW, self.V), dtype=f32, device=dev),
            head_part=(torch.empty(self.ops.head_workspace(N, self.V), dtype=f32, device=dev)
                       if self.fused_head else None),
            onehot=(torch.empty(N, 8 * ((self.V + 7) // 8), dtype=bf16, device=dev)
                    if (training and self.V <= SEG_LDS_MAX_V) else None),
            colpart=(torch.empty(self.ops.xent_wide_waves(N) * self.V, dtype=f32, device=dev)
                     if (training and self._wide_xent(N)) else None),
            **plan,
            dtop=torch.empty(T, B, H, dtype=f32, device=dev) if training else None,
            dx=torch.empty(T, B, H, dtype=f32, device=dev) if training else None,
            dx_bf=torch.empty(N, H, dtype=bf16, device=dev) if training else None,
            db_part=(torch.empty(self.L, nrow, GW, dtype=f32, device=dev)
                     if training else None),
            dew_part=(torch.empty(max(B // 16, 1), self.V, GW, dtype=f32, device=dev)
                      if (training and self.V <= 128) else None),
            # one hand-off counter region per persistent launch (fwd layers, then bwd layers),
            # zeroed together by the step's prep launch
            cnt=torch.zeros(2 * self.L, max(2 * (B // 16 + 1), plan["pair_nbg"]) * (T + 1) * 4,
                            dtype=torch.int32, device=dev),
            ring=torch.zeros(2 * B * (H // 2), dtype=torch.int64, device=dev),
            # fragment-tiled hand-off rings of the persistent GRU: [h or dZc, r⊙h, dZg]
            grings=((torch.empty(2 * B * H, dtype=bf16, device=dev),
                     torch.empty(2 * B * H, dtype=bf16, device=dev),
                     torch.empty(2 * B * 2 * H, dtype=bf16, device=dev))
                    if (m == "gru" and os.environ.get("DCR_FRAG", "1") != "0") else None),
            # fragment-tiled h hand-off rings of the wavefront forward (persist_common.h)
            hrings=((torch.empty(2 * Bp * H, dtype=bf16, device=dev),
                     torch.empty(2 * Bp * H, dtype=bf16, device=dev))
                    if (os.environ.get("DCR_FRAG", "1") != "0" or plan["pair"]) else None),
            # fragment-tiled dZ hand-off ring of the persistent BPTT (persist_common.h)
            o_drop=(torch.empty(N, H, dtype=bf16, device=dev)
                    if (training and self._dropout(True)) else None),
            zring=(torch.empty(2 * Bp * GW, dtype=bf16, device=dev)
                   if (training and (os.environ.get("DCR_FRAG", "1") != "0" or plan["pair_bwd"]))
                   else None),
        )
        # second dZ ring for the two-layer wavefront BPTT (one ring per layer)
        bufs["zring2"] = (torch.empty(2 * Bp * GW, dtype=bf16, device=dev)
                          if bufs["pair_bwd"] else None)
        # layers run by the persistent LSTM kernels (their final state is written into fresh
        # tensors, their bias gradients come from the kernels' db_part partials)
        npair = 2 * (self.L // 2) if bufs["pair"] else 0
        bufs["pers_layers"] = set(range(npair)) | (set(range(npair, self.L)) if bufs["persist"]
                                                   else set())
        bufs["pair_rows"] = 2 * bufs["pair_nbg"] // max(bufs["pair_g"], 1)
        self._bufs[key] = bufs
        return bufs

    def _wide_xent(self, N: int) -> bool:
        """Library logits GEMM + one-read CE kernel (xent_wide) for vocabularies the fused head
        does not cover (V > 256)."""
        return (not self.fused_head and self.V >= 256 and os.environ.get("DCR_WIDE_XENT", "1") != "0"
                and bool(self.ops.xent_wide_supported(self.V)))

    def _side_stream(self):
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.dev)
        return self._side

    def _exclusive_ok(self, bufs) -> bool:
        """One-workgroup-per-CU persistent variants need the whole GPU to themselves: only when
        no collective (RCCL) or side-stream kernel can run beside them."""
        if not bufs["xfuse"] or os.environ.get("DCR_EXCLUSIVE", "1") == "0":
            return False
        return self._world() == 1

    @staticmethod
    def _world() -> int:
        import torch.distributed as dist

        return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1

    def _persist_plan(self, B: int, training: bool, T: int = 1 << 30) -> dict:
        """Residency plan for the persistent kernels at batch ``B``.

        Every workgroup of a persistent grid spins on its neighbours, so the whole grid must be
        co-resident.  ``lstm_persist_occupancy`` reports how many workgroups of the exact
        instantiation fit on one CU (registers + LDS).  The kernels run in one of two modes:

        * ``overlap``: RCCL buckets and the side-stream weight-gradient GEMMs run *beside* the
          BPTT kernels, so every BPTT grid must leave a spare workgroup slot on each CU
          (grid <= (occupancy - 1) * CUs);
        * ``exclusive``: nothing runs beside the persistent kernels (weight GEMMs in stream order,
          all-reduce buckets released after the last BPTT launch), which allows the faster
          one-workgroup-per-CU BPTT variant (all hand-off loads in flight, PF_EXCL).

        Exclusive is preferred whenever its BPTT variant fits: with the weight GEMMs split-K in
        stream order it measured 2.74-2.80 vs 3.03-3.06 ms/step for overlap (H=512, B=256, same
        box) -- a chip-filling GEMM beside the latency-bound recurrence slows both.  Under data
        parallelism the gradient buckets are released right after the last BPTT launch, so the
        all-reduce still overlaps the layer-0 weight GEMMs.  ``DCR_MODE=overlap|exclusive``
        forces a mode.
        """
        plan = dict(persist=False, xfuse=False, mode="exclusive", bwd_excl=False,
                    gru_persist=False, pair=False, pair_bwd=False, big_fwd=False, pair_g=0,
                    pair_nbg=0)
        o = self.ops
        if T < self.persist_min_t:
            # a persistent grid first loads every weight slice into registers (~6 MB for the
            # 2-layer H=512 pair); for a handful of steps (sampling: T = 1) the per-step kernels,
            # which stream W_h from L2, are faster (sampling 50 -> see scripts/bench_sample.py)
            return plan
        if self.use_persist and self.cfg.model == "gru":
            # persistent GRU (gru_persist.hip): the C++ side picks the unit block whose fwd and
            # bwd grids are co-resident; always exclusive (nothing beside it)
            plan["gru_persist"] = bool(o.gru_persist_ub(self.H, B))
            return plan
        if (self.use_persist and self.cfg.model == "lstm" and self.H > 1024
                and os.environ.get("DCR_FRAG", "1") != "0"
                and self.use_big_fwd and bool(o.lstm_big_supported(self.H, B))):
            # large H (lstm_big.hip): weights-resident forward with 8-unit shards; the BPTT
            # stays on the per-step kernels
            plan["big_fwd"] = True
            return plan
        if not (self.use_persist and self.cfg.model == "lstm"):
            return plan
        # two-layer wavefront kernels (lstm2_persist.hip) for layers (0,1), (2,3), ...: any
        # batch (padded to 32-row groups, G groups per workgroup), H in {128..512}
        if self.L >= 2 and self.use_pair:
            G = int(o.lstm2_plan(self.H, B, int(os.environ.get("DCR_PAIR_G", "0"))))
            if G:
                plan.update(pair=True, pair_g=G, pair_nbg=int(o.lstm2_nbg(B, G)),
                            pair_bwd=training and self.use_pair_bwd)
                if training:
                    plan["mode"] = "exclusive"  # one workgroup per CU: nothing runs beside it
        if not bool(o.lstm_persist_supported(self.H, B)):
            return plan
        H, cus, grid = self.H, int(o.num_cus()), int(o.lstm_persist_grid(self.H, B))
        vdew = self.V if (training and self.V <= 128) else 0

        def occ(bwd, flags, v=0):
            return int(o.lstm_persist_occupancy(bwd, H, B, v, flags))

        def fits(bwd, flags, margin=0):
            return all(grid <= (occ(bwd, flags, v) - margin) * cus for v in {0, vdew})

        fwd_flags = PF_GRANULE if self.handoff == "granule" else 0
        if not (fits(0, fwd_flags) and (not training or fits(1, 0))):
            return plan
        plan["persist"] = True
        plan["xfuse"] = (os.environ.get("DCR_XFUSE", "1") != "0"
                         and bool(o.lstm_persist_xfuse_supported(H, B)))
        if not training:
            return plan
        shared_ok = fits(1, 0, margin=1)
        excl_ok = fits(1, PF_EXCL)
        forced = os.environ.get("DCR_MODE", "")
        if forced == "overlap" and shared_ok:
            mode = "overlap"
        elif forced == "exclusive":
            mode = "exclusive"
        elif excl_ok:
            mode = "exclusive"
        else:
            mode = "overlap" if (shared_ok and self.side_overlap) else "exclusive"
        if plan["pair_bwd"]:
            mode = "exclusive"  # one workgroup per CU (register-bound): nothing runs beside it
        plan["mode"] = mode
        plan["bwd_excl"] = mode == "exclusive" and excl_ok
        return plan

    def check_errors(self):
        """Raise if a persistent kernel hit its spin timeout (forces a device sync).  The word
        is cleared so the caller may recover (e.g. restore a checkpoint and continue)."""
        v = int(self.err.item())
        if v:
            self.err.zero_()
            if self._err_host is not None:
                self._err_host.zero_()
            raise RuntimeError(f"persistent recurrent kernel timed out (code {v}); the "
                               "optimizer skipped the step's update.  Another process sharing "
                               "this GPU can cause this (one rank per GPU); DCR_PERSIST=0 "
                               "selects the per-step kernels")

    def _dropout(self, training: bool) -> bool:
        c = self.cfg
        return training and (c.input_keep_prob < 1.0 or c.output_keep_prob < 1.0)

    def _drop_masks(self, T: int, B: int) -> dict:
        """This step's dropout masks as bits (csrc/dropout.hip), drawn once per training step.

        DropoutWrapper(input_keep_prob, output_keep_prob) around every layer plus the
        embedding dropout with output_keep_prob (model.py:31-34, 58-59; A-13) compose into ONE
        mask per layer input -- layer 0: embedding x input dropout, layer l > 0: layer l-1's
        output dropout x layer l's input dropout; independent Bernoulli draws multiply, so each
        is one draw with keep = output_keep_prob * input_keep_prob -- and one on the top
        layer's output (keep = output_keep_prob).  The persistent pair kernels read their
        fragments' bits in-kernel; the other routes use ``ops.mask_apply``."""
        c = self.cfg
        p_in = float(c.output_keep_prob) * float(c.input_keep_prob)
        p_out = float(c.output_keep_prob)
        key = (T, B)
        m = self._dm_bufs.get(key)
        if m is None:
            nb = lambda: torch.empty(T, B, self.H // 8, dtype=torch.uint8, device=self.dev)  # noqa: E731
            m = self._dm_bufs[key] = dict(
                inb=[nb() for _ in range(self.L)] if p_in < 1.0 else [None] * self.L,
                out=nb() if p_out < 1.0 else None)
        self._drop_step += 1
        stream = self._drop_step << 8
        for layer, bits in enumerate(m["inb"]):
            if bits is not None:
                self.ops.dropout_bits(bits, self._drop_seed, stream + layer, p_in)
        if m["out"] is not None:
            self.ops.dropout_bits(m["out"], self._drop_seed, stream + 255, p_out)
        dm = dict(inb=m["inb"], out=m["out"], sin=1.0 / p_in, sout=1.0 / p_out)
        self.last_dropout_masks = dm
        return dm

    def _masked(self, x: torch.Tensor, bits: Optional[torch.Tensor], scale: float,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """x ⊙ mask · scale over [N, K] rows (time-major, as the bits); ``out`` may be ``x``."""
        if bits is None:
            return x
        N, K = bits.shape[0] * bits.shape[1], bits.shape[2] * 8
        x2 = x.reshape(N, K)
        o = torch.empty_like(x2) if out is None else out.view(N, K)
        self.ops.mask_apply(x2, bits, scale, o)
        return o

    # ------------------------------------------------------------------ forward
    def _forward(self, ids_tm: torch.Tensor, state, training: bool, want_logits: bool = True,
                 logits_bias: bool = True):
        T, B = ids_tm.shape
        H, N = self.H, T * B
        tasks = self._prep()
        bufs = self._buffers(B, T, training)
        drop = self._dropout(training)
        dm = self._drop_masks(T, B) if drop else None
        # initial state into slot 0 of the sequence buffers, hand-off counters zeroed: all in
        # the same prep launch as the weight layouts
        for layer in range(self.L):
            lb, st = bufs["layers"][layer], state[layer]
            pairs = ([(st[0], lb.cbuf[0]), (st[1], lb.hbuf[0])] if self.cfg.model in ("lstm", "nas")
                     else [(st[0], lb.hbuf[0])] + ([(st[0], lb.h32[0])] if lb.h32 is not None else []))
            for src, dst in pairs:
                if src.dtype == f32 and src.dim() == 2 and src.stride(1) == 1:
                    tasks.append((src, dst, 0))
                else:
                    dst.copy_(src)
        if bufs["persist"] or bufs["pair"] or bufs["gru_persist"] or bufs["big_fwd"]:
            tasks.append((bufs["cnt"], bufs["cnt"], 2))
        self._run_prep(tasks)
        # the persistent LSTM kernels write the final (c, h) straight into fresh tensors that
        # become the returned TBPTT state (no copies of cbuf[T] / hlast32 afterwards)
        fresh = bufs["pers_layers"] if self.cfg.model == "lstm" else set()
        for layer in fresh:
            lb = bufs["layers"][layer]
            lb.hlast32 = torch.empty(B, H, dtype=f32, device=self.dev)
            lb.clast32 = torch.empty(B, H, dtype=f32, device=self.dev)
        x_prev = None  # bf16 [T, B, H] input for the next layer
        paired = -1  # layer already computed by the previous layer's two-layer wavefront
        for layer in range(self.L):
            if layer == paired:
                continue
            lw, lb = self._w[layer], bufs["layers"][layer]
            gather = (layer == 0 and not drop and self.cfg.model != "nas")
            ids_arg = None
            # the forward never has a concurrent kernel (the previous step's all-reduce is joined
            # before the optimizer), so the one-workgroup-per-CU fused variant is safe here
            xfuse = (bufs["persist"] and layer > 0 and not drop and lw.WxT is not None
                     and bufs["xfuse"])
            if xfuse:
                lb.x_in = x_prev.reshape(N, H)
                self.ops.lstm_persist_fwd(lw.WhT, lw.bias, None, lb.hbuf, lb.cbuf, lb.gates,
                                          lb.hlast32, bufs["cnt"][layer], self.err, FORGET_BIAS,
                                          self.spin_limit, None, None, lw.WxT, x_prev, lw.bias,
                                          cnt_zeroed=True,
                                          hring=bufs["hrings"][0] if bufs["hrings"] else None,
                                          clast32=lb.clast32)
                x_prev = lb.hbuf[1:]
                continue
            if gather:
                zx = self._head["table"]
                ids_arg = ids_tm
            else:
                inb = dm["inb"][layer] if dm else None
                if layer == 0:  # the embedding rows (masked: embedding x input dropout)
                    X = lb.x_drop if inb is not None else torch.empty(N, H, dtype=bf16,
                                                                      device=self.dev)
                    self.ops.embed_dropout(ids_tm.reshape(-1), self._head["E"], inb,
                                           dm["sin"] if dm else 1.0, X)
                else:
                    X = x_prev.reshape(N, H)
                    if inb is not None:
                        X = self._masked(X, inb, dm["sin"], out=lb.x_drop)
                lb.x_in = X if X.is_contiguous() else X.contiguous()
                _mm_into(lb.x_in, lw.Wx, lb.zx.view(N, self.GW), bias=lw.bias)
                zx = lb.zx
            if bufs["pair"] and layer + 1 < self.L:
                # layers (l, l+1) as one wavefront launch (lstm2_persist.hip): T+1 ticks; layer
                # l+1's input dropout is applied to its fragments in-kernel
                lw1, lb1 = self._w[layer + 1], bufs["layers"][layer + 1]
                xm = dm["inb"][layer + 1] if dm else None
                self.ops.lstm2_persist_fwd(lw.WhT, lw1.WhT, lw1.WxT, zx, ids_arg, lw1.bias,
                                           lb.hbuf, lb.cbuf, lb.gates, lb.hlast32,
                                           lb1.hbuf, lb1.cbuf, lb1.gates, lb1.hlast32,
                                           bufs["cnt"][layer], bufs["cnt"][layer + 1], self.err,
                                           FORGET_BIAS, self.spin_limit, *bufs["hrings"],
                                           bufs["pair_g"], lb.clast32, lb1.clast32, None, xm,
                                           dm["sin"] if dm else 1.0)
                # layer l+1's (masked) input rows for its weight gradient
                lb1.x_in = (self._masked(lb.hbuf[1:], xm, dm["sin"], out=lb1.x_drop)
                            if xm is not None else lb.hbuf[1:].reshape(N, H))
                x_prev = lb1.hbuf[1:]
                paired = layer + 1
                continue
            if bufs["persist"]:
                self.ops.lstm_persist_fwd(lw.WhT, zx, ids_arg, lb.hbuf, lb.cbuf, lb.gates,
                                          lb.hlast32, bufs["cnt"][layer], self.err, FORGET_BIAS,
                                          self.spin_limit,
                                          bufs["ring"] if self.handoff == "granule" else None,
                                          cnt_zeroed=True,
                                          hring=(bufs["hrings"][0] if bufs["hrings"]
                                                 and self.handoff != "granule" else None),
                                          clast32=lb.clast32)
            elif bufs["big_fwd"]:
                self.ops.lstm_big_fwd(lw.WhT, zx, ids_arg, lb.hbuf, lb.cbuf, lb.gates,
                                      lb.hlast32, bufs["cnt"][layer], self.err, FORGET_BIAS,
                                      self.spin_limit, bufs["hrings"][0], cnt_zeroed=True)
            elif bufs["gru_persist"]:
                gr = bufs["grings"]
                self.ops.gru_persist_fwd(lw.WhT, lw.WT2, zx, ids_arg, lb.hbuf, lb.h32, lb.rh,
                                         lb.gates, None, bufs["cnt"][layer], self.err,
                                         self.spin_limit, cnt_zeroed=True,
                                         ring0=gr[0] if gr else None, ring1=gr[1] if gr else None)
            elif self._lib_step("fwd", B):
                self._lstm_fwd_lib(lw, lb, zx, ids_arg, bufs)
            else:
                self.ops.rnn_fwd_seq(self.cell, lw.WhT, lw.WT2, zx, ids_arg, lb.hbuf, lb.h32,
                                     lb.cbuf, lb.gates, lb.pre, lb.aux, lb.rh, lb.hlast32,
                                     FORGET_BIAS)
            x_prev = lb.hbuf[1:]
        O = x_prev.reshape(N, H)
        if dm is not None and dm["out"] is not None:  # the top layer's output dropout
            O = self._masked(O, dm["out"], dm["sout"], out=bufs["o_drop"])
        if not O.is_contiguous():
            O = O.contiguous()
        logits = bufs["logits"]
        if want_logits:
            # the wide-vocabulary CE adds the bias itself: a bias-initialised GEMM output would
            # cost an extra [N, V] fp32 broadcast copy (1 GB at V = 8192)
            _mm_into(O, self._head["Ws"], logits, bias=self._head["bs"] if logits_bias else None)
        new_state = []
        for layer in range(self.L):
            lb = bufs["layers"][layer]
            if self.cfg.model in ("lstm", "nas"):
                new_state.append((lb.clast32, lb.hlast32) if layer in fresh
                                 else (lb.cbuf[T].clone(), lb.hlast32.clone()))
            elif self.cfg.model == "gru":
                new_state.append((lb.h32[T].clone(),))
            else:
                new_state.append((lb.hlast32.clone(),))
        return bufs, O, logits, new_state

    # ------------------------------------------------------------------ training step
    def train_step(self, x, y, state, on_ready=None, want_extras: bool = False):
        ids_tm = x.t().contiguous()
        tgt = y.t().contiguous().view(-1)
        T, B = ids_tm.shape
        H, V, N, GW = self.H, self.V, T * B, self.GW
        wide = self._wide_xent(T * B)
        bufs, O, logits, new_state = self._forward(ids_tm, state, True,
                                                   want_logits=not self.fused_head,
                                                   logits_bias=not wide)
        dlog = bufs["dlogits"]
        s, hd = self.store, self._head
        if self.fused_head:
            # one launch: logits (only if asked for) -> CE -> bf16 dlogits, d softmax_b, dtop
            self.ops.head(O, hd["WsT"], hd["Wsk"], hd["bs"], tgt, 1.0 / N,
                          logits if want_extras else None, bufs["row_loss"], dlog,
                          bufs["dtop"].view(N, H), s.gview("rnnlm/softmax_b"),
                          bufs["head_part"], bufs["loss"])
            _mm_tn(O, dlog, s.gview("rnnlm/softmax_w"))
            dtop = bufs["dtop"].view(T, B, H)
        elif wide:
            # wide vocabulary: one-read CE (bias added in-kernel), d softmax_b fused (xent_wide)
            self.ops.xent_wide(logits, hd["bs"], tgt, 1.0 / N, bufs["row_loss"], dlog,
                               bufs["colpart"], s.gview("rnnlm/softmax_b"), bufs["xpart"],
                               bufs["loss"])
            if want_extras:
                logits += hd["bs"]
            _mm_tn(O, dlog, s.gview("rnnlm/softmax_w"))
            dtop = _mm_into(dlog, hd["Ws"].t(), bufs["dtop"].view(N, H)).view(T, B, H)
        else:
            self.ops.xent(logits, tgt, 1.0 / N, bufs["row_loss"], dlog, bufs["xpart"],
                          bufs["loss"])
            # ---- head gradients
            _mm_tn(O, dlog, s.gview("rnnlm/softmax_w"))
            self.ops.segsum(dlog, None, 1, bufs["colsum"][:, :V], bufs["ws"], False)
            s.gview("rnnlm/softmax_b").copy_(bufs["colsum"][0, :V])
            dtop = _mm_into(dlog, hd["Ws"].t(), bufs["dtop"].view(N, H)).view(T, B, H)
        persistent = bufs["persist"] or bufs["pair"] or bufs["gru_persist"]
        overlap = bufs["mode"] == "overlap" or not persistent
        pending = []
        user_ready = None
        if on_ready is not None and not overlap:
            # exclusive mode: nothing may run beside the persistent BPTT grids, so the gradient
            # buckets are released (in the same order) only after the last BPTT launch; from
            # then on readiness is forwarded directly (the remaining weight GEMMs overlap RCCL)
            user_ready = on_ready
            on_ready = pending.append

        def _release():
            for off in pending:
                user_ready(off)
            pending.clear()
            return user_ready
        if on_ready is not None:
            sb = s.by_name["rnnlm/softmax_b"]
            on_ready(sb.offset + sb.numel)
        drop = self._dropout(True)
        dm = self.last_dropout_masks if drop else None
        deferred = []
        paired_done = -1  # lower layer whose BPTT already ran inside a two-layer wavefront
        # TF clip-norm term from dx_tok = dZ0·W_x0ᵀ: needed as an extra GEMM only on the layer-0
        # gather route (every other route materialises dx_tok anyway)
        gather0 = not drop and self.cfg.model != "nas"
        fused_dew0 = bufs["persist"] and gather0 and V <= 128 and self.fused_dew
        tok_gemm = self.tf_norm and gather0 and not (V > SEG_LDS_MAX_V and not fused_dew0)
        for layer in reversed(range(self.L)):
            lw, lb = self._w[layer], bufs["layers"][layer]
            names = [sp.name for sp in cell_specs(self.cfg, layer)]
            pair_hi = bufs["pair_bwd"] and layer % 2 == 1 and dtop is not None
            # the top layer's output dropout
            omask = dm["out"] if (dm is not None and layer == self.L - 1) else None
            if dtop is not None:
                dtop = dtop.contiguous()
                if omask is not None:
                    dtop = self._masked(dtop, omask, dm["sout"], out=dtop).view(T, B, H)
            zx_nas = lb.zx if self.cfg.model == "nas" else None
            written = False  # this layer's kernel/bias gradients already in the flat buffer
            gather = (layer == 0 and not drop and self.cfg.model != "nas")
            fused_dew = bufs["persist"] and gather and V <= 128 and self.fused_dew
            if pair_hi:
                # layers (layer-1, layer) as one reverse wavefront (lstm2_persist.hip): T+1
                # ticks, the lower layer's dtop = dZ·W_xᵀ of this layer computed in-kernel
                lo = layer - 1
                lw0, lb0 = self._w[lo], bufs["layers"][lo]
                nr = bufs["pair_rows"]
                self.ops.lstm2_persist_bwd(lw0.Wh, lw.Wh, lw.Wx, dtop, lb0.gates, lb0.cbuf,
                                           lb.gates, lb.cbuf, lb0.dz, lb.dz, bufs["zring"],
                                           bufs["zring2"], bufs["db_part"][lo][:nr],
                                           bufs["db_part"][layer][:nr], bufs["cnt"][self.L + lo],
                                           bufs["cnt"][self.L + layer], self.err,
                                           self.spin_limit, bufs["pair_g"], None,
                                           dm["inb"][layer] if dm else None,
                                           dm["sin"] if dm else 1.0)
                paired_done = lo
                if lo == 0 and user_ready is not None:
                    on_ready = _release()
            elif layer == paired_done:
                pass
            elif bufs["persist"]:
                above = None
                if dtop is None:  # dtop of this layer is fused: dZ_above · W_x,aboveᵀ in-kernel
                    above = (self._w[layer + 1].Wx, bufs["layers"][layer + 1].dz)
                self.ops.lstm_persist_bwd(lw.Wh, dtop if dtop is not None else bufs["dtop"],
                                          lb.dz, lb.gates, lb.cbuf, bufs["cnt"][self.L + layer],
                                          self.err, self.spin_limit,
                                          bufs["db_part"][layer][: max(B // 16, 1)],
                                          ids_tm if fused_dew else None,
                                          bufs["dew_part"] if fused_dew else None, V, None,
                                          above[0] if above else None,
                                          above[1] if above else None,
                                          exclusive=bufs["bwd_excl"] and above is None,
                                          cnt_zeroed=True, zring=bufs["zring"])
                if layer == 0 and user_ready is not None:
                    # the last persistent grid is queued: buckets may now run beside the
                    # (non-persistent) layer-0 weight GEMMs
                    on_ready = _release()
            elif bufs["gru_persist"]:
                gr = bufs["grings"]
                self.ops.gru_persist_bwd(lw.W2, lw.Wh, dtop, lb.dz, lb.gates, lb.h32,
                                         bufs["cnt"][self.L + layer], self.err, self.spin_limit,
                                         cnt_zeroed=True, ring0=gr[0] if gr else None,
                                         ring1=gr[2] if gr else None)
                if layer == 0 and user_ready is not None:
                    on_ready = _release()
            elif self._lib_step("bwd", B):
                self._lstm_bwd_lib(lw, lb, dtop, bufs)
            else:
                self.ops.rnn_bwd_seq(self.cell, lw.Wh, lw.W2, dtop, lb.dz, lb.dzx, lb.gates,
                                     lb.pre, lb.aux, zx_nas, lb.cbuf, lb.h32, lb.hbuf, bufs["dc"],
                                     bufs["gpart"])
            dZ = lb.dz.view(N, GW)
            dZx = lb.dzx.view(N, GW) if lb.dzx is not None else dZ
            Hprev = lb.hbuf[:T].reshape(N, H)
            if (bufs["persist"] and layer > 0 and not drop and self.fused_dtop and not pair_hi
                    and layer != paired_done and self._exclusive_ok(bufs)):
                # The layer below fuses dtop = dZ·W_xᵀ into its BPTT kernel.  That kernel holds
                # W_h and W_x^{above} in registers (one workgroup per CU, grid = all CUs), so
                # NOTHING may run beside it (a concurrent kernel holding CUs could deadlock the
                # grid's residency): this layer's weight gradients are deferred until after it.
                dbias = self._bias_sum(self._db_part(bufs, layer), names)

                def _wgrads(names=names, Hprev=Hprev, dZ=dZ, dZx=dZx, lb=lb, dbias=dbias,
                            layer=layer):
                    _mm_tn(Hprev, dZ, s.gview(names[0])[H:])
                    _mm_tn(lb.x_in, dZx, s.gview(names[0])[:H])
                    s.gview(names[1]).copy_(dbias)
                    if on_ready is not None:
                        on_ready(s.layer_range(layer)[1])
                deferred.append(_wgrads)
                dtop = None
                continue
            if (bufs["persist"] and layer > 0 and not drop and self.side_overlap and overlap
                    and not pair_hi):
                # Off the critical path: this layer's weight gradients (two [H x N]·[N x 4H]
                # GEMMs) run on a side stream concurrently with the latency-bound BPTT of the
                # layer below; the layer's all-reduce bucket is launched from that stream, so
                # RCCL orders itself after the GEMMs.  Only dX stays on the critical path.
                dbias = self._bias_sum(self._db_part(bufs, layer), names)
                ev = torch.cuda.Event()
                ev.record()
                side = self._side_stream()
                with torch.cuda.stream(side):
                    side.wait_event(ev)
                    _mm_tn(Hprev, dZ, s.gview(names[0])[H:], split=False)
                    _mm_tn(lb.x_in, dZx, s.gview(names[0])[:H], split=False)
                    s.gview(names[1]).copy_(dbias)
                    dbias.record_stream(side)
                    if on_ready is not None:
                        on_ready(s.layer_range(layer)[1])
                dtop = _mm_into(dZx, lw.Wx.t(), bufs["dx"].view(N, H)).view(T, B, H)
                self._side_used = True
                continue
            for fn in deferred:  # weight grads of the layers above (after the fused BPTT)
                fn()
            deferred.clear()
            # recurrent-weight gradients
            if self.cfg.model == "gru":
                gk, gb, ck, cb = names
                _mm_tn(Hprev, dZ[:, : 2 * H], s.gview(gk)[H:])
                _mm_tn(lb.rh.view(N, H), dZ[:, 2 * H:], s.gview(ck)[H:])
            elif self.cfg.model == "nas":
                _mm_tn(Hprev, dZ, s.gview(names[1]))
            else:
                _mm_tn(Hprev, dZ, s.gview(names[0])[H:])
            if gather and V > SEG_LDS_MAX_V and not fused_dew:
                # wide vocabulary: the [V, GW] dEW segment sum would be an atomic scatter of
                # N x GW values plus two fp32 [V, GW] GEMMs; the dense route scatters N x H
                # instead: dW_x0 = E[ids]ᵀ·dZ0 (split-K), dE = segsum(dZ0·W_x0ᵀ)
                Eb = hd.get("Ebf")                                  # refreshed with the table
                X0 = (Eb[ids_tm.view(-1).long()] if Eb is not None
                      else hd["E"][ids_tm.view(-1).long()].to(bf16))    # [N, H]
                dWx = _mm_tn(X0, dZx)
                if layer in bufs["pers_layers"]:
                    dbias = self._bias_sum(self._db_part(bufs, layer), names)
                else:
                    self.ops.segsum(dZx, None, 1, bufs["colsum"][:, :GW], bufs["ws"], False)
                    dbias = bufs["colsum"][0, :GW]
                dXf = _mm_into(dZx, lw.Wx.t(), bufs["dx"].view(N, H))
                self._embed_grad(dXf, ids_tm, bufs)
                self._token_norm(dXf)
            elif gather:
                if fused_dew:
                    dEW = bufs["dew_part"].sum(0)            # [V, GW] fp32 (fused in BPTT)
                elif self.dew_mode == "gemm" and bufs["onehot"] is not None:
                    # exact 1.0 one-hot entries: the same fp32 sums of the bf16 dZ values as a
                    # scatter, as one split-K MFMA GEMM (K = T·B tokens)
                    oh = bufs["onehot"]
                    oh.zero_()
                    oh.scatter_(1, ids_tm.view(-1, 1).long(), 1.0)
                    dEW = _mm_tn(oh, dZx)[:V]                 # rows >= V are zero padding
                else:
                    dEW = torch.empty(V, GW, dtype=f32, device=self.dev)
                    self.ops.segsum(dZx, ids_tm.view(-1), V, dEW, bufs["ws"], False)
                dWx = hd["E"].t() @ dEW                      # [H, GW] fp32
                dbias = dEW.sum(0)
                # layer 0's own gradients are final here: report them before the embedding
                # gradient and the token-norm GEMM, so that under data parallelism the
                # layer-0 bucket's all-reduce overlaps that work and the last bucket is only
                # the embedding + norm slot
                self._write_input_grads(layer, names, dWx, dbias)
                written = True
                if on_ready is not None:
                    self._join_side()
                    on_ready(s.layer_range(0)[1])
                torch.mm(dEW, lw.Wx32.t(), out=s.gview("embedding"))
                if tok_gemm:
                    self._token_norm_gemm(dZx, lw.Wx)
            else:
                dWx = (_mm_tn(lb.x_in, dZx, s.gview(names[0])[:H])
                       if self.cfg.model in ("lstm", "rnn") else _mm_tn(lb.x_in, dZx))
                if layer in bufs["pers_layers"]:
                    dbias = self._bias_sum(self._db_part(bufs, layer), names)  # fused in BPTT
                else:
                    self.ops.segsum(dZx, None, 1, bufs["colsum"][:, :GW], bufs["ws"], False)
                    dbias = bufs["colsum"][0, :GW]
                if pair_hi:  # the lower layer's dtop was fused into the wavefront BPTT
                    self._write_input_grads(layer, names, dWx, dbias)
                    if on_ready is not None:
                        on_ready(s.layer_range(layer)[1])
                    dtop = None
                    continue
                if layer > 0:
                    dX = _mm_into(dZx, lw.Wx.t(), bufs["dx"].view(N, H)).view(T, B, H)
                else:  # only the embedding gradient reads it: bf16 rows for the segment sum
                    dX = torch.mm(dZx, lw.Wx.t(), out=bufs["dx_bf"]).view(T, B, H)
                if dm is not None and dm["inb"][layer] is not None:  # this layer's input mask
                    dX = self._masked(dX, dm["inb"][layer], dm["sin"], out=dX).view(T, B, H)
                if layer > 0:
                    dtop = dX
                else:
                    # (bf16 as the GEMM wrote it: the segment sum and the norm accumulate in
                    # fp32 either way; an fp32 copy would only add a pass over [N, H])
                    dXt = dX.reshape(N, H)
                    self._embed_grad(dXt, ids_tm, bufs)
                    self._token_norm(dXt)
            if not written:
                self._write_input_grads(layer, names, dWx, dbias)
            if layer == 0:
                # side-stream work (overlapped weight GEMMs of the layers above) may share the
                # remaining buckets: join before reporting them ready
                self._join_side()
            if on_ready is not None:
                on_ready(None if layer == 0 else s.layer_range(layer)[1])
        self._join_side()
        if pending:
            _release()
        extras = {"logits": logits, "loss": bufs["row_loss"]} if want_extras else None
        self._steps += 1
        if persistent or bufs["big_fwd"]:
            self._poll_errors()
        return bufs["loss"][0], new_state, extras

    def _poll_errors(self) -> None:
        """Non-blocking check of the persistent kernels' error word: each step copies it into
        pinned host memory behind its own work and reads the copy of an earlier step, so a
        spin timeout raises within a step or two without a device sync.  (The optimizer skips
        its update on device while the word is set: TFAdam(guard=err).)"""
        if self._err_host is None:
            self._err_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        v = int(self._err_host[0])
        if v:
            self.check_errors()
        self._err_host.copy_(self.err, non_blocking=True)

    def _embed_grad(self, dXf: torch.Tensor, ids_tm: torch.Tensor, bufs) -> None:
        """dE = segsum(dX_tok, ids) into the gradient buffer.  Wide vocabularies take the
        fp32-atomic route; there the ids are sorted first (a frequent id is then one register
        run per 32-row chunk instead of one atomic per occurrence: 127 -> see BASELINE.md)."""
        ids = ids_tm.view(-1)
        out = self.store.gview("embedding")
        if self.V > SEG_LDS_MAX_V and os.environ.get("DCR_SEG_SORT", "1") != "0":
            sid, perm = torch.sort(ids)
            self.ops.segsum(dXf, sid, self.V, out, bufs["ws"], False, perm.int())
        else:
            self.ops.segsum(dXf, ids, self.V, out, bufs["ws"], False)

    def _token_norm(self, dx_tok: torch.Tensor) -> None:
        """TF clip-norm term of the embedding (ModelConfig.clip_norm == "tf"): the sum of
        squares of the per-token input gradients (the IndexedSlices values), written into the
        gradient buffer's norm slot (all-reduced with the last bucket, read by adam_clip)."""
        if not self.tf_norm:
            return
        n = dx_tok.numel()
        if self._npart is None or self._npart.numel() < self.ops.opt_num_partials(n):
            self._npart = torch.empty(self.ops.opt_num_partials(n), dtype=f32, device=self.dev)
        self.ops.sumsq(dx_tok.contiguous(), self._npart, self.store.norm_slot_view())

    # ------------------------------------------------------------------ large-H library steps
    def _lib_step(self, direction: str, B: int) -> bool:
        """Per-time-step recurrent GEMM on the library path + epilogue-only cell kernel, for
        LSTM with H > 1024 (no weights-resident kernel there).  The fused per-step kernels
        re-read the whole step payload once per 16-unit block (128 x at H = 2048), so their
        step time grows linearly with the batch; a library GEMM reads W_h once per step
        (scripts/bench_step_gemms.py: 17-25 us for B = 64-256).  auto: BPTT always, forward
        from B >= 128 (at B = 64 the fused forward step, 16.7 us, beats GEMM + epilogue).
        DCR_LIBSTEP=0 / 1 forces either way."""
        if self.cfg.model != "lstm":
            return False
        if self.libstep == "0":
            return False
        if self.libstep == "1":
            return True
        if self.H <= 1024:
            return False
        return direction == "bwd" or B >= 128

    def _lstm_fwd_lib(self, lw, lb, zx, ids, bufs) -> None:
        T, B = lb.gates.shape[0], lb.gates.shape[1]
        S = self._step_gemm_splits(B, self.GW, self.H)
        zrec = bufs.get("zrec")
        if zrec is None:
            zrec = bufs["zrec"] = torch.empty(max(S, 1), B, self.GW, dtype=f32, device=self.dev)

        def body(zx, ids):
            for t in range(T):
                if S:  # split-K step GEMM (step_gemm.hip) into S slabs, summed by the cell kernel
                    self.ops.step_gemm(lb.hbuf[t], lw.WhT, zrec)
                else:  # B operand as W_hᵀ-transposed (NT form): 20.7 vs 25.6 us at B = 256
                    torch.mm(lb.hbuf[t], lw.WhT.t(), out_dtype=f32, out=zrec[0])
                self.ops.lstm_step_ew_fwd(zrec, zx if ids is not None else zx[t],
                                          ids[t] if ids is not None else None, lb.cbuf[t],
                                          lb.hbuf[t + 1], lb.hlast32 if t == T - 1 else None,
                                          lb.cbuf[t + 1], lb.gates[t], FORGET_BIAS)

        self._run_lib_loop(bufs, ("fwd", id(lb)), body, zx, ids,
                           a_static=lb.zx is not None and zx.data_ptr() == lb.zx.data_ptr())

    def _lstm_bwd_lib(self, lw, lb, dtop, bufs) -> None:
        T, B = dtop.shape[0], dtop.shape[1]
        S = self._step_gemm_splits(B, self.H, self.GW)
        dh = bufs.get("dhrec")
        if dh is None:
            dh = bufs["dhrec"] = torch.empty(max(S, 1), B, self.H, dtype=f32, device=self.dev)
        dc = bufs["dc"]
        WhT = lw.Wh.t()

        def body(dtop, _unused):
            dc.zero_()
            for t in reversed(range(T)):
                # dh = dtop_t + dZ_{t+1}·W_hᵀ: the GEMM writes the recurrent part, the cell
                # kernel adds dtop_t (an addmm with a 2-D input costs a separate copy launch)
                if t < T - 1 and S:
                    self.ops.step_gemm(lb.dz[t + 1], lw.Wh, dh)
                elif t < T - 1:
                    torch.mm(lb.dz[t + 1], WhT, out_dtype=f32, out=dh[0])
                self.ops.lstm_step_ew_bwd(dtop[t], dh if t < T - 1 else None, lb.gates[t],
                                          lb.cbuf[t + 1], lb.cbuf[t], dc, lb.dz[t])

        static = any(buf is not None and dtop.data_ptr() == buf.data_ptr()
                     for buf in (bufs["dtop"], bufs["dx"]))
        self._run_lib_loop(bufs, ("bwd", id(lb)), body, dtop, None, a_static=static)

    def _run_lib_loop(self, bufs, key, body, a, b, a_static: bool = False) -> None:
        """Run a T-step library loop (2 launches per step) as a replayed hipGraph: eager,
        the per-step host launch cost (~15 us) is as long as the GPU's step at B = 64.  The
        graph is captured on the first call with static copies of the loop's varying inputs
        (a: zx / table / dtop, b: ids) and replayed afterwards; everything else it touches
        (h, c, gates, dZ buffers, the bf16 weights refreshed in place) is persistent.
        ``a_static``: ``a`` is itself a persistent buffer (dense zx, the dtop / dx buffers),
        captured directly instead of through a copy.  DCR_LIB_GRAPH=0 runs eagerly."""
        if os.environ.get("DCR_LIB_GRAPH", "1") == "0":
            body(a, b)
            return
        # the graphs live with the buffers they were captured on (and die with them)
        graphs = bufs.setdefault("lib_graphs", {})
        ent = graphs.get(key)
        if ent is None or ent[1].shape != a.shape or (b is not None and ent[2].shape != b.shape):
            sa = a if a_static else a.clone()
            sb = b.clone() if b is not None else None
            body(sa, sb)  # warm-up outside capture (library handles, workspaces)
            g = torch.cuda.CUDAGraph()
            try:
                s = torch.cuda.Stream(device=self.dev)
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    with torch.cuda.graph(g, stream=s):
                        body(sa, sb)
                torch.cuda.current_stream().wait_stream(s)
            except RuntimeError:
                graphs[key] = ("eager", None, None)
                body(a, b)
                return
            graphs[key] = ent = (g, sa, sb)
        if ent[0] == "eager":
            body(a, b)
            return
        g, sa, sb = ent
        if sa.data_ptr() != a.data_ptr():
            sa.copy_(a)
        if sb is not None and sb.data_ptr() != b.data_ptr():
            sb.copy_(b)
        g.replay()

    def _step_gemm_splits(self, B: int, N: int, K: int) -> int:
        """Split count of the native split-K step GEMM (csrc/step_gemm.hip) for an [B, K] x
        [N, K]ᵀ step product, or 0 to use the library GEMM (the default; DCR_STEP_GEMM=native
        selects the kernel where the shape allows)."""
        if self.step_gemm_mode != "native":
            return 0
        return int(self.ops.step_gemm_splits(B, N, K))

    def _join_side(self) -> None:
        if self._side_used:
            torch.cuda.current_stream().wait_stream(self._side)
            self._side_used = False

    def _token_norm_gemm(self, dz0: torch.Tensor, wx0: torch.Tensor) -> None:
        """sum_tok ||dZ0_tok·W_x0ᵀ||² into the norm slot.  Default: the library GEMM to bf16
        rows + the sumsq kernel (66 us at the headline shape, scripts/bench_tok_norm.py);
        DCR_TOK_NORM=fused: the fused MFMA kernel (optim.hip tok_norm, the [N, H] product never
        materialised, LDS-DMA ring) -- correct, 92 us at 745 TFLOP/s, not yet at the library
        GEMM's ~1 PFLOP/s.  A side-stream overlap with the weight GEMMs was measured slower
        than running in line: both are chip-filling."""
        N, K = dz0.shape
        if self.tok_norm_fused and self.ops.tok_norm_supported(N, wx0.shape[0], K):
            n = (N // 128) * (wx0.shape[0] // 64)  # >= workgroups of any tile choice
            if self._tpart is None or self._tpart.numel() < n:
                self._tpart = torch.empty(n, dtype=f32, device=self.dev)
            self.ops.tok_norm(dz0, wx0, self._tpart, self.store.norm_slot_view())
        else:
            self._token_norm(torch.mm(dz0, wx0.t()))

    @staticmethod
    def _db_part(bufs, layer: int) -> torch.Tensor:
        """The rows of the bias-gradient partials the layer's persistent BPTT kernel wrote."""
        if bufs["pair_bwd"] and layer < 2 * (len(bufs["layers"]) // 2):
            return bufs["db_part"][layer][: bufs["pair_rows"]]
        return bufs["db_part"][layer][: max(bufs["layers"][0].hbuf.shape[1] // 16, 1)]

    def _bias_sum(self, part: torch.Tensor, names) -> torch.Tensor:
        """Sum the per-batch-group bias partials; for cells with one [GW] bias the sum is
        written straight into its gradient slice (the later copy_ is then a no-op)."""
        if self.cfg.model in ("lstm", "rnn"):
            return torch.sum(part, 0, out=self.store.gview(names[1]))
        return part.sum(0)

    def _write_input_grads(self, layer: int, names, dWx: torch.Tensor, dbias: torch.Tensor):
        s, H = self.store, self.H
        if self.cfg.model == "gru":
            gk, gb, ck, cb = names
            s.gview(gk)[:H].copy_(dWx[:, : 2 * H])
            s.gview(ck)[:H].copy_(dWx[:, 2 * H:])
            s.gview(gb).copy_(dbias[: 2 * H])
            s.gview(cb).copy_(dbias[2 * H:])
        elif self.cfg.model == "nas":
            s.gview(names[0]).copy_(dWx)
        else:
            _put(s.gview(names[0])[:H], dWx)
            _put(s.gview(names[1]), dbias)

    # ------------------------------------------------------------------ inference
    @torch.no_grad()
    def step_logits(self, x_t: torch.Tensor, state):
        ids_tm = x_t.t().contiguous()
        bufs, O, logits, new_state = self._forward(ids_tm, state, False)
        T, B = ids_tm.shape
        lg = logits.view(T, B, self.V)[-1].clone()
        return lg, new_state

    @torch.no_grad()
    def eval_loss(self, x, y, state):
        ids_tm = x.t().contiguous()
        tgt = y.t().contiguous().view(-1)
        bufs, O, logits, new_state = self._forward(ids_tm, state, False,
                                                   want_logits=not self.fused_head)
        if self.fused_head:
            hd = self._head
            self.ops.head(O, hd["WsT"], None, hd["bs"], tgt, 1.0, None, None, None, None, None,
                          bufs["head_part"], bufs["loss"])
        else:
            self.ops.xent(logits, tgt, 1.0, None, None, bufs["xpart"], bufs["loss"])
        return bufs["loss"][0].clone(), new_state

    @torch.no_grad()
    def sample_sequence(self, prime_ids, num: int, sampling_type: int, seed: int, num_samples: int,
                        space_id: int = -1, use_graph: bool = True):
        """Device-side autoregressive sampling (model.py:105-140); returns [S][num] ids.

        Every generated character is [recurrent step kernels of all layers, ``dcr::sample_step``]
        (csrc/sample.hip: softmax head + argmax / inverse-CDF draw, the pick written straight
        into the next step's input id).  The step is captured once into a hipGraph and replayed
        ``num - 1`` times, so the loop runs without a host round trip or per-kernel launch
        cost; the host reads the ids once at the end."""
        from ..models.reference import zero_state

        S = num_samples
        if num <= 0:
            return [[] for _ in range(S)]
        if not self.ops.sample_supported(self.V, self.H):
            return self._sample_sequence_torch(prime_ids, num, sampling_type, seed, S, space_id)
        state = zero_state(self.cfg, S, self.dev)
        for cid in prime_ids[:-1]:  # warm the state on prime[:-1] (model.py:107-111)
            x = torch.full((S, 1), cid, dtype=torch.int32, device=self.dev)
            _, state = self.step_logits(x, state)
        i32 = dict(dtype=torch.int32, device=self.dev)
        cur = torch.full((S,), int(prime_ids[-1]), **i32)
        out = torch.zeros(S, num, **i32)
        pos = torch.zeros(S, **i32)
        ctr = torch.zeros(S, **i32)
        st = [tuple(t.clone() for t in layer) for layer in state]
        self._run_prep(self._prep())
        WsT = self._head["Ws"].t().contiguous()            # [V, H] bf16, fixed while sampling
        bs = self._head["bs"]
        seed = int(seed) & ((1 << 63) - 1)

        def one():
            _, O, _, new = self._forward(cur.view(1, S), st, False, want_logits=False)
            self.ops.sample_step(O, WsT, bs, cur, out, pos, ctr, None, None, int(sampling_type),
                                 int(space_id), seed)
            for a, b in zip(st, new):
                for x, y in zip(a, b):
                    x.copy_(y)

        one()  # first character eagerly (also allocates the step's buffers)
        if num > 1:
            graph = None
            if use_graph and os.environ.get("DCR_SAMPLE_GRAPH", "1") != "0":
                try:
                    graph = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(graph):
                        one()
                except RuntimeError:
                    graph = None
            for _ in range(num - 1):
                if graph is not None:
                    graph.replay()
                else:
                    one()
        return out.cpu().tolist()

    @torch.no_grad()
    def _sample_sequence_torch(self, prime_ids, num, sampling_type, seed, S, space_id):
        """Library-op sampling loop for shapes the sampling kernel does not cover."""
        from ..models.reference import zero_state

        state = zero_state(self.cfg, S, self.dev)
        g = torch.Generator(device=self.dev)
        g.manual_seed(int(seed))
        for cid in prime_ids[:-1]:
            x = torch.full((S, 1), cid, dtype=torch.int32, device=self.dev)
            _, state = self.step_logits(x, state)
        cur = torch.full((S, 1), prime_ids[-1], dtype=torch.int32, device=self.dev)
        out = torch.empty(S, num, dtype=torch.int32, device=self.dev)
        for i in range(num):
            logits, state = self.step_logits(cur, state)
            p = torch.softmax(logits, -1)
            cdf = torch.cumsum(p, -1)
            r = torch.rand(S, 1, device=self.dev, generator=g) * cdf[:, -1:]
            pick = torch.searchsorted(cdf, r).clamp_(max=self.V - 1).to(torch.int32)
            if sampling_type == 0:
                pick = p.argmax(-1, keepdim=True).to(torch.int32)
            elif sampling_type == 2:
                am = p.argmax(-1, keepdim=True).to(torch.int32)
                pick = torch.where(cur == space_id, pick, am)
            out[:, i: i + 1] = pick
            cur = pick
        return out.cpu().tolist()
