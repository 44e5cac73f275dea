"""Per-(B, T, training) activation and workspace buffers of the native backend, allocated once
per step shape (HBM is plentiful: 288 GB per MI355X) and reused every step."""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch

from .gemm import bf16, f32
from .layouts import SEG_LDS_MAX_V
from .plan import ExecutionPlan, make_plan


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
    x_merged: bool = False                   # x_in and h_{t-1} interleaved: one dW GEMM


class BuffersMixin:
    def _persist_plan(self, B: int, training: bool, T: int = 1 << 30) -> ExecutionPlan:
        return make_plan(self.ops, self.cfg, self.knobs, B, training, T, self.side_overlap)

    def _buffers(self, B: int, T: int, training: bool) -> dict:
        key = (B, T, training)
        if key in self._bufs:
            return self._bufs[key]
        H, GW, dev, m = self.H, self.GW, self.dev, self.cfg.model
        N = B * T
        plan = self._persist_plan(B, training, T)
        # hand-off rings: the batch padded to whole 32-row groups (pair kernels) / 16-row tiles
        Bp = max(-(-B // 32) * 32, 32 * plan.pair_nbg)
        Bg = -(-B // 64) * 64  # GRU rings: whole groups of up to 4 16-row tiles
        nrow = max(-(-B // 16), plan.pair_rows, 1)
        drop = self._dropout(training)
        layers = []
        for layer in range(self.L):
            dense = layer > 0 or drop
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
            if training and drop:
                lb.x_drop = torch.empty(N, H, dtype=bf16, device=dev)
            layers.append(lb)
        # pair-interleaved h (training, two-layer wavefront forwards): layers (l, l+1) write
        # their h rows into one [T+2, B, 2H] buffer C with row t+1 = [h_l(t), h_l+1(t-1)], i.e.
        # exactly the rows [x_t, h_{t-1}] of layer l+1's kernel [2H, 4H]: its two weight
        # gradients become ONE [2H x 4H] token-reduction GEMM over C (backward.py)
        # (scripts/micro/dw_gemm_forms.py: 3 GEMMs + slab sums 273 us -> 233 us).
        # hbuf_l = C[0:T+1, :, :H], hbuf_l+1 = C[1:T+2, :, H:] (row stride 2H).
        # With dropout, layer l+1's input is the MASKED h_l: the pair forward's mask pass then
        # writes those rows into C's x half instead (mode "x"), layer l+1's h stays in the h
        # half, and layer l's h lives in the x half of a second buffer (the pair kernel wants one
        # row stride for both layers' h).
        pair_h = {}
        if training and plan.pair and m == "lstm" and self.knobs.on("pair_dw"):
            for lo in range(0, 2 * (self.L // 2), 2):
                if lo > 0 and plan.persist and plan.xfuse and not drop:
                    continue  # forward.py runs these layers on the fused single-layer kernels
                C = torch.empty(T + 2, B, 2 * H, dtype=bf16, device=dev)
                layers[lo + 1].hbuf = C[1:T + 2, :, H:]
                if drop:
                    C0 = torch.empty(T + 1, B, 2 * H, dtype=bf16, device=dev)
                    layers[lo].hbuf = C0[:, :, :H]
                    layers[lo + 1].x_drop = C[1:T + 1, :, :H].reshape(N, H)
                    pair_h[lo + 1] = (C, "x")
                else:
                    layers[lo].hbuf = C[0:T + 1, :, :H]
                    pair_h[lo + 1] = (C, "h")
        ws = max(self.ops.segsum_workspace(N, GW, self.V), self.ops.segsum_workspace(N, H, self.V),
                 self.ops.segsum_workspace(N, GW, 1), self.ops.segsum_workspace(N, self.V, 1), 1)
        e = lambda *shape, dt=f32: torch.empty(*shape, dtype=dt, device=dev)  # noqa: E731
        bufs = dict(
            plan=plan,
            layers=layers,
            pair_h=pair_h,
            logits=e(N, self.V),
            dlogits=e(N, self.V, dt=bf16) if training else None,
            dlogits_pad=None,
            row_loss=e(N),
            xpart=e(self.ops.xent_num_partials(N)),
            loss=e(2, 4),  # two 16-B slots, ping-pong by step parity (see train_step)
            dc=e(B, H),
            gpart=e(B, H) if m == "gru" else None,
            ws=e(ws),
            colsum=e(1, max(GW, self.V)),
            head_part=e(self.ops.head_workspace(N, self.V)) if self.fused_head else None,
            # fused wide head: per-workgroup loss partials and d softmax_b column partials
            hw_part=e(self.ops.head_wide_workspace(N)) if self.wide_head else None,
            hw_colpart=(e(self.ops.head_wide_colpart_rows(N) * self.V)
                        if (training and self.wide_head) else None),
            onehot=(e(N, 8 * ((self.V + 7) // 8), dt=bf16)
                    if (training and self.V <= SEG_LDS_MAX_V and self.dew_mode == "gemm")
                    else None),
            dew=(e(8 * ((self.V + 7) // 8), GW)
                 if (training and self.V <= SEG_LDS_MAX_V and self.dew_mode == "gemm") else None),
            # time-major ids / targets of the batch, written by the step's prep launch
            ids_tm=torch.empty(T, B, dtype=torch.int32, device=dev) if training else None,
            tgt_tm=torch.empty(T, B, dtype=torch.int32, device=dev) if training else None,
            colpart=(e(self.ops.xent_wide_waves(N) * self.V)
                     if (training and self._wide_xent(N)) else None),
            dtop=e(T, B, H) if training else None,
            dx=e(T, B, H) if training else None,
            dx_bf=e(N, H, dt=bf16) if training else None,
            db_part=e(self.L, nrow, GW) if training else None,
            dew_part=(e(-(-B // 16), self.V, GW)
                      if (training and self.V <= 128 and self.dew_mode == "fused") else None),
            # one hand-off counter region per persistent launch (fwd layers, then bwd layers),
            # zeroed together by the step's prep launch
            cnt=torch.zeros(2 * self.L, max(2 * (B // 16 + 1), plan.pair_nbg) * (T + 1) * 4,
                            dtype=torch.int32, device=dev),
            # fragment-tiled hand-off rings of the persistent GRU: [h or dZc, r⊙h, dZg], sized
            # for the batch padded to whole 64-row groups (a ragged batch's padded rows live
            # only in the rings)
            grings=((e(2 * Bg * H, dt=bf16), e(2 * Bg * H, dt=bf16), e(2 * Bg * 2 * H, dt=bf16))
                    if m == "gru" else None),
            # fragment-tiled h hand-off rings of the persistent forwards (persist_common.h)
            hrings=(e(2 * Bp * H, dt=bf16), e(2 * Bp * H, dt=bf16)) if m == "lstm" else None,
            # fragment-tiled dZ hand-off rings of the persistent BPTTs (one per layer of a pair)
            zring=e(2 * Bp * GW, dt=bf16) if (training and m == "lstm") else None,
            zring2=e(2 * Bp * GW, dt=bf16) if plan.pair_bwd else None,
            o_drop=e(N, H, dt=bf16) if (training and drop) else None,
            # fp32 partial ring of the reduce-scatter pair BPTT (csrc/lstm2_bwd_rs.hip; no
            # dropout; opt-in DCR_DEBUG=bwd_rs=1: slower than the all-gather kernel)
            prs=(e(int(self.ops.lstm2_bwd_rs_ring_floats(H, B)))
                 if (plan.pair_bwd and not drop and m == "lstm"
                     and self.knobs.dbg("bwd_rs", "0") == "1"
                     and bool(self.ops.lstm2_bwd_rs_ok(H, B))) else None),
        )
        if training and self.fused_head and self.V <= 256 and self.knobs.on("dws_wgrad"):
            # the fused head writes its bf16 dlogits into rows of 256 whose other columns stay
            # zero: the softmax_w gradient Oᵀ·dlogits is then a [H x 256] problem of the step's
            # wgrad launch (backward.py) instead of a library GEMM of its own
            bufs["dlogits_pad"] = torch.zeros(N, 256, dtype=bf16, device=dev)
            bufs["dlogits"] = bufs["dlogits_pad"][:, : self.V]
        # layers run by the persistent LSTM kernels (their final state is written into fresh
        # tensors, their bias gradients come from the kernels' db_part partials)
        npair = 2 * (self.L // 2) if plan.pair else 0
        bufs["pers_layers"] = set(range(npair)) | (set(range(npair, self.L)) if plan.persist
                                                   else set())
        # layers whose BPTT kernel writes bias-gradient partials (db_part)
        bufs["bpart_layers"] = (bufs["pers_layers"] if plan.persist_bwd
                                else set(range(npair)))
        if (m == "gru" and training and getattr(plan, "gru_persist", False)
                and self.knobs.on("gru_bpart")):
            # the persistent GRU BPTT writes its bias partials too (csrc/gru_persist.hip)
            bufs["bpart_layers"] = set(range(self.L))
        self._bufs[key] = bufs
        return bufs

    def _wide_xent(self, N: int) -> bool:
        """Library logits GEMM + one-read CE kernel (xent_wide) for vocabularies the fused head
        does not cover (V > 256) when the fused wide head does not either."""
        return (not self.fused_head and not self.wide_head and self.V >= 256 and self.knobs.on("wide_xent")
                and bool(self.ops.xent_wide_supported(self.V)))

    def _side_stream(self):
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.dev)
        return self._side

    @staticmethod
    def _db_part(bufs, layer: int) -> torch.Tensor:
        """The rows of the bias-gradient partials the layer's persistent BPTT kernel wrote."""
        P = bufs["plan"]
        if P.pair_bwd and layer < 2 * (len(bufs["layers"]) // 2):
            return bufs["db_part"][layer][: P.pair_rows]
        return bufs["db_part"][layer][: -(-bufs["layers"][0].hbuf.shape[1] // 16)]

    def _bias_sum(self, part: torch.Tensor, names, q=None) -> torch.Tensor:
        """Sum the per-batch-group bias partials; for cells with one [GW] bias the sum is
        written straight into its gradient slice (the later copy_ is then a no-op), deferred
        to the queue's next flush when one is given (gemm.SumQueue)."""
        if self.cfg.model in ("lstm", "rnn"):
            if q is not None:
                return q.add_colsum(part, self.store.gview(names[1]))
            return torch.sum(part, 0, out=self.store.gview(names[1]))
        if self.cfg.model == "gru":
            # [r | u] columns -> the gates bias, [c] -> the candidate bias; written here (None:
            # nothing left for _write_input_grads to copy)
            H = self.H
            gb, cb = self.store.gview(names[1]), self.store.gview(names[3])
            if q is not None:
                q.add_colsum(part[:, : 2 * H], gb)
                q.add_colsum(part[:, 2 * H:], cb)
            else:
                torch.sum(part[:, : 2 * H], 0, out=gb)
                torch.sum(part[:, 2 * H:], 0, out=cb)
            return None
        return part.sum(0)
