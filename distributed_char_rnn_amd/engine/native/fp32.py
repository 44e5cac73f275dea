"""Native fp32 execution (``--dtype fp32`` on a GPU): the reference's fp32 graph (model.py:43-98)
with every recurrent cell step -- forward and BPTT -- on the fp32-operand HIP kernels of
csrc/cell_f32.hip (v_mfma_f32_16x16x4_f32: exact fp32 products, fp32 state, activation cache
and gradients), instead of the bf16-operand kernels of the default path.

What it is for: the bf16 kernels round every MFMA operand, so their distance from the fp32
oracle mixes operand rounding with any kernel error; this path computes the same cells with no
rounding, so a disagreement between it and the oracle (≤ 1e-4 relative, tests/test_fp32.py) is
a kernel bug, and one between it and the bf16 path is rounding.  It is a numerics mode, not the
fast path (fp32 MFMA runs at 1/16 of the bf16 rate).

Layout of a layer (LSTM / GRU / BasicRNN; NAS stays on the autograd oracle):
* the input projection of all T steps, X·W_x + b, is one library fp32 GEMM (autograd);
* the recurrence is one autograd Function whose forward / backward are the C++ time loops over
  the per-step kernels (ops ``f32_fwd_seq`` / ``f32_bwd_seq``); its backward returns dZ (the
  input projection's gradient, from which autograd forms dW_x, db and dX) and the recurrent
  weight gradient as one [H, T·B] x [T·B, GW] GEMM;
* embedding, dropout, the head, the loss, the TF clip-norm term and the gradient write-out are
  the oracle's (models/reference.py ReferenceBackend), so the two differ only in the cells.
"""
from __future__ import annotations

from typing import Optional

import torch

from ...models.params import ModelConfig, ParamStore
from ...models.reference import LSTM_FORGET_BIAS, ReferenceBackend, State, _dropout, layer_weights

CELL_IDS = {"lstm": 0, "gru": 1, "rnn": 3}  # csrc/kernels.h CellKind (GRU = CELL_GRU_A)


def supported(cfg: ModelConfig) -> bool:
    return cfg.model in CELL_IDS and cfg.rnn_size % 16 == 0


class _Recurrence(torch.autograd.Function):
    """zx [T, B, GW] (input projection + bias), initial state -> outputs [T, B, H] and the final
    cell state (LSTM; an empty tensor otherwise).  ``w``: W_h [H, GW] (LSTM / RNN) or
    (Wg_h [H, 2H], Wc_h [H, H]) for the GRU."""

    @staticmethod
    def forward(ctx, ops, cell: int, zx, h0, c0, *w):
        T, B, GW = zx.shape
        H = h0.shape[1]
        lstm, gru = cell == CELL_IDS["lstm"], cell == CELL_IDS["gru"]
        hs = zx.new_empty(T + 1, B, H)
        hs[0].copy_(h0)
        cs = zx.new_empty(T + 1, B, H) if lstm else None
        if lstm:
            cs[0].copy_(c0)
        gates = zx.new_empty(T, B, GW) if (lstm or gru) else None
        rh = zx.new_empty(T, B, H) if gru else None
        WT = w[0].t().contiguous()
        WT2 = w[1].t().contiguous() if gru else None
        ops.f32_fwd_seq(cell, WT, WT2, zx.contiguous(), hs, cs, gates, rh, LSTM_FORGET_BIAS)
        ctx.ops, ctx.cell = ops, cell
        ctx.save_for_backward(hs, cs, gates, rh, *w)
        c_last = cs[T] if lstm else zx.new_empty(0)
        ctx.mark_non_differentiable(c_last)
        return hs[1:], c_last

    @staticmethod
    def backward(ctx, d_out, _d_c):
        hs, cs, gates, rh, *w = ctx.saved_tensors
        T1, B, H = hs.shape
        T = T1 - 1
        gru = ctx.cell == CELL_IDS["gru"]
        GW = 3 * H if gru else w[0].shape[1]
        dz = hs.new_empty(T, B, GW)
        work0 = hs.new_zeros(B, H)  # the LSTM dc carry starts at zero
        work1 = hs.new_empty(B, H)
        W, W2 = (w[1].contiguous(), w[0].contiguous()) if gru else (w[0].contiguous(), None)
        dtop = d_out.contiguous() if d_out is not None else None
        ctx.ops.f32_bwd_seq(ctx.cell, W, W2, dtop, hs, cs, gates, dz, work0, work1)
        dzf = dz.view(T * B, GW)
        hprev = hs[:T].reshape(T * B, H)
        if gru:
            dws = (hprev.t() @ dzf[:, : 2 * H], rh.view(T * B, H).t() @ dzf[:, 2 * H:])
        else:
            dws = (hprev.t() @ dzf,)
        return (None, None, dz, None, None) + dws


def forward_f32(ops, cfg: ModelConfig, params: dict, x: torch.Tensor, state: State,
                training: bool = True, gen: Optional[torch.Generator] = None,
                taps: Optional[dict] = None):
    """models.reference.forward with each layer's recurrence on the fp32 kernels (same
    outputs: logits [B·T, V] batch-major, the final state, outputs [B, T, H]).  Dropout masks
    are drawn for all T at once (same distribution as the per-step draws)."""
    B, T = x.shape
    H = cfg.rnn_size
    emb = params["embedding"][x.long()]  # [B, T, H]
    if taps is not None:
        taps["emb"] = emb
    inp = emb.transpose(0, 1)  # time-major [T, B, H]
    if training and cfg.output_keep_prob:
        inp = _dropout(inp, cfg.output_keep_prob, gen)
    wrap = training and (cfg.output_keep_prob < 1.0 or cfg.input_keep_prob < 1.0)
    cell = CELL_IDS[cfg.model]
    new_state = []
    for layer in range(cfg.num_layers):
        if wrap:
            inp = _dropout(inp, cfg.input_keep_prob, gen)
        X = inp.reshape(T * B, H)
        w = layer_weights(cfg, params, layer)
        st = state[layer]
        if cfg.model == "gru":
            gk, gb, ck, cb = w
            zx = torch.cat([X @ gk[:H] + gb, X @ ck[:H] + cb], 1).view(T, B, 3 * H)
            out, _ = _Recurrence.apply(ops, cell, zx, st[0], None, gk[H:], ck[H:])
            new_state.append((out[-1],))
        else:
            kernel, bias = w
            zx = (X @ kernel[:H] + bias).view(T, B, -1)
            if cfg.model == "lstm":
                out, c_last = _Recurrence.apply(ops, cell, zx, st[1], st[0], kernel[H:])
                new_state.append((c_last, out[-1]))
            else:
                out, _ = _Recurrence.apply(ops, cell, zx, st[0], None, kernel[H:])
                new_state.append((out[-1],))
        if wrap:
            out = _dropout(out, cfg.output_keep_prob, gen)
        inp = out
    out = inp.transpose(0, 1)  # [B, T, H]
    logits = out.reshape(B * T, H) @ params["rnnlm/softmax_w"] + params["rnnlm/softmax_b"]
    return logits, new_state, out


class NativeFp32Backend(ReferenceBackend):
    """The oracle's training step with the fp32 native recurrence (see the module docstring)."""

    def __init__(self, store: ParamStore, seed: int = 0):
        from ...ops import native

        if not supported(store.cfg):
            raise ValueError(f"native fp32: unsupported cell / rnn_size ({store.cfg.model}, "
                             f"{store.cfg.rnn_size})")
        super().__init__(store, seed=seed)
        self.ops = native.ops()

    def _forward(self, cfg, params, x, state, training=True, gen=None, taps=None, masks=None):
        if masks is not None:
            raise ValueError("explicit dropout masks: the oracle backend only")
        return forward_f32(self.ops, cfg, params, x, state, training, gen, taps)
