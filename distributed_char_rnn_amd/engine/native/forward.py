"""Forward pass of the native backend (model.py:54-76): embedding -> [dropout] -> L recurrent
layers -> [output dropout] -> softmax head, over the hand-written kernels of csrc/."""
from __future__ import annotations

from typing import Optional

import torch

from .gemm import bf16, f32, mm_into

FORGET_BIAS = 1.0


class ForwardMixin:
    # ------------------------------------------------------------------ dropout
    def _dropout(self, training: bool) -> bool:
        c = self.cfg
        return training and (c.input_keep_prob < 1.0 or c.output_keep_prob < 1.0)

    def _drop_masks(self, T: int, B: int, defer: bool = False) -> dict:
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
            # all masks of a step in one buffer, filled by one launch (segment per mask)
            n_in = self.L if p_in < 1.0 else 0
            n = n_in + (1 if p_out < 1.0 else 0)
            allb = torch.empty(n, T, B, self.H // 8, dtype=torch.uint8, device=self.dev)
            m = self._dm_bufs[key] = dict(
                all=allb, n_in=n_in,
                inb=[allb[i] for i in range(n_in)] if n_in else [None] * self.L,
                out=allb[n_in] if p_out < 1.0 else None)
        self._drop_step += 1
        stream = self._drop_step << 8
        streams = [stream + layer for layer in range(m["n_in"])]
        keeps = [p_in] * m["n_in"]
        if m["out"] is not None:
            streams.append(stream + 255)
            keeps.append(p_out)
        dm = dict(inb=m["inb"], out=m["out"], sin=1.0 / p_in, sout=1.0 / p_out)
        if streams:
            if defer:  # launched by _draw_masks (with layer 0's masked embedding rows)
                dm["pending"] = (m["all"], streams, keeps)
            else:
                self.ops.dropout_bits_multi(m["all"], self._drop_seed, streams, keeps)
        self.last_dropout_masks = dm
        return dm

    def _draw_masks(self, dm: Optional[dict], ids=None, E=None, X=None) -> None:
        """The deferred mask launch of ``_drop_masks(defer=True)``; with ``X`` the same launch
        writes layer 0's masked embedding rows E[ids] ⊙ mask / keep (segment 0 is layer 0's
        input mask), bit for bit the embed_dropout kernel's."""
        pend = dm.pop("pending", None) if dm else None
        if pend is None:
            return
        allb, streams, keeps = pend
        if X is not None:
            self.ops.dropout_bits_multi(allb, self._drop_seed, streams, keeps, ids, E, dm["sin"], X)
        else:
            self.ops.dropout_bits_multi(allb, self._drop_seed, streams, keeps)

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

    def _xin_ok(self) -> bool:
        v = getattr(self, "_xin_cache", None)
        if v is None:
            v = self._xin_cache = bool(self.ops.lstm2_xin_ok(self.H))
        return v

    # ------------------------------------------------------------------ forward
    def _forward(self, ids_tm: torch.Tensor, state, training: bool, want_logits: bool = True,
                 logits_bias: bool = True, extra_tasks: Optional[list] = None):
        """``extra_tasks``: more prep tasks for the step's one prep launch (the batch's ids)."""
        T, B = ids_tm.shape
        H, N = self.H, T * B
        tasks = self._prep() + list(extra_tasks or [])
        bufs = self._buffers(B, T, training)
        P = bufs["plan"]
        drop = self._dropout(training)
        # (launched after the prep launch has written the ids: with layer 0's embedding rows)
        dm = self._drop_masks(T, B, defer=True) if drop else None
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
        if P.persistent:
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
        o_done = False  # the top output-dropout rows written by the top pair's forward
        for layer in range(self.L):
            if layer == paired:
                continue
            lw, lb = self._w[layer], bufs["layers"][layer]
            gather = (layer == 0 and not drop and self.cfg.model != "nas")
            ids_arg = None
            # the forward never has a concurrent kernel (the previous step's all-reduce is joined
            # before the optimizer), so the one-workgroup-per-CU fused variant is safe here
            xfuse = P.persist and P.xfuse and layer > 0 and not drop and lw.WxT is not None
            if xfuse:
                if not x_prev.is_contiguous():  # h of a pair-interleaved layer (row stride 2H)
                    x_prev = x_prev.contiguous()
                lb.x_in = x_prev.reshape(N, H)
                self.ops.lstm_persist_fwd(lw.WhT, lw.bias, None, lb.hbuf, lb.cbuf, lb.gates,
                                          lb.hlast32, bufs["cnt"][layer], self.err, FORGET_BIAS,
                                          self.spin_limit, bufs["hrings"][0], None, lw.WxT,
                                          x_prev, lw.bias, cnt_zeroed=True, clast32=lb.clast32)
                x_prev = lb.hbuf[1:]
                continue
            xin = False
            if gather:
                zx = self._head["table"]
                ids_arg = ids_tm
            else:
                inb = dm["inb"][layer] if dm else None
                if layer == 0:  # the embedding rows (masked: embedding x input dropout)
                    X = lb.x_drop if inb is not None else torch.empty(N, H, dtype=bf16,
                                                                      device=self.dev)
                    fuse = (dm is not None and inb is not None and "pending" in dm
                            and H % 32 == 0 and self.knobs.debug.get("bits_embed", "1") != "0")
                    if fuse:
                        self._draw_masks(dm, ids_tm.reshape(-1), self._head["E"], X)
                    else:
                        self._draw_masks(dm)
                        self.ops.embed_dropout(ids_tm.reshape(-1), self._head["E"], inb,
                                               dm["sin"] if dm else 1.0, X)
                else:
                    X = x_prev.reshape(N, H)
                    if inb is not None:
                        X = self._masked(X, inb, dm["sin"], out=lb.x_drop)
                # the G = 1 two-layer forward projects these bf16 rows in-kernel (no library
                # GEMM, no [N, 4H] fp32 zx round trip; the rows are loaded one tick ahead behind
                # the payload): dropout headline 1.937 vs 1.958 ms for the library route, same
                # box, 3 alternating rounds (round 3, rows loaded at the tick start: 2.32 vs 2.20
                # -- slower).  DCR_DEBUG=xin=0 forces the library route.
                xin = (P.pair and layer + 1 < self.L and P.pair_g == 1 and lw.WxT is not None
                       and self.knobs.debug.get("xin", "1") != "0" and self._xin_ok())
                # (row-strided rows -- the h of a pair-interleaved layer -- feed the library
                # GEMMs as they are; the in-kernel projection wants dense rows)
                lb.x_in = X.contiguous() if (xin or X.stride(-1) != 1) else X
                if xin:
                    zx = lb.x_in
                else:
                    # the two-layer LSTM and the GRU kernels add the input bias in their
                    # epilogue: the library GEMM with a bias ran as GEMM + a separate [N, GW]
                    # fp32 add pass (41 us / 114 us per layer in the dropout headline / GRU-1024
                    # B = 256 profiles)
                    bias_in_kernel = ((P.pair and layer + 1 < self.L) or P.gru_persist
                                      or (P.persist and H > 1024)
                                      or (not P.persist and self._lib_step("fwd", B)))
                    mm_into(lb.x_in, lw.Wx, lb.zx.view(N, self.GW),
                            bias=None if bias_in_kernel else lw.bias)
                    zx = lb.zx
            if P.pair and layer + 1 < self.L:
                # layers (l, l+1) as one wavefront launch (lstm2_persist.hip): T+1 ticks; layer
                # l+1's input dropout is applied to its fragments in-kernel
                lw1, lb1 = self._w[layer + 1], bufs["layers"][layer + 1]
                xm = dm["inb"][layer + 1] if dm else None
                # G = 1: the kernel writes layer l+1's masked input rows (x_drop) itself, beside
                # layer l's row-major h (no separate mask pass; DCR_DEBUG=xdst=0: the pass)
                xdst = (lb1.x_drop if (xm is not None and P.pair_g == 1 and lb1.x_drop is not None
                                       and self.knobs.debug.get("xdst", "1") != "0") else None)
                # ... and, for the top pair, the output-dropout rows the head reads (o_drop)
                om = dm["out"] if (dm and xdst is not None and layer + 2 == self.L) else None
                odst = bufs["o_drop"] if om is not None else None
                self.ops.lstm2_persist_fwd(lw.WhT, lw1.WhT, lw1.WxT, zx, ids_arg, lw1.bias,
                                           lb.hbuf, lb.cbuf, lb.gates, lb.hlast32,
                                           lb1.hbuf, lb1.cbuf, lb1.gates, lb1.hlast32,
                                           bufs["cnt"][layer], bufs["cnt"][layer + 1], self.err,
                                           FORGET_BIAS, self.spin_limit, *bufs["hrings"],
                                           P.pair_g, lb.clast32, lb1.clast32, None, xm,
                                           dm["sin"] if dm else 1.0,
                                           lw.bias if ids_arg is None else None,
                                           lb.x_in if xin else None, lw.WxT if xin else None,
                                           xdst, om, dm["sout"] if om is not None else 1.0,
                                           odst)
                o_done = odst is not None
                # layer l+1's (masked) input rows for its weight gradient; unmasked rows of a
                # pair-interleaved buffer feed ONE GEMM for both of its weight gradients
                if xdst is not None:
                    lb1.x_in = xdst.view(N, H)
                else:
                    lb1.x_in = (self._masked(lb.hbuf[1:], xm, dm["sin"], out=lb1.x_drop)
                                if xm is not None else lb.hbuf[1:].reshape(N, H))
                ph = bufs.get("pair_h", {}).get(layer + 1)
                lb1.x_merged = ph is not None and (xm is None) == (ph[1] == "h")
                x_prev = lb1.hbuf[1:]
                paired = layer + 1
                continue
            if P.persist:
                self.ops.lstm_persist_fwd(lw.WhT, zx, ids_arg, lb.hbuf, lb.cbuf, lb.gates,
                                          lb.hlast32, bufs["cnt"][layer], self.err, FORGET_BIAS,
                                          self.spin_limit, bufs["hrings"][0], cnt_zeroed=True,
                                          clast32=lb.clast32,
                                          bias=lw.bias if (ids_arg is None and H > 1024) else None)
            elif P.gru_persist:
                gr = bufs["grings"]
                # the final h straight into a fresh tensor: the returned TBPTT state (no copy)
                lb.hlast32 = torch.empty(B, H, dtype=f32, device=self.dev)
                self.ops.gru_persist_fwd(lw.WhT, lw.WT2, zx, ids_arg, lb.hbuf, lb.h32, lb.rh,
                                         lb.gates, lb.hlast32, bufs["cnt"][layer], self.err,
                                         self.spin_limit, cnt_zeroed=True, ring0=gr[0],
                                         ring1=gr[1], bias_x=lw.bias if ids_arg is None else None)
            elif self._lib_step("fwd", B):
                self._lstm_fwd_lib(lw, lb, zx, ids_arg, bufs,
                                   bias=lw.bias if ids_arg is None else None)
            else:
                self.ops.rnn_fwd_seq(self.cell, lw.WhT, lw.WT2, zx, ids_arg, lb.hbuf, lb.h32,
                                     lb.cbuf, lb.gates, lb.pre, lb.aux, lb.rh, lb.hlast32,
                                     FORGET_BIAS)
            x_prev = lb.hbuf[1:]
        O = x_prev.reshape(N, H)
        if dm is not None and dm["out"] is not None:  # the top layer's output dropout
            O = (bufs["o_drop"] if o_done   # written by the top pair's forward
                 else self._masked(O, dm["out"], dm["sout"], out=bufs["o_drop"]))
        if O.stride(-1) != 1 or O.stride(0) % 8:  # the heads take row-strided O (ldo)
            O = O.contiguous()
        logits = bufs["logits"]
        if want_logits:
            # the wide-vocabulary CE adds the bias itself: a bias-initialised GEMM output would
            # cost an extra [N, V] fp32 broadcast copy (1 GB at V = 8192)
            mm_into(O, self._head["Ws"], logits, bias=self._head["bs"] if logits_bias else None)
        new_state = []
        for layer in range(self.L):
            lb = bufs["layers"][layer]
            if self.cfg.model in ("lstm", "nas"):
                new_state.append((lb.clast32, lb.hlast32) if layer in fresh
                                 else (lb.cbuf[T].clone(), lb.hlast32.clone()))
            elif self.cfg.model == "gru":
                new_state.append((lb.hlast32,) if P.gru_persist else (lb.h32[T].clone(),))
            else:
                new_state.append((lb.hlast32.clone(),))
        return bufs, O, logits, new_state
