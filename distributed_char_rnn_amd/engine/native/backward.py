"""Training step of the native backend: forward, fused softmax-CE, BPTT and the weight
gradients (the reference's tf.gradients + clip_by_global_norm inputs, model.py:88-98), with
gradient ranges reported ready (``on_ready``) for the bucketed all-reduce as they become final."""
from __future__ import annotations

import torch

from ...models.params import cell_specs
from .gemm import SumQueue, f32, mm_into, mm_tn, mm_tn_cols, mm_tn_pad, put
from .layouts import SEG_LDS_MAX_V
from .tail import TailQueue



def bucket_probe(on_ready):
    """Which gradient-ready reports complete a bucket: ``launches_at(offset)`` of an on_ready
    object that exposes it, or of the GradSync / ShardedStep a bound ``ready`` belongs to.  None
    for any other callable: the backward then flushes its deferred sums on every report (safe,
    one flush per report)."""
    probe = getattr(on_ready, "launches_at", None)
    if probe is None:
        probe = getattr(getattr(on_ready, "__self__", None), "launches_at", None)
    return probe

class BackwardMixin:
    def train_step(self, x, y, state, on_ready=None, want_extras: bool = False):
        B, T = x.shape
        H, V, N, GW = self.H, self.V, T * B, self.GW
        wide = self._wide_xent(T * B)
        # the batch's time-major ids (and the one-hot rows of the embedding-table gradient) are
        # produced by the step's prep launch, not by separate transpose / scatter kernels
        bufs0 = self._buffers(B, T, True)
        ids_tm, tgt = bufs0["ids_tm"], bufs0["tgt_tm"].view(-1)
        id_tasks = self._id_tasks(x, y, bufs0)
        bufs, O, logits, new_state = self._forward(ids_tm, state, True,
                                                   want_logits=not (self.fused_head
                                                                    or self.wide_head),
                                                   logits_bias=not wide, extra_tasks=id_tasks)
        # wide vocabulary: the embedding gradient's id sort (three counting-sort launches,
        # csrc/embed.hip id_sort) runs on the side stream beside the (non-persistent) wide head
        # instead of at the end of the backward; the main stream joins it before the
        # persistent BPTT launches
        self._sorted_ids = None
        self._de_zeroed = False
        sort_ev = None
        if (self.V > SEG_LDS_MAX_V and self.knobs.on("seg_sort") and not self._dropout(True)
                and self.cfg.model != "nas" and not self.capturing):
            side = self._side_stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                # (its first launch also clears the embedding gradient the atomic segment sum
                # accumulates into: no fill launch on the main stream)
                self._sorted_ids = self._sort_ids(ids_tm.view(-1),
                                                  zero=self.store.gview("embedding"))
                sort_ev = torch.cuda.Event()
                sort_ev.record(side)
            for t_ in self._sorted_ids:
                t_.record_stream(torch.cuda.current_stream())
        # deferred slab / bias sums of this step: one prep launch per flush (gemm.SumQueue), or
        # on the LSTM gather route one tail FINALIZE launch (csrc/tail.hip) that also computes
        # the layer-0 products and the global norm for the fused Adam
        dp = on_ready is not None
        use_wgrad = self.knobs.on("wgrad")  # hand-written token-reduction GEMMs (csrc/wgrad.hip)
        tail = self._tail_backward_ok(bufs0)
        q = (TailQueue(self, wgrad=use_wgrad, collectives=dp) if tail
             else SumQueue(self.ops, wgrad=use_wgrad))
        self._tail_total_ok = False
        if on_ready is not None:
            cb_user = on_ready

            probe = bucket_probe(cb_user)

            def on_ready(off, _cb=cb_user):  # noqa: F811 - sums complete before a bucket leaves
                if probe is not None and not probe(off):
                    return  # completes no bucket: no flush (its sums join the next one)
                q.flush()
                _cb(off)
        P = bufs["plan"]
        dlog = bufs["dlogits"]
        # the returned loss is read by the caller after the NEXT step was enqueued (trainer
        # logging): alternate two slots so that step does not overwrite it
        li = self._steps & 1
        loss_buf = bufs["loss"][li, :1]
        s, hd = self.store, self._head
        drop = self._dropout(True)
        dm = self.last_dropout_masks if drop else None
        head_omask = None  # the top output dropout applied by the head kernel to dtop
        if self.fused_head:
            # one launch: logits (only if asked for) -> CE -> bf16 dlogits, d softmax_b, dtop
            # (masked by the top layer's output dropout in-kernel: no fp32 pass over dtop)
            head_omask = dm["out"] if (dm is not None and self.knobs.on("head_omask")) else None
            self.ops.head(O, hd["WsT"], hd["Wsk"], hd["bs"], tgt, 1.0 / N,
                          logits if want_extras else None, bufs["row_loss"], dlog,
                          bufs["dtop"].view(N, H), s.gview("rnnlm/softmax_b"),
                          bufs["head_part"], loss_buf, head_omask,
                          dm["sout"] if dm is not None else 1.0)
            if bufs["dlogits_pad"] is not None:
                # (data parallel: the softmax gradients' bucket also holds layer L-1's weight
                # gradient, so this problem joins that layer's wgrad launch -- on_ready skips
                # the flush of a report that completes no bucket)
                mm_tn_pad(O, bufs["dlogits_pad"], s.gview("rnnlm/softmax_w"), q=q)
            else:
                mm_tn(O, dlog, s.gview("rnnlm/softmax_w"), q=q)
            if tail:  # d softmax_b (written by the head kernel): a norm term of the finalize
                q.add_sumsq(s.gview("rnnlm/softmax_b"))
            dtop = bufs["dtop"].view(T, B, H)
        elif self.wide_head:
            # wide vocabulary, one launch: logits (recomputed, never written unless asked for)
            # -> CE -> bf16 dlogits + d softmax_b partials (csrc/head_wide.hip)
            self.ops.head_wide(O, hd["WsTw"], hd["bs"], tgt, 1.0 / N, bufs["row_loss"], dlog,
                               logits if want_extras else None, bufs["hw_colpart"],
                               s.gview("rnnlm/softmax_b"), bufs["hw_part"], loss_buf)
            mm_tn(O, dlog, s.gview("rnnlm/softmax_w"), q=q)
            if tail:  # d softmax_b (written by the head's column-sum launch): a norm term
                q.add_sumsq(s.gview("rnnlm/softmax_b"))
            dtop = self._dtop_wide(dlog, bufs["dtop"].view(N, H)).view(T, B, H)
        elif wide:
            # wide vocabulary: one-read CE (bias added in-kernel), d softmax_b fused (xent_wide)
            self.ops.xent_wide(logits, hd["bs"], tgt, 1.0 / N, bufs["row_loss"], dlog,
                               bufs["colpart"], s.gview("rnnlm/softmax_b"), bufs["xpart"],
                               loss_buf)
            if want_extras:
                logits += hd["bs"]
            mm_tn(O, dlog, s.gview("rnnlm/softmax_w"), q=q)
            dtop = self._dtop_wide(dlog, bufs["dtop"].view(N, H)).view(T, B, H)
        else:
            self.ops.xent(logits, tgt, 1.0 / N, bufs["row_loss"], dlog, bufs["xpart"], loss_buf)
            # ---- head gradients
            mm_tn(O, dlog, s.gview("rnnlm/softmax_w"), q=q)
            self.ops.segsum(dlog, None, 1, bufs["colsum"][:, :V], bufs["ws"], False)
            s.gview("rnnlm/softmax_b").copy_(bufs["colsum"][0, :V])
            dtop = mm_into(dlog, hd["Ws"].t(), bufs["dtop"].view(N, H)).view(T, B, H)
        if sort_ev is not None:  # nothing may share CUs with the persistent BPTT grid
            torch.cuda.current_stream().wait_event(sort_ev)
        overlap = P.mode == "overlap" or not P.persistent
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
        paired_done = -1  # lower layer whose BPTT already ran inside a two-layer wavefront
        # TF clip-norm term from dx_tok = dZ0·W_x0ᵀ: needed as an extra GEMM only on the layer-0
        # gather route (every other route materialises dx_tok anyway)
        gather0 = not drop and self.cfg.model != "nas"
        fused_dew0 = P.persist and P.persist_bwd and gather0 and V <= 128 and self.dew_mode == "fused"
        tok_gemm = self.tf_norm and gather0 and not (V > SEG_LDS_MAX_V and not fused_dew0)
        for layer in reversed(range(self.L)):
            lw, lb = self._w[layer], bufs["layers"][layer]
            names = [sp.name for sp in cell_specs(self.cfg, layer)]
            pair_hi = P.pair_bwd and layer % 2 == 1 and dtop is not None
            # the top layer's output dropout
            omask = (dm["out"] if (dm is not None and layer == self.L - 1
                                   and head_omask is None) else None)
            if dtop is not None:
                dtop = dtop.contiguous()
                if omask is not None:
                    dtop = self._masked(dtop, omask, dm["sout"], out=dtop).view(T, B, H)
            zx_nas = lb.zx if self.cfg.model == "nas" else None
            written = False  # this layer's kernel/bias gradients already in the flat buffer
            gather = (layer == 0 and not drop and self.cfg.model != "nas")
            fused_dew = P.persist and P.persist_bwd and gather and V <= 128 and self.dew_mode == "fused"
            if pair_hi:
                # layers (layer-1, layer) as one reverse wavefront (lstm2_persist.hip): T+1
                # ticks, the lower layer's dtop = dZ·W_xᵀ of this layer computed in-kernel
                lo = layer - 1
                lw0, lb0 = self._w[lo], bufs["layers"][lo]
                nr = P.pair_rows
                self.ops.lstm2_persist_bwd(lw0.Wh, lw.Wh, lw.Wx, dtop, lb0.gates, lb0.cbuf,
                                           lb.gates, lb.cbuf, lb0.dz, lb.dz, bufs["zring"],
                                           bufs["zring2"], bufs["db_part"][lo][:nr],
                                           bufs["db_part"][layer][:nr], bufs["cnt"][self.L + lo],
                                           bufs["cnt"][self.L + layer], self.err,
                                           self.spin_limit, P.pair_g, None,
                                           dm["inb"][layer] if dm else None,
                                           dm["sin"] if dm else 1.0, bufs.get("prs"))
                paired_done = lo
                if lo == 0 and user_ready is not None:
                    on_ready = _release()
            elif layer == paired_done:
                pass
            elif P.persist and P.persist_bwd:
                self.ops.lstm_persist_bwd(lw.Wh, dtop, lb.dz, lb.gates, lb.cbuf,
                                          bufs["cnt"][self.L + layer], self.err, self.spin_limit,
                                          bufs["zring"], bufs["db_part"][layer][: -(-B // 16)],
                                          ids_tm if fused_dew else None,
                                          bufs["dew_part"] if fused_dew else None, V,
                                          exclusive=P.bwd_excl, cnt_zeroed=True)
                if layer == 0 and user_ready is not None:
                    # the last persistent grid is queued: buckets may now run beside the
                    # (non-persistent) layer-0 weight GEMMs
                    on_ready = _release()
            elif P.gru_persist:
                gr = bufs["grings"]
                self.ops.gru_persist_bwd(lw.W2, lw.Wh, dtop, lb.dz, lb.gates, lb.h32,
                                         bufs["cnt"][self.L + layer], self.err, self.spin_limit,
                                         cnt_zeroed=True, ring0=gr[0], ring1=gr[2],
                                         db_part=(self._db_part(bufs, layer)
                                                  if layer in bufs["bpart_layers"] else None))
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
            if (P.persist and layer > 0 and not drop and self.side_overlap and overlap
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
                    mm_tn(Hprev, dZ, s.gview(names[0])[H:], split=False)
                    mm_tn(lb.x_in, dZx, s.gview(names[0])[:H], split=False)
                    s.gview(names[1]).copy_(dbias)
                    dbias.record_stream(side)
                    if on_ready is not None:
                        on_ready(s.layer_range(layer)[1])
                dtop = mm_into(dZx, lw.Wx.t(), bufs["dx"].view(N, H)).view(T, B, H)
                self._side_used = True
                continue
            # recurrent-weight gradients
            if self.cfg.model == "gru":
                gk, gb, ck, cb = names
                mm_tn(Hprev, dZ[:, : 2 * H], s.gview(gk)[H:], q=q)
                mm_tn(lb.rh.view(N, H), dZ[:, 2 * H:], s.gview(ck)[H:], q=q)
            elif self.cfg.model == "nas":
                mm_tn(Hprev, dZ, s.gview(names[1]), q=q)
            elif lb.x_merged:
                # pair-interleaved h (buffers.py): rows [x_t, h_{t-1}] of this layer's kernel
                # lie side by side, so its W_x and W_h gradients are ONE [2H x 4H] GEMM
                C = bufs["pair_h"][layer][0]
                mm_tn(C[1:T + 1].reshape(N, 2 * H), dZ, s.gview(names[0]), q=q)
            else:
                mm_tn(Hprev, dZ, s.gview(names[0])[H:], q=q)
            if gather and V > SEG_LDS_MAX_V and not fused_dew:
                # wide vocabulary: the [V, GW] dEW segment sum would be an atomic scatter of
                # N x GW values plus two fp32 [V, GW] GEMMs; the dense route scatters N x H
                # instead: dW_x0 = E[ids]ᵀ·dZ0 (split-K), dE = segsum(dZ0·W_x0ᵀ)
                # X0 = E[ids] as bf16 rows: one gather kernel (embed_dropout without a mask)
                X0 = getattr(self, "_x0_rows", None)
                if X0 is None:  # (written by this step's prep launch otherwise, _id_tasks)
                    X0 = bufs["dx_bf"]
                    self.ops.embed_dropout(ids_tm.reshape(-1), hd["E"], None, 1.0, X0)
                # (written into the gradient buffer; the slab and bias-partial sums go to the
                # step's deferred flush instead of separate reduce launches)
                lstm_like = self.cfg.model in ("lstm", "rnn")
                dWx = (mm_tn(X0, dZx, s.gview(names[0])[:H], q=q) if lstm_like
                       else mm_tn(X0, dZx))
                if layer in bufs["bpart_layers"]:
                    dbias = self._bias_sum(self._db_part(bufs, layer), names,
                                           q if lstm_like else None)
                else:
                    self.ops.segsum(dZx, None, 1, bufs["colsum"][:, :GW], bufs["ws"], False)
                    dbias = bufs["colsum"][0, :GW]
                if (self.tf_norm and self.knobs.on("dx_fused")
                        and int(self.ops.tokennorm_supported(N, H, dZx.shape[1]))):
                    # one launch: the fp32 dX rows and their TF token-norm term
                    ws = self._tn_workspace()
                    dXf = bufs["dx"].view(N, H)
                    self.ops.tokennorm_store(dZx, lw.Wx, dXf, ws[0], ws[1],
                                             self.store.norm_slot_view())
                    self._embed_grad(dXf, ids_tm, bufs)
                else:
                    dXf = mm_into(dZx, lw.Wx.t(), bufs["dx"].view(N, H))
                    self._embed_grad(dXf, ids_tm, bufs)
                    self._token_norm(dXf)
            elif gather and tail and self._tail_gather_ok(layer, bufs, fused_dew):
                # tail route: dEW's split-K slabs, dW_x0 = Eᵀ·dEW and dE = dEW·W_x0ᵀ all in the
                # step's FINALIZE launch (the products wait in-launch for the dEW slab sum)
                self._bias_sum(self._db_part(bufs, layer), names, q)
                dew = bufs["dew"]
                q.signal_on(dew, 0)
                mm_tn(bufs["onehot"], dZx, dew, q=q)
                GW_ = dew.shape[1]
                if self.cfg.model == "gru":
                    # W_x0's gradient belongs to two kernels: gates [:, :2H], candidate [:, 2H:]
                    gk, _, ck, _ = names
                    q.add_mm(s.gview(gk)[:H], hd["E"], (1, H), dew, (GW_, 1), V, wait=0)
                    q.add_mm(s.gview(ck)[:H], hd["E"], (1, H), dew[:, 2 * H:], (GW_, 1), V,
                             wait=0)
                else:
                    q.add_mm(s.gview(names[0])[:H], hd["E"], (1, H), dew, (GW_, 1), V, wait=0)
                q.add_mm(s.gview("embedding"), dew, (GW_, 1), lw.Wx32, (1, GW_), GW_, wait=0)
                written = True
                if on_ready is not None:
                    self._join_side()
                    on_ready(s.layer_range(0)[1])
                if tok_gemm:
                    self._token_norm_gemm(dZx, lw.Wx)
            elif gather:
                # the bias gradient from the BPTT kernel's partials: summed in the same flush
                # as dEW's slabs (rather than a column sum of dEW after it)
                part_bias = layer in bufs["bpart_layers"] and self.cfg.model in ("lstm", "rnn",
                                                                                  "gru")
                if part_bias:
                    dbias = self._bias_sum(self._db_part(bufs, layer), names, q)
                dEW = self._dew(dZx, ids_tm, bufs, fused_dew, q)  # [V, GW] fp32 (flushes q)
                dWx = (torch.mm(hd["E"].t(), dEW, out=s.gview(names[0])[:H])
                       if self.cfg.model in ("lstm", "rnn") else hd["E"].t() @ dEW)  # [H, GW]
                if not part_bias:
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
                    # sum_tok ||dZ0_tok·W_x0ᵀ||² into the norm slot: library GEMM to bf16 rows
                    # + the sumsq kernel (66 us at the headline shape)
                    self._token_norm_gemm(dZx, lw.Wx)
            else:
                if lb.x_merged:  # written by the merged GEMM above
                    dWx = s.gview(names[0])[:H]
                elif self.cfg.model == "gru" and self.knobs.on("gru_dwx"):
                    # [H, 3H] split over the gates / candidate kernels by the flush's slab sums
                    gk, _, ck, _ = names
                    mm_tn_cols(lb.x_in, dZx, [(0, 2 * H, s.gview(gk)[:H]),
                                              (2 * H, 3 * H, s.gview(ck)[:H])], q)
                    dWx = None
                else:
                    dWx = (mm_tn(lb.x_in, dZx, s.gview(names[0])[:H], q=q)
                           if self.cfg.model in ("lstm", "rnn") else mm_tn(lb.x_in, dZx))
                if layer in bufs["bpart_layers"]:
                    dbias = self._bias_sum(self._db_part(bufs, layer), names, q)  # fused in BPTT
                else:
                    self.ops.segsum(dZx, None, 1, bufs["colsum"][:, :GW], bufs["ws"], False)
                    dbias = bufs["colsum"][0, :GW]
                if pair_hi:  # the lower layer's dtop was fused into the wavefront BPTT
                    self._write_input_grads(layer, names, dWx, dbias)
                    if on_ready is not None:
                        # a bucket cut (zero.shard_buckets rounds cuts down) may end inside a
                        # layer above whose gradients a side stream wrote: join it first
                        self._join_side()
                        on_ready(s.layer_range(layer)[1])
                    dtop = None
                    continue
                fused_dx = (layer == 0 and dm is not None and dm["inb"][0] is not None
                             and dm["inb"][0].data_ptr() % 8 == 0
                             and self.tf_norm and self.knobs.on("dx_fused")
                             and int(self.ops.tokennorm_supported(N, H, dZx.shape[1])))
                if fused_dx:
                    # one launch: dX = (dZ0·W_x0ᵀ) ⊙ mask / keep as bf16 rows and its TF
                    # token-norm term into the norm slot (csrc/tokennorm.hip masked form)
                    ws = self._tn_workspace()
                    self.ops.tokennorm_masked(dZx, lw.Wx, dm["inb"][0].view(-1), dm["sin"],
                                              bufs["dx_bf"].view(N, H), ws[0], ws[1],
                                              self.store.norm_slot_view())
                    dX = bufs["dx_bf"].view(T, B, H)
                elif layer > 0:
                    dX = mm_into(dZx, lw.Wx.t(), bufs["dx"].view(N, H)).view(T, B, H)
                else:  # only the embedding gradient reads it: bf16 rows for the segment sum
                    dX = torch.mm(dZx, lw.Wx.t(), out=bufs["dx_bf"]).view(T, B, H)
                if (not fused_dx and dm is not None
                        and dm["inb"][layer] is not None):  # this layer's input mask
                    dX = self._masked(dX, dm["inb"][layer], dm["sin"], out=dX).view(T, B, H)
                if layer > 0:
                    dtop = dX
                else:
                    # (bf16 as the GEMM wrote it: the segment sum and the norm accumulate in
                    # fp32 either way)
                    dXt = dX.reshape(N, H)
                    self._embed_grad(dXt, ids_tm, bufs)
                    if not fused_dx:  # (else written by the masked token-norm launch)
                        self._token_norm(dXt)
            if not written:
                self._write_input_grads(layer, names, dWx, dbias)
            if layer == 0:
                # side-stream work (overlapped weight GEMMs of the layers above) may share the
                # remaining buckets: join before reporting them ready
                self._join_side()
            if on_ready is not None:
                on_ready(None if layer == 0 else s.layer_range(layer)[1])
        if tail:
            # the last flush also leaves the global sum of squares for the fused Adam when
            # nothing (no data-parallel exchange) changes the gradients before the update
            if self._tail_total is None:
                self._tail_total = torch.zeros(1, dtype=f32, device=self.dev)
            self._tail_total_ok = q.flush(total_out=None if dp else self._tail_total)
        else:
            q.flush()
        self._join_side()
        if pending:
            _release()
        extras = {"logits": logits, "loss": bufs["row_loss"]} if want_extras else None
        self._steps += 1
        if P.persistent and not self.capturing and not self.defer_err_poll:
            self._poll_errors()
        return loss_buf[0], new_state, extras

    def _tail_backward_ok(self, bufs) -> bool:
        """The step's deferred gradient work (slab sums, bias sums, the gather route's
        products) runs as tail FINALIZE launches (csrc/tail.hip) instead of prep-launch flushes:
        LSTM / BasicRNN / GRU with the fused head or the wide head.  On the wide head's step the
        FINALIZE (24 us) also leaves the global norm -- every norm term but the embedding's
        (outside the norm prefix in TF clip mode, the token-norm slot stands in) is one of its
        outputs -- so the fused Adam needs no sum-of-squares launch: prep flush 18-21 us +
        sumsq_final 11 us before (DCR_DEBUG=fin_wide=0 restores that route)."""
        return (self.knobs.on("tail") and self.cfg.model in ("lstm", "rnn", "gru")
                and (self.fused_head or (self.wide_head and self.knobs.dbg("fin_wide", "1") == "1"))
                and int(self.ops.tail_grid()) > 0)

    def _tail_gather_ok(self, layer: int, bufs, fused_dew: bool) -> bool:
        """The layer-0 gather route's products in the finalize: the one-hot dEW GEMM with the
        bias gradient from the BPTT kernel's partials."""
        return (layer in bufs["bpart_layers"] and not fused_dew and self.dew_mode == "gemm"
                and bufs["onehot"] is not None and self.V <= SEG_LDS_MAX_V
                and self.cfg.model in ("lstm", "rnn", "gru"))

    def _id_tasks(self, x: torch.Tensor, y: torch.Tensor, bufs) -> list:
        """Prep tasks (csrc/prep.hip) of the batch: x, y [B, T] int32 -> time-major [T, B]
        copies, and on the layer-0 gather route the bf16 one-hot rows [T*B, VP] of dEW's GEMM."""
        if x.dim() != 2 or x.stride(1) != 1:
            x = x.contiguous()
        if y.dim() != 2 or y.stride(1) != 1:
            y = y.contiguous()
        tasks = [(x, bufs["ids_tm"], 1), (y, bufs["tgt_tm"], 1)]
        if (bufs["onehot"] is not None and not self._dropout(True)
                and self.cfg.model != "nas"):
            tasks.append((x, bufs["onehot"], 5))
        # wide vocabulary: the time-major bf16 embedding rows X0 = E[ids] (dW_x0 = X0ᵀ·dZ0 of
        # the dense backward route) as a GATHER task of the same launch, not a gather launch in
        # the middle of the backward
        self._x0_rows = None
        if (self.V > SEG_LDS_MAX_V and not self._dropout(True) and self.cfg.model != "nas"
                and self.knobs.on("x0_prep")):
            N = x.shape[0] * x.shape[1]
            X0 = bufs.get("x0_rows")
            if X0 is None or X0.shape != (N, self.H):
                X0 = bufs["x0_rows"] = torch.empty(N, self.H, dtype=torch.bfloat16,
                                                   device=self.dev)
            tasks.append((x, X0, 7, [self.store.view("embedding")]))
            self._x0_rows = X0
        return tasks

    def _dew(self, dZ0: torch.Tensor, ids_tm: torch.Tensor, bufs, fused: bool,
             q: SumQueue) -> torch.Tensor:
        """Layer-0 embedding-table gradient dEW = onehot(ids)ᵀ·dZ0 [V, GW] (gather route: the
        forward read Zx0 = (E·W_x0 + b0)[ids]).  ``gemm`` (default): split-K MFMA library GEMM
        against an exact 0/1 one-hot matrix -- the same fp32 sums of the bf16 dZ values as a
        scatter; ``segsum``: the one-hot MFMA segment-sum kernel (csrc/embed.hip); ``fused``:
        LDS partials accumulated inside the single-layer persistent BPTT."""
        V = self.V
        if fused:
            return bufs["dew_part"].sum(0)
        if self.dew_mode == "gemm" and bufs["onehot"] is not None:
            # the one-hot rows were written by this step's prep launch (_id_tasks)
            mm_tn(bufs["onehot"], dZ0, bufs["dew"], q=q)
            q.flush()
            return bufs["dew"][:V]                    # rows >= V are zero padding
        dEW = torch.empty(V, self.GW, dtype=f32, device=self.dev)
        self.ops.segsum(dZ0, ids_tm.view(-1), V, dEW, bufs["ws"], False)
        return dEW

    ERR_POLL_EVERY = 4

    def _poll_errors(self) -> None:
        """Non-blocking check of the persistent kernels' error word: every ERR_POLL_EVERY-th
        step copies it into pinned host memory behind its own work (a ~5 us blit launch, so
        not every step) and every step reads the latest copy, so a spin timeout raises within
        a few steps without a device sync.  (The optimizer skips its update on device while
        the word is set -- TFAdam(guard=err) -- so no step in between corrupts the weights.)"""
        if self._err_host is None:
            self._err_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        v = int(self._err_host[0])
        if v:
            self.check_errors()
        if self._steps % self.ERR_POLL_EVERY == 1:
            self._err_host.copy_(self.err, non_blocking=True)

    def _embed_grad(self, dX: torch.Tensor, ids_tm: torch.Tensor, bufs) -> None:
        """dE = segsum(dX_tok, ids) into the gradient buffer.  Wide vocabularies take the
        fp32-atomic route; there the ids are sorted first (a frequent id is then one register
        run per 32-row chunk instead of one atomic per occurrence)."""
        ids = ids_tm.view(-1)
        out = self.store.gview("embedding")
        if self.V > SEG_LDS_MAX_V and self.knobs.on("seg_sort"):
            zeroed = False
            if self._sorted_ids is not None:  # sorted beside the head (train_step)
                sid, perm = self._sorted_ids
                zeroed = self._de_zeroed
            else:
                sid, perm = self._sort_ids(ids)
            self.ops.segsum(dX, sid, self.V, out, bufs["ws"], zeroed, perm)
        else:
            self.ops.segsum(dX, ids, self.V, out, bufs["ws"], False)

    def _sort_ids(self, ids: torch.Tensor, zero: torch.Tensor = None):
        """(sorted ids, source positions) as int32 -- torch.sort(ids, stable=True) -- by the
        V-bucketed counting sort (csrc/embed.hip id_sort: histogram, scan, ballot-ranked
        scatter) where the vocabulary fits its LDS histogram, else the library sort.
        ``zero``: an fp32 buffer the sort's first launch clears (``self._de_zeroed`` tells
        whether it did)."""
        n = ids.numel()
        nws = int(self.ops.id_sort_workspace(n, self.V))
        if nws and self.knobs.on("id_sort"):
            i32 = dict(dtype=torch.int32, device=ids.device)
            ws, sid, perm = torch.empty(nws, **i32), torch.empty(n, **i32), torch.empty(n, **i32)
            done = self.ops.id_sort(ids.contiguous(), self.V, ws, sid, perm, zero)
            if zero is not None:
                self._de_zeroed = bool(done)
            return sid, perm
        sid, perm = torch.sort(ids, stable=True)
        return sid, perm.int()

    def _token_norm(self, dx_tok: torch.Tensor) -> None:
        """TF clip-norm term of the embedding (ModelConfig.clip_norm == "tf"): the sum of
        squares of the per-token input gradients (the IndexedSlices values), written into the
        gradient buffer's norm slot (all-reduced with the last bucket, read by adam_clip)."""
        if not self.tf_norm:
            return
        n = dx_tok.numel()
        if self._npart is None or self._npart.numel() < self.ops.opt_num_partials(n):
            self._npart = torch.empty(self.ops.opt_num_partials(n), dtype=f32, device=self.dev)
            # ticket of the one-launch form (zeroed once; the kernel's last block resets it)
            self._ntick = torch.zeros(1, dtype=torch.int32, device=self.dev)
        self.ops.sumsq(dx_tok.contiguous(), self._npart, self.store.norm_slot_view(),
                       self._ntick)

    def _token_norm_gemm(self, dZ: torch.Tensor, Wx: torch.Tensor) -> None:
        """TF clip-norm term sum_tok ||dZ_tok·W_xᵀ||² into the norm slot: one hand-written MFMA
        launch that squares its accumulators in registers (csrc/tokennorm.hip) -- no dx rows in
        HBM, no second pass; the library GEMM + sumsq form for shapes it does not tile."""
        if not self.tf_norm:
            return
        N, K = dZ.shape
        if self.knobs.on("tokennorm") and int(self.ops.tokennorm_supported(N, Wx.shape[0], K)):
            ws = self._tn_workspace()
            self.ops.tokennorm(dZ, Wx, ws[0], ws[1], self.store.norm_slot_view())
            return
        self._token_norm(torch.mm(dZ, Wx.t()))

    def _tn_workspace(self):
        """Partials + ticket of the token-norm launches (the ticket starts at zero and every
        launch leaves it at zero)."""
        if self._tn_ws is None:
            self._tn_ws = (torch.empty(1024, dtype=f32, device=self.dev),
                           torch.zeros(1, dtype=torch.int32, device=self.dev))
        return self._tn_ws

    def _dtop_wide(self, dlog: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        """dtop = dlogits · softmax_wᵀ (model.py:76's input gradient) for the wide vocabulary:
        the token-norm pipeline's store form (csrc/tokennorm.hip gemm_nt, both operands
        K = V-contiguous) where it tiles, else the library GEMM."""
        Ws = self._head["Ws"]  # [H, V] bf16
        N, V = dlog.shape
        if self.knobs.on("dtop_nt") and int(self.ops.gemm_nt_supported(N, Ws.shape[0], V)):
            self.ops.gemm_nt(dlog, Ws, out)
            return out
        return mm_into(dlog, Ws.t(), out)

    def _join_side(self) -> None:
        if self._side_used:
            torch.cuda.current_stream().wait_stream(self._side)
            self._side_used = False

    def _write_input_grads(self, layer: int, names, dWx: torch.Tensor, dbias: torch.Tensor):
        s, H = self.store, self.H
        if self.cfg.model == "gru":
            gk, gb, ck, cb = names
            if dWx is not None:  # (None: written by mm_tn_cols's deferred slab sums)
                s.gview(gk)[:H].copy_(dWx[:, : 2 * H])
                s.gview(ck)[:H].copy_(dWx[:, 2 * H:])
            if dbias is not None:  # (None: column sums of the BPTT partials, _bias_sum)
                s.gview(gb).copy_(dbias[: 2 * H])
                s.gview(cb).copy_(dbias[2 * H:])
        elif self.cfg.model == "nas":
            s.gview(names[0]).copy_(dWx)
        else:
            put(s.gview(names[0])[:H], dWx)
            put(s.gview(names[1]), dbias)
