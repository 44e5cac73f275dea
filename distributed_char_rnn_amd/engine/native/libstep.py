"""Large-H LSTM path (rnn_size > 1024, BASELINE config 4): one launch per time step, each
layer's T-step loop captured once as a hipGraph and replayed (the reference runs the same
per-step MatMul + pointwise cell inside its static unroll, model.py:72).

Two forms of a step: the fused MFMA step kernels of csrc/lstm_gemm_step.hip -- the recurrent
GEMM of the step with the LSTM cell (forward) or cell-backward (BPTT) epilogue in registers, no
fp32 [B, 4H] pre-activation round trip -- and the library form, a hipBLASLt GEMM per step
followed by an epilogue-only cell kernel (csrc/lstm_ew.hip).  Each direction and batch takes the
one measured faster (``_big_step_ok``); ``DCR_DEBUG=bigstep=0|2`` forces library | fused.
"""
from __future__ import annotations

import torch

from .forward import FORGET_BIAS
from .gemm import f32


class LibStepMixin:
    def _lib_step(self, direction: str, B: int) -> bool:
        """One launch per time step for LSTM with H > 1024 where the persistent kernels of
        lstm_persist_nt.hip do not apply (B > 64 at H = 2048, or T below the persistent
        minimum), both directions: the library-form forward also beats the fused per-step
        kernels of rnn_step.hip (4-layer LSTM-2048, T = 512, B = 64: 87.7 vs 92.4 ms per
        training step, same box).  DCR_RECURRENCE=library forces this path for any H,
        =step disables it."""
        if self.cfg.model != "lstm" or self.knobs.recurrence == "step":
            return False
        if self.knobs.recurrence == "library":
            return True
        if self.H <= 1024:
            return False
        return True

    # forward steps at B >= 96 beat the library form (scripts/micro/big_step_bench.py, H = 2048:
    # B = 128 13.7 vs 17.3 us, B = 512 26.9 vs 32.2, B = 1024 45.7 vs 49.9); at B = 64 the
    # library form is faster (13.7 vs 15.5) and so is the BPTT step at every batch (split-K
    # slabs of K = 4H: 22.6 vs 20.6 us at B = 64, 82 vs 56 at B = 1024)
    BIG_FWD_MIN_B = 96

    def _big_step_ok(self, direction: str, B: int) -> bool:
        """Fused MFMA step kernels (csrc/lstm_gemm_step.hip) for this direction and batch.
        DCR_DEBUG=bigstep=0: never, =1 (default): where measured faster, =2: always."""
        mode = self.knobs.dbg("bigstep", "1")
        if mode == "0" or not bool(self.ops.big_step_supported(B, self.H)):
            return False
        return mode == "2" or (direction == "fwd" and B >= self.BIG_FWD_MIN_B)

    def _big_ws(self, bufs, bwd: bool, B: int):
        """Split-K slabs + arrival tickets of the fused step kernels (the tickets start at zero
        and every launch leaves them at zero)."""
        key = "big_ws_bwd" if bwd else "big_ws_fwd"
        S = int(self.knobs.dbg("bigstep_s", "0"))
        ent = bufs.get(key)
        if ent is None or ent[2] != (B, S):
            wf, nt = self.ops.big_step_workspace(bwd, B, self.H, S)
            ent = bufs[key] = (torch.empty(max(int(wf), 4), dtype=f32, device=self.dev),
                               torch.zeros(max(int(nt), 1), dtype=torch.int32, device=self.dev),
                               (B, S))
        return ent[0], ent[1], S

    def _lstm_fwd_lib(self, lw, lb, zx, ids, bufs, bias=None) -> None:
        """``bias``: the input bias, added by the cell epilogue when the dense ``zx`` was
        written without it (a bias-initialised library GEMM output is a separate [T·B, 4H]
        fp32 broadcast pass: 16 GB per layer for config 4 at B = 1024)."""
        T, B = lb.gates.shape[0], lb.gates.shape[1]
        if self._big_step_ok("fwd", B):
            ws, cnt, S = self._big_ws(bufs, False, B)

            def body(zx, ids):
                for t in range(T):
                    self.ops.lstm_big_step_fwd(
                        lw.WhT, lb.hbuf[t], zx if ids is not None else zx[t],
                        ids[t] if ids is not None else None, lb.cbuf[t], lb.hbuf[t + 1],
                        lb.hlast32 if t == T - 1 else None, lb.cbuf[t + 1], lb.gates[t], ws, cnt,
                        FORGET_BIAS, S, bias)
        else:
            zrec = bufs.get("zrec")
            if zrec is None:
                zrec = bufs["zrec"] = torch.empty(1, B, self.GW, dtype=f32, device=self.dev)

            def body(zx, ids):
                for t in range(T):
                    # B operand as W_hᵀ-transposed (NT form): 20.7 vs 25.6 us at B = 256
                    torch.mm(lb.hbuf[t], lw.WhT.t(), out_dtype=f32, out=zrec[0])
                    self.ops.lstm_step_ew_fwd(zrec, zx if ids is not None else zx[t],
                                              ids[t] if ids is not None else None, lb.cbuf[t],
                                              lb.hbuf[t + 1], lb.hlast32 if t == T - 1 else None,
                                              lb.cbuf[t + 1], lb.gates[t], FORGET_BIAS, bias)

        self._run_lib_loop(bufs, ("fwd", id(lb)), body, zx, ids,
                           a_static=lb.zx is not None and zx.data_ptr() == lb.zx.data_ptr())

    def _lstm_bwd_lib(self, lw, lb, dtop, bufs) -> None:
        T, B = dtop.shape[0], dtop.shape[1]
        dc = bufs["dc"]
        if self._big_step_ok("bwd", B):
            ws, cnt, S = self._big_ws(bufs, True, B)

            def body(dtop, _unused):
                dc.zero_()
                # the last step has no recurrent term: the epilogue-only cell kernel
                self.ops.lstm_step_ew_bwd(dtop[T - 1], None, lb.gates[T - 1], lb.cbuf[T],
                                          lb.cbuf[T - 1], dc, lb.dz[T - 1])
                for t in reversed(range(T - 1)):
                    self.ops.lstm_big_step_bwd(lw.Wh, lb.dz[t + 1], dtop[t], lb.gates[t],
                                               lb.cbuf[t + 1], lb.cbuf[t], dc, lb.dz[t], ws, cnt,
                                               S)
        else:
            # dZ·W_hᵀ as S split-K slabs over K = 4H (the cell kernel sums them): the unsplit
            # [B, 8192] x [8192, 2048] product tiles a [B, 2048] output into too few workgroups
            # (scripts/micro/step_gemm_large_b.py: B = 256 28.7 -> 19.3 us at S = 2, B = 512
            # 34.7 -> 23.2 us and B = 1024 47.1 -> 36.7 us at S = 4)
            S = 4 if B >= 512 else 2 if B >= 256 else 1
            dh = bufs.get("dhrec")
            if dh is None or dh.shape[0] != S:
                dh = bufs["dhrec"] = torch.empty(S, B, self.H, dtype=f32, device=self.dev)
            G4 = 4 * self.H
            WhT = lw.Wh.t() if S == 1 else lw.Wh.view(self.H, S, G4 // S).permute(1, 2, 0)

            def body(dtop, _unused):
                dc.zero_()
                for t in reversed(range(T)):
                    # dh = dtop_t + dZ_{t+1}·W_hᵀ: the GEMM writes the recurrent part, the cell
                    # kernel adds dtop_t (an addmm with a 2-D input costs a separate copy launch)
                    if t < T - 1:
                        if S == 1:
                            torch.mm(lb.dz[t + 1], WhT, out_dtype=f32, out=dh[0])
                        else:
                            torch.bmm(lb.dz[t + 1].view(B, S, G4 // S).transpose(0, 1), WhT,
                                      out_dtype=f32, out=dh)
                    self.ops.lstm_step_ew_bwd(dtop[t], dh if t < T - 1 else None, lb.gates[t],
                                              lb.cbuf[t + 1], lb.cbuf[t], dc, lb.dz[t])

        static = any(buf is not None and dtop.data_ptr() == buf.data_ptr()
                     for buf in (bufs["dtop"], bufs["dx"]))
        self._run_lib_loop(bufs, ("bwd", id(lb)), body, dtop, None, a_static=static)

    def _run_lib_loop(self, bufs, key, body, a, b, a_static: bool = False) -> None:
        """Run a T-step loop (one or two launches per step) as a replayed hipGraph: eager,
        the per-step host launch cost (~15 us) is as long as the GPU's step at B = 64.  The
        graph is captured on the first call with static copies of the loop's varying inputs
        (a: zx / table / dtop, b: ids) and replayed afterwards; everything else it touches
        (h, c, gates, dZ buffers, the bf16 weights refreshed in place) is persistent.
        ``a_static``: ``a`` is itself a persistent buffer (dense zx, the dtop / dx buffers),
        captured directly instead of through a copy.  DCR_DEBUG=lib_graph=0 runs eagerly."""
        if not self.knobs.on("lib_graph"):
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
