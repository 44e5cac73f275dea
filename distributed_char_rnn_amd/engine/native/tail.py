"""Task tables of the step's tail kernel (csrc/tail.hip): FINALIZE (slab sums, bias column sums,
the layer-0 gather route's fp32 products, the global norm) and the fused ADAM update that writes
every bf16 kernel layout (model.py:88-98: clip_by_global_norm + AdamOptimizer.apply_gradients).

A table is a list of tasks, each ``TAIL_WORDS`` int64 words (csrc/ops.cpp ``tail``): pointers
travel as ``data_ptr()`` integers, so the table keeps references to every tensor it names.
Producers must precede the tasks that wait on them (csrc/tail.hip: dependency counters)."""
from __future__ import annotations

from typing import List, Optional

import torch

SUM, COLSUM, SUMSQ, MM, ADAM = 0, 1, 2, 3, 4
TAIL_WORDS = 27
MM_SHORT_K = 128  # csrc/tail.hip: MM with k <= 128 runs LDS-staged 64 x 64 tiles, longer k 16 x 16
MAX_DEPS = 4      # csrc/kernels.h kTailMaxDeps
MM_ROWS = 80      # csrc/tail.hip kMmRows: rows per long-MM tile


def _a16(t: torch.Tensor) -> bool:
    return t.data_ptr() % 16 == 0


def task_tiles(op: int, rows: int, cols: int, k: int, nslab: int = 0, vec4: int = 1) -> int:
    """Tiles of one task (csrc/tail.hip tail_tiles)."""
    if op == SUM:
        return -(-rows // 64) * -(-cols // 64)
    if op == ADAM:
        return -(-rows // (64 if vec4 else 16)) * -(-cols // 64)
    if op == COLSUM:
        return -(-cols // 64)
    if op == SUMSQ:
        return -(-(rows * cols) // 4096)
    if op == MM:
        if k <= MM_SHORT_K:
            return -(-rows // 64) * -(-cols // 64)
        return max(nslab, 1) * -(-rows // MM_ROWS) * -(-cols // 16)
    raise ValueError(op)


MAX_TILES = 16384  # csrc/kernels.h kTailMaxTiles: tiles of one launch


class TailTable:
    def __init__(self, max_tasks: int = 16, launch_tasks: Optional[int] = None):
        """``max_tasks``: tasks this table may hold; ``launch_tasks``: tasks per launch (the
        kernel's by-value table) when a larger logical table is partitioned into launches."""
        self.calls = []  # (method, args, kwargs) of every task, for partition()
        self.launch_tasks = launch_tasks or max_tasks
        self.words: List[int] = []
        self.keep: List[torch.Tensor] = []
        self.ops: List[int] = []
        self.tiles: List[int] = []
        self.max_tasks = max_tasks
        self.sig_tiles = {}  # dependency counter -> producer tiles
        self.waits = 0       # tasks that wait in-launch on a dependency counter

    def __len__(self) -> int:
        return len(self.ops)

    def partition(self, max_tiles: int = MAX_TILES) -> List["TailTable"]:
        """This table as consecutive launches of at most ``max_tiles`` tiles (and max_tasks
        tasks) each, in task order.  A task whose producers all ran in an earlier launch waits
        for nothing (stream order); a counter's ``need`` counts this launch's producers."""
        lt = self.launch_tasks
        if sum(self.tiles) <= max_tiles and len(self.ops) <= lt:
            return [self]
        out, cur = [], TailTable(lt)
        for (meth, args, kw), nt in zip(self._flat_calls(), self.tiles):
            if nt > max_tiles:
                raise ValueError(f"tail task of {nt} tiles > {max_tiles}")
            if len(cur) and (sum(cur.tiles) + nt > max_tiles or len(cur) >= cur.max_tasks):
                out.append(cur)
                cur = TailTable(lt)
            kw = dict(kw)
            if kw.get("wait", -1) >= 0 and cur.sig_tiles.get(kw["wait"], 0) <= 0:
                kw["wait"] = -1
            getattr(cur, meth)(*args, **kw)
        out.append(cur)
        return out

    def _flat_calls(self):
        """One (method, args, kwargs) per task: a k-slab MM call is two tasks (MM + SUM)."""
        for meth, args, kw in self.calls:
            if meth == "mm" and kw.get("slabs") is not None:
                out, a, sa, b, sb, k = args
                kw = dict(kw)
                slabs, slab_sig = kw.pop("slabs"), kw.pop("slab_sig")
                norm, sig = kw.pop("norm", False), kw.pop("sig", -1)
                yield ("_mm_slab_task", (out, a, sa, b, sb, k, slabs, slab_sig), kw)
                yield ("sum", (slabs, out, norm), dict(sig=sig, wait=slab_sig))
            else:
                yield meth, args, kw

    def _mm_slab_task(self, out, a, sa, b, sb, k, slabs, slab_sig, **kw):
        """The MM task of a k-slab product alone (its SUM is a separate call)."""
        S, rows, cols = slabs.shape
        ar, ak = sa
        bk, bc = sb
        self.calls.append(("_mm_slab_task", (out, a, sa, b, sb, k, slabs, slab_sig), kw))
        bias = kw.get("bias")
        self._add(MM, rows, cols, wait=kw.get("wait", -1), sig=slab_sig, nslab=S,
                  dst=slabs.data_ptr(), dst_ld=cols, off=rows * cols, k=k, a=a.data_ptr(),
                  ar=ar, ak=ak, b=b.data_ptr(), bk=bk, bc=bc,
                  bias=0 if bias is None else bias.data_ptr(),
                  keep=(out, a, b, slabs) + (() if bias is None else (bias,)))

    def _add(self, op, rows, cols, *, norm=0, wait=-1, sig=-1, vec4=0, nslab=0, k=0, o1_t=0,
             o2_t=0, a=0, ar=0, ak=0, b=0, bk=0, bc=0, bias=0, dst=0, dst_ld=0, off=0, ld=0, o1=0,
             o1_ld=0, o2=0, o2_ld=0, keep=()):
        if len(self.ops) >= self.max_tasks:
            raise ValueError(f"tail table: more than {self.max_tasks} tasks")
        need = 0
        if wait >= 0:
            need = self.sig_tiles.get(wait, 0)
            if need <= 0:
                raise ValueError(f"tail table: nothing signals counter {wait} before this task")
            self.waits += 1
        nt = task_tiles(op, rows, cols, k, nslab, int(vec4))
        if sig >= 0:
            self.sig_tiles[sig] = self.sig_tiles.get(sig, 0) + nt
        self.words += [op, rows, cols, int(norm), wait, need, sig, int(vec4), nslab, k, o1_t, o2_t,
                       a, ar, ak, b, bk, bc, bias, dst, dst_ld, off, ld, o1, o1_ld, o2, o2_ld]
        self.keep += list(keep)
        self.ops.append(op)
        self.tiles.append(nt)

    # ---- FINALIZE ----------------------------------------------------------------------------
    def sum(self, part: torch.Tensor, out: torch.Tensor, norm: bool, sig: int = -1,
            wait: int = -1):
        """out [rows, cols] = sum over the slabs of part [S, rows, cols] (fp32)."""
        self.calls.append(("sum", (part, out, norm), dict(sig=sig, wait=wait)))
        assert part.dim() == 3 and out.dim() == 2 and part.stride(2) == 1 and out.stride(1) == 1
        assert tuple(part.shape[1:]) == tuple(out.shape) and part.dtype == out.dtype == torch.float32
        S, rows, cols = part.shape
        n = rows * cols
        if (part.stride(1) == cols and out.stride(0) == cols and n % 256 == 0
                and part.stride(0) % 4 == 0 and _a16(part) and _a16(out)):
            # contiguous rows (e.g. softmax_w [H, 65]): summed as [n / 256, 256] float4 tiles
            # instead of the odd-width scalar path
            part = part.as_strided((S, n // 256, 256), (part.stride(0), 256, 1))
            out = out.view(-1).view(n // 256, 256)
            rows, cols = n // 256, 256
        vec4 = (cols % 4 == 0 and part.stride(1) % 4 == 0 and part.stride(0) % 4 == 0
                and out.stride(0) % 4 == 0 and _a16(part) and _a16(out))
        self._add(SUM, rows, cols, norm=norm, sig=sig, wait=wait, vec4=vec4, nslab=S, a=part.data_ptr(),
                  ar=part.stride(1), ak=part.stride(0), dst=out.data_ptr(), dst_ld=out.stride(0),
                  keep=(part, out))

    def colsum(self, part: torch.Tensor, out: torch.Tensor, norm: bool):
        """out [cols] = column sums of part [R, cols] (fp32, fixed order)."""
        self.calls.append(("colsum", (part, out, norm), {}))
        assert part.dim() == 2 and part.stride(1) == 1 and out.is_contiguous()
        assert out.numel() == part.shape[1]
        self._add(COLSUM, 1, part.shape[1], norm=norm, k=part.shape[0], a=part.data_ptr(),
                  ar=part.stride(0), dst=out.data_ptr(), dst_ld=part.shape[1], keep=(part, out))

    def sumsq(self, x: torch.Tensor):
        """A norm term finished elsewhere (contiguous fp32)."""
        self.calls.append(("sumsq", (x,), {}))
        assert x.is_contiguous() and x.dtype == torch.float32
        self._add(SUMSQ, 1, x.numel(), norm=1, a=x.data_ptr(), keep=(x,))

    def mm(self, out: torch.Tensor, a: torch.Tensor, a_strides, b: torch.Tensor, b_strides,
           k: int, bias: Optional[torch.Tensor] = None, norm: bool = False, wait: int = -1,
           sig: int = -1, slabs: Optional[torch.Tensor] = None, slab_sig: int = -1):
        """out[r, c] = bias[c] + sum_k a[r ar + k ak] * b[k bk + c bc] (fp32).  ``slabs``
        ([S, rows, cols] fp32, S > 1, k > MM_SHORT_K): the reduction split into S k-slabs over
        more workgroups, written there and signalled on ``slab_sig``; a SUM task waiting on it
        adds them into ``out`` in slab order."""
        n_calls = len(self.calls)
        assert out.dim() == 2 and out.stride(1) == 1 and out.dtype == torch.float32
        ar, ak = a_strides
        bk, bc = b_strides
        rows, cols = out.shape
        # every element the strides address lies inside the operands (a view's extent: from its
        # first element to its last, e.g. a column block of a wider matrix)
        def ext(t):
            return 1 + sum((n - 1) * st for n, st in zip(t.shape, t.stride())) if t.numel() else 0

        assert (rows - 1) * ar + (k - 1) * ak < ext(a) and (k - 1) * bk + (cols - 1) * bc < ext(b)
        ops = dict(k=k, a=a.data_ptr(), ar=ar, ak=ak, b=b.data_ptr(), bk=bk, bc=bc,
                   bias=0 if bias is None else bias.data_ptr())
        keep = (out, a, b) + (() if bias is None else (bias,))
        if slabs is None:
            self.calls.append(("mm", (out, a, a_strides, b, b_strides, k),
                               dict(bias=bias, norm=norm, wait=wait, sig=sig)))
            self._add(MM, rows, cols, norm=norm, wait=wait, sig=sig, dst=out.data_ptr(),
                      dst_ld=out.stride(0), keep=keep, **ops)
            return
        S = slabs.shape[0]
        assert (S > 1 and k > MM_SHORT_K and slab_sig >= 0 and slabs.is_contiguous()
                and tuple(slabs.shape) == (S, rows, cols) and slabs.dtype == torch.float32)
        self._add(MM, rows, cols, wait=wait, sig=slab_sig, nslab=S, dst=slabs.data_ptr(),
                  dst_ld=cols, off=rows * cols, keep=keep + (slabs,), **ops)
        self.sum(slabs, out, norm, sig=sig, wait=slab_sig)
        # one recorded call for both tasks (partition() splits it again)
        del self.calls[n_calls:]
        self.calls.append(("mm", (out, a, a_strides, b, b_strides, k),
                           dict(bias=bias, norm=norm, wait=wait, sig=sig, slabs=slabs,
                                slab_sig=slab_sig)))

    # ---- ADAM --------------------------------------------------------------------------------
    def adam(self, off: int, rows: int, cols: int, ld: int, outs=(), sig: int = -1,
             keep=()):
        """One parameter region flat[off + r ld + c]; ``outs``: up to two (bf16 tensor, row
        stride, transposed) layout outputs of it (besides the flat bf16 mirror)."""
        self.calls.append(("adam", (off, rows, cols, ld), dict(outs=outs, sig=sig, keep=keep)))
        assert len(outs) <= 2
        w = dict(o1=0, o1_ld=0, o1_t=0, o2=0, o2_ld=0, o2_t=0)
        vec4 = off % 4 == 0 and ld % 4 == 0 and cols % 4 == 0
        for i, (t, tld, tr) in enumerate(outs):
            assert t.dtype == torch.bfloat16
            n = "o1" if i == 0 else "o2"
            w[n], w[n + "_ld"], w[n + "_t"] = t.data_ptr(), tld, int(tr)
            if not tr:
                vec4 = vec4 and tld % 4 == 0 and t.data_ptr() % 8 == 0
        self._add(ADAM, rows, cols, sig=sig, vec4=vec4, off=off, ld=ld,
                  keep=tuple(t for t, _, _ in outs) + tuple(keep), **w)


def run(ops, table: TailTable, phase: int, ws: dict, err: torch.Tensor, spin_limit: int, *,
        total_out=None, total_in=None, extra=None, p=None, g=None, m=None, v=None, mirror=None,
        n_norm: int = 0, lr_t: float = 0.0, b1: float = 0.9, b2: float = 0.999,
        eps: float = 1e-8, clip: float = 0.0, gscale: float = 1.0, lr_dev=None, skip_if=None,
        norm_out=None, dynamic: bool = True):
    """``dynamic``: atomic tile queue, safe when the grid is not co-resident (another process
    on the GPU); False: static tiles, for a GPU this process has alone (the persistent
    recurrence's assumption, csrc/tail.hip)."""
    ops.tail(table.words, phase, ws["part"], ws["sync"], ws["dep"], err, spin_limit, total_out,
             total_in, extra, p, g, m, v, mirror, n_norm, lr_t, b1, b2, eps, clip, gscale, lr_dev,
             skip_if, norm_out, dynamic)


def workspace(ops, device) -> dict:
    """Per-workgroup partials and the (zeroed, self-resetting) ticket / dependency counters."""
    n_sync, n_dep = (int(w) for w in ops.tail_ws_words())
    return dict(part=torch.zeros(16384, dtype=torch.float32, device=device),
                sync=torch.zeros(n_sync, dtype=torch.int32, device=device),
                dep=torch.zeros(n_dep, dtype=torch.int32, device=device))


class TailQueue:
    """The backward's deferred gradient work as ONE tail FINALIZE launch per flush (the role of
    gemm.SumQueue's prep flush): split-K slab sums, bias column sums, the layer-0 gather route's
    fp32 products dW_x0 = Eᵀ·dEW and dE = dEW·W_x0ᵀ (waiting in-launch for the dEW slab sum),
    norm terms finished elsewhere, and -- on the step's last flush when nothing will change the
    gradients before the update -- the global sum of squares for the fused Adam."""

    SUM, COLSUM = 3, 4  # gemm.SumQueue task kinds (mm_tn / _bias_sum call add_sum / add_colsum)

    def __init__(self, backend, wgrad: bool = False, collectives: bool = False):
        from .gemm import SumQueue

        self.be = backend
        # gradient buckets may be in flight on RCCL's stream while a flush runs (data
        # parallel): its collectives hold CUs, so a flush whose tiles wait in-launch on other
        # tiles takes the atomic tile queue (static tiles need the whole grid co-resident)
        self.collectives = collectives
        self.ops = backend.ops
        self._gemmq = SumQueue(backend.ops, wgrad=wgrad)  # its wgrad grouping, not its flush
        self.wgrad = wgrad
        self.sums = []      # (part, out, sig)
        self.colsums = []   # (part, out)
        self.sumsqs = []    # contiguous fp32 gradient views
        self.mms = []       # (out, a, a_strides, b, b_strides, k, wait)
        self._signals = {}  # out data_ptr -> dependency counter its slab sum signals

    # -- the SumQueue interface used by gemm.mm_tn / backward._bias_sum ----------------------
    def wgrad_ok(self, a, b, out, padded: bool = False) -> bool:
        return self._gemmq.wgrad_ok(a, b, out, padded)

    def add_gemm(self, a, b, out, fallback=None):
        return self._gemmq.add_gemm(a, b, out, fallback)

    def add_sum(self, part, out, sig: int = -1):
        if sig < 0:
            sig = self._signals.get(out.data_ptr(), -1)
        self.sums.append((part, out, sig))
        return out

    def signal_on(self, out: torch.Tensor, counter: int) -> None:
        """The slab sum into ``out`` (queued later by mm_tn) signals dependency ``counter``."""
        self._signals[out.data_ptr()] = counter

    def add_colsum(self, part, out):
        self.colsums.append((part, out))
        return out

    # -- tail-only tasks -----------------------------------------------------------------------
    def add_sumsq(self, g):
        self.sumsqs.append(g)

    def add_mm(self, out, a, a_strides, b, b_strides, k, wait: int = -1):
        self.mms.append((out, a, a_strides, b, b_strides, k, wait))
        return out

    @staticmethod
    def _mm_slabs(rows: int, cols: int, k: int, grid: int) -> int:
        """k-slabs for a long-reduction MM whose 16 x 16 tiles alone would leave most of the
        grid idle (dE = dEW·W_x0ᵀ: 160 tiles of k = 2048): about one tile per workgroup, at
        least 256 k per slab."""
        if k <= MM_SHORT_K:
            return 1
        tiles = -(-rows // MM_ROWS) * -(-cols // 16)
        return max(1, min(grid // max(tiles, 1), k // 64, 8))

    def _slab_buf(self, S: int, rows: int, cols: int) -> torch.Tensor:
        bufs = self.be.__dict__.setdefault("_tail_slabs", {})
        key = (S, rows, cols)
        if key not in bufs:
            bufs[key] = torch.empty(S, rows, cols, dtype=torch.float32, device=self.be.dev)
        return bufs[key]

    def _norm_range(self, out: torch.Tensor):
        """(flat offset, elements) of a gradient view inside the norm prefix, else None."""
        s = self.be.store
        base = s.grad.data_ptr()
        off = (out.data_ptr() - base) // 4
        if out.dtype != torch.float32 or not (0 <= off < s.grad.numel()):
            return None
        if not out.is_contiguous():
            raise AssertionError("tail: gradient outputs must be contiguous views")
        n_norm, _ = s.norm_terms()
        if off >= n_norm:
            return None
        if off + out.numel() > n_norm:
            raise AssertionError("tail: an output straddles the norm prefix")
        return off, out.numel()

    def flush(self, total_out: Optional[torch.Tensor] = None) -> bool:
        """One FINALIZE launch over everything queued.  ``total_out``: also the global sum of
        squares (+ the norm slot) -- returned True only if the queued norm terms tile the whole
        norm prefix (otherwise the fused Adam computes the norm itself)."""
        g = self._gemmq
        if g.gemms:
            g._run_gemms()  # hand-written wgrad launches; their slab sums land in g.tasks
        for part, out, kind in g.tasks:
            (self.add_sum if kind == self.SUM else self.add_colsum)(part, out)
        g.tasks.clear()
        if not (self.sums or self.colsums or self.sumsqs or self.mms) and total_out is None:
            return False
        be = self.be
        # (a logical table: more tasks than one launch's table become consecutive launches,
        # partition(); the GRU's per-layer slab and bias sums exceed one)
        tab = TailTable(1 << 12, launch_tasks=int(self.ops.tail_max_tasks()))
        spans = []

        def norm_of(out):
            r = self._norm_range(out)
            if r is not None:
                spans.append(r)
            return r is not None
        # producers first (the slab sums that signal a dependency counter), the products waiting
        # on them last: their tiles come in the launch's last round, when their producers are
        # long done (dealt in the first round right after the producers, their workgroups spun
        # instead of summing: FINALIZE 55 vs 45 us)
        for part, out, sig in sorted(self.sums, key=lambda t: t[2] < 0):
            if part.dim() == 2:
                part = part.unsqueeze(0)
            tab.sum(part, out, norm_of(out), sig)
        for part, out in self.colsums:
            tab.colsum(part, out.view(-1), norm_of(out))
        for x in self.sumsqs:
            if norm_of(x):  # (outside the norm prefix: nothing to do)
                tab.sumsq(x)
        self._put_mms(tab, norm_of, int(self.ops.tail_grid()))
        self.sums, self.colsums, self.sumsqs, self.mms = [], [], [], []
        return self._launch(tab, spans, total_out)

    def _put_mms(self, tab, norm_of, grid):
        for out, a, sa, b, sb, k, wait in self.mms:
            # (a producer that did not become a slab sum of this launch -- a GEMM short enough
            # to run unsplit -- wrote its output in stream order before it: nothing to wait for)
            wait = wait if tab.sig_tiles.get(wait, 0) > 0 else -1
            S = self._mm_slabs(out.shape[0], out.shape[1], k, grid)
            if S > 1 and len(tab) + 2 <= tab.max_tasks and len(tab.sig_tiles) < MAX_DEPS:
                c = min(set(range(MAX_DEPS)) - set(tab.sig_tiles))
                tab.mm(out, a, sa, b, sb, k, norm=norm_of(out), wait=wait,
                       slabs=self._slab_buf(S, *out.shape), slab_sig=c)
            else:
                tab.mm(out, a, sa, b, sb, k, norm=norm_of(out), wait=wait)

    def _launch(self, tab, spans, total_out) -> bool:
        be = self.be
        if not len(tab):
            return False
        ok = False
        if total_out is not None:
            # every parameter inside the norm prefix must be an output of this launch (the
            # alignment padding between tensors holds zero gradients: gaps there are fine)
            n_norm, _ = be.store.norm_terms()
            spans.sort()
            ok = all(b[0] >= a[0] + a[1] for a, b in zip(spans, spans[1:]))  # no overlaps
            merged = []
            for o, n in spans:
                if merged and merged[-1][0] + merged[-1][1] == o:
                    merged[-1] = (merged[-1][0], merged[-1][1] + n)
                else:
                    merged.append((o, n))
            covered = lambda lo, hi: any(o <= lo and hi <= o + n for o, n in merged)  # noqa: E731
            ok = ok and all(covered(sp.offset, sp.offset + sp.numel) for sp in be.store.specs
                            if sp.offset < n_norm)
        if getattr(be, "_fin_ws", None) is None:
            be._fin_ws = workspace(self.ops, be.dev)
        s = be.store
        _, use_slot = s.norm_terms()
        # several launches: each adds its terms to the previous one's total (the kernel's
        # ``extra`` addend; the first one's is the norm slot)
        extra = s.norm_slot_view() if (ok and use_slot) else None
        for t in tab.partition():
            run(self.ops, t, 0, be._fin_ws, be.err, be.spin_limit,
                total_out=total_out if ok else None, extra=extra,
                dynamic=be.tail_dynamic() or (self.collectives and t.waits > 0))
            extra = total_out if ok else None
        return ok
