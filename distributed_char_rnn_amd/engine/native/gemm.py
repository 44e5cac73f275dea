"""Library GEMM helpers of the native backend (hipBLASLt through torch): bf16 MFMA operands,
fp32 outputs written straight into gradient views, split-K for token reductions."""
from __future__ import annotations

from typing import Optional

import os

import torch

bf16 = torch.bfloat16
f32 = torch.float32


def mm(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """bf16 x bf16 -> fp32 GEMM on the MFMA library path."""
    return torch.mm(a, b, out_dtype=f32)


_OUT_OK = [None]


def mm_into(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor,
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
    out.copy_(mm(a, b) if bias is None else torch.addmm(bias, a, b, out_dtype=f32))
    return out


def split_k(K: int, M: int, Nn: int) -> int:
    """Split factor for a token-reduction GEMM with a small [M, Nn] output: the library tiles
    such an output into a few dozen workgroups (the 512x2048, K=32768 weight gradient ran on 73
    of 256 CUs at 335 TFLOP/s), so the reduction is split into S batched slices instead
    (scripts/bench_gemms.py: 205 -> 97 us at S=8; the 512x65 head gradient 133 -> 27 us)."""
    if K < 1024 or -(-M // 128) * -(-Nn // 256) >= 128:
        return 1
    if K < 8192:
        # short token reductions (the reference default, B = 50 x T = 50 = 2500 tokens): the
        # [128, 512] weight gradients ran on 8 workgroups at ~30 us each; slices of >= 256 tokens
        S = 8
        while S > 1 and (K % S or K // S < 256):
            S //= 2
        return S
    S = 8 if M * Nn >= (1 << 18) else 16
    if _SPLIT_CAP:
        S = _SPLIT_CAP if _SPLIT_CAP > 0 else min(S, -_SPLIT_CAP)
    while S > 1 and (K % S or K // S < 1024):
        S //= 2
    return S


# (measurement knob) the split factor of the long token reductions above: n > 0 forces n, n < 0
# caps at -n (same-box A/B: a cap of 4 cost 53 us per headline step, 2 cost 250 us)
_SPLIT_CAP = int(os.environ.get("DCR_SPLITK_CAP", "0") or 0)


WGRAD_MAX_TILES = 128  # output tiles per weight-gradient problem on the hand-written kernel


class SumQueue:
    """Deferred reductions of one training step, executed together as ONE prep launch
    (csrc/prep.hip SUM / COLSUM tasks) instead of one torch reduce kernel each (~5-10 us per
    launch on MI355X, seven of them per headline step).  Entries: split-K slabs of the weight
    GEMMs (``mm_tn(..., q=queue)``) and the persistent kernels' bias partials.  A destination
    is valid only after :meth:`flush`; the backend flushes before it reads one and before it
    reports a gradient range ready for the all-reduce."""

    SUM, COLSUM = 3, 4

    def __init__(self, ops, wgrad: bool = False):
        self.ops = ops
        self.tasks = []
        # token-reduction GEMMs deferred to the flush, run there as hand-written wgrad launches
        # (csrc/wgrad.hip: 256 x 256 tiles, split-K slabs; one launch for every pending GEMM of
        # one shape, so the headline's three weight gradients share one 240-workgroup grid)
        self.wgrad = wgrad
        self.gemms = []

    def wgrad_ok(self, a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor],
                 padded: bool = False) -> bool:
        """``padded``: ``out`` takes the first out.shape[1] columns of aᵀ·b (b zero-padded)."""
        if not self.wgrad or out is None or out.dim() != 2 or out.stride(1) != 1:
            return False
        for t in (a, b):
            if (t.dtype != bf16 or not t.is_cuda or t.dim() != 2 or t.stride(1) != 1
                    or t.stride(0) % 8 or t.data_ptr() % 16):
                return False
        K, M = a.shape
        N = b.shape[1]
        # large outputs stay on the library GEMM: hipBLASLt's big-tile kernels run those near
        # peak (config 4 at B = 1024, [4096 x 8192] per layer pair: 439.7 vs 449.3 ms per step
        # with the hand-written kernel); up to WGRAD_MAX_TILES 256 x 256 tiles (the headline's
        # 32 + 16, config 5's 64) the hand-written one is at parity or ahead
        shape_ok = (out.shape[0] == M and out.shape[1] <= N) if padded else tuple(out.shape) == (M, N)
        return (b.shape[0] == K and shape_ok
                and (M // 256) * (N // 256) <= WGRAD_MAX_TILES
                and int(self.ops.wgrad_plan(1, M, N, K)) > 0)

    # modelled cost (us) of computing an optional problem elsewhere (the softmax_w gradient's
    # library GEMM: ~20 us in the headline trace)
    OPTIONAL_ELSEWHERE_US = 20.0

    def add_gemm(self, a: torch.Tensor, b: torch.Tensor, out: torch.Tensor,
                 fallback=None) -> torch.Tensor:
        """aᵀ·b into ``out`` [M, N'] (N' <= b's N: the first N' columns -- b zero-padded).
        ``fallback``: the problem is optional -- if its tiles would push the launch into a
        worse split (e.g. a second round of workgroups), ``fallback()`` computes it instead."""
        self.gemms.append((a, b, out, fallback))
        return out

    def _run_gemms(self) -> None:
        """The pending token-reduction GEMMs as hand-written wgrad launches: up to 4 problems of
        one token count per launch, whatever their shapes (the step's layer-1 [2H x 4H] and
        layer-0 [H x 4H] gradients share one grid), one split count for the launch."""
        groups = {}
        for a, b, out, fb in self.gemms:
            groups.setdefault(a.shape[0], []).append((a, b, out, fb))
        self.gemms = []
        tiles_of = lambda t: (t[0].shape[1] // 256) * (t[1].shape[1] // 256)  # noqa: E731
        for K, items in groups.items():
            opt = [t for t in items if t[3] is not None]
            if opt and len(items) <= 4:
                # drop the optional problems when the launch without them (plus their own
                # routes) is modelled cheaper: the dropout headline's 64 + 2 tiles would need
                # a second round of workgroups (S = 7) where 64 tiles fill one (S = 4)
                t_all = sum(tiles_of(t) for t in items)
                t_req = t_all - sum(tiles_of(t) for t in opt)
                c_all = float(self.ops.wgrad_plan_cost(t_all, K))
                c_req = (float(self.ops.wgrad_plan_cost(t_req, K)) if t_req else 0.0) \
                    + self.OPTIONAL_ELSEWHERE_US * len(opt)
                if c_req < c_all:
                    for t in opt:
                        t[3]()
                    items = [t for t in items if t[3] is None]
            items = [t[:3] for t in items]
            for i in range(0, len(items), 4):  # csrc/kernels.h kWgradMaxProblems
                chunk = items[i: i + 4]
                tiles = sum((a.shape[1] // 256) * (b.shape[1] // 256) for a, b, _ in chunk)
                S = int(self.ops.wgrad_plan_tiles(tiles, K))
                parts = [torch.empty(S, a.shape[1], b.shape[1], dtype=f32, device=a.device)
                         for a, b, _ in chunk]
                self.ops.wgrad([c[0] for c in chunk], [c[1] for c in chunk], parts)
                for part, (_, _, out) in zip(parts, chunk):
                    self.add_sum(part[:, :, : out.shape[1]], out)

    def add_sum(self, part: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        self.tasks.append((part, out, self.SUM))
        return out

    def add_colsum(self, part: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        self.tasks.append((part, out, self.COLSUM))
        return out

    def flush(self) -> None:
        if self.gemms:
            self._run_gemms()
        if not self.tasks:
            return
        cap = int(self.ops.prep_max_tasks())
        for i in range(0, len(self.tasks), cap):
            chunk = self.tasks[i: i + cap]
            self.ops.prep([t[0] for t in chunk], [t[1] for t in chunk], [t[2] for t in chunk], [])
        self.tasks.clear()


def mm_tn(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None,
          split: bool = True, q: Optional[SumQueue] = None) -> torch.Tensor:
    """fp32 ``aᵀ·b`` for token-major bf16 operands ``a`` [K, M] and ``b`` [K, Nn] (weight
    gradients: K = T·B tokens), split-K over batched MFMA GEMMs + one fp32 sum when the output
    is too small to fill the chip.  ``split=False`` for GEMMs that run beside a persistent
    kernel on a side stream: there a chip-filling grid only steals the recurrence's CUs
    (measured: 256-workgroup split-K beside BPTT stretched both).  With a queue ``q`` (and an
    ``out``) the slab sum is deferred to ``q.flush()``; shapes the hand-written wgrad kernel
    covers (M, Nn multiples of 256, K of 32) are deferred whole and run there."""
    K, M = a.shape
    Nn = b.shape[1]
    if q is not None and q.wgrad_ok(a, b, out):
        return q.add_gemm(a, b, out)
    S = split_k(K, M, Nn) if split else 1
    if S == 1:
        if out is None:
            return mm(a.t(), b)
        mm_into(a.t(), b, out)
        if q is not None and hasattr(q, "add_sumsq"):
            q.add_sumsq(out)  # (tail finalize: written here, still a term of the global norm)
        return out
    part = torch.bmm(a.unflatten(0, (S, K // S)).transpose(1, 2), b.unflatten(0, (S, K // S)),
                     out_dtype=f32)
    if out is None:
        return part.sum(0)
    if q is not None and out.dim() == 2 and out.stride(1) == 1:
        return q.add_sum(part, out)
    torch.sum(part, 0, out=out)
    return out


def mm_tn_pad(a: torch.Tensor, b_pad: torch.Tensor, out: torch.Tensor, q: SumQueue) -> None:
    """``out`` [M, n] = aᵀ·b_pad[:, :n] where b_pad's columns >= n are zero (the fused head's
    dlogits rows padded to 256): a whole-tile problem of the queue's wgrad launch (the padding
    costs that launch nothing while its grid stays under one workgroup per CU), else the
    library GEMM on the n columns."""
    K, M = a.shape
    def library():
        mm_tn(a, b_pad[:, : out.shape[1]], out, q=q)

    if q.wgrad_ok(a, b_pad, out, padded=True):
        q.add_gemm(a, b_pad, out, fallback=library)
        return
    library()


def mm_tn_cols(a: torch.Tensor, b: torch.Tensor, outs, q: SumQueue) -> None:
    """``aᵀ·b`` whose output columns go to several destinations: ``outs`` = [(c0, c1, out),
    ...] takes columns [c0, c1) into ``out`` (the GRU's input-weight gradient [H, 3H] belongs
    to two kernels: gates [:, :2H] and candidate [:, 2H:]).  One split-K GEMM; each
    destination's slab sum is a task of the queue's flush -- no full-width temporary, sum and
    copies."""
    K, M = a.shape
    S = split_k(K, M, b.shape[1])
    if S == 1:
        full = mm(a.t(), b)
        for c0, c1, out in outs:
            out.copy_(full[:, c0:c1])
        return
    part = torch.bmm(a.unflatten(0, (S, K // S)).transpose(1, 2), b.unflatten(0, (S, K // S)),
                     out_dtype=f32)
    for c0, c1, out in outs:
        q.add_sum(part[:, :, c0:c1], out)


def put(dst: torch.Tensor, src: torch.Tensor):
    """dst.copy_(src) unless src already is dst's memory (results written in place)."""
    if not (src.data_ptr() == dst.data_ptr() and src.shape == dst.shape
            and src.stride() == dst.stride()):
        dst.copy_(src)
