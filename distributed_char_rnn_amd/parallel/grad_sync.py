"""Bucketed, backward-overlapped gradient all-reduce over the flat gradient buffer.

Replaces the reference's per-step worker->PS gradient push + PS-side ApplyAdam (CS3/CS4 of
SURVEY.md §2.4, model.py:98 under replica_device_setter, train.py:132-133) with synchronous
data parallelism: every rank keeps a full replica, gradients are summed with RCCL all-reduce
and every rank applies the identical clipped Adam update.

The flat gradient buffer is laid out in reverse backward-availability order (softmax head,
top layer, ..., layer 0, embedding; models/params.py), so buckets are *contiguous slices*.
The backend calls :meth:`ready(upto)` when every gradient below flat offset ``upto`` is final;
all buckets completely below it are launched immediately as async all-reduces on RCCL's own
stream (which orders itself after the work already queued on the compute stream), so the
head's and upper layers' communication overlaps the BPTT of lower layers.  :meth:`finish`
joins the outstanding work and averages.

Bucket sizing (``--bucket_mb``): xGMI is point-to-point, 7 links x ~153 GB/s per MI355X; a
ring all-reduce of S bytes on N GPUs moves 2(N-1)/N·S per link, so an 8 MB bucket is ~90 us of
wire time on 8 GPUs -- large enough to amortise RCCL's per-call latency (~10-30 us), small
enough that the first bucket starts while BPTT of the lower layers still has >=1 ms to run.

``wire_dtype="bf16"`` halves the bytes without summing in bf16: each bucket's world chunks
travel once through an all_to_all, every rank sums its chunk in fp32, and the sums return
through an all_gather (one rounding of the final sum instead of one per ring hop).  The sharded
alternative (reduce-scatter + optimizer on a 1/world shard) is parallel/zero.py.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

from ..models.params import ParamStore


class GradSync:
    def __init__(self, store: ParamStore, world_size: int, bucket_mb: float = 8.0,
                 wire_dtype: str = "fp32", group=None, enabled: Optional[bool] = None,
                 guard: Optional[torch.Tensor] = None, timing: bool = False):
        """``guard``: the rank's persistent-kernel error word.  A rank whose recurrence timed out
        contributed garbage gradients to the sum, so EVERY rank must skip that update (a local
        guard alone would let the healthy ranks apply it while the faulty one skips, and the
        replicas would diverge).  The word rides along with the last bucket: it is copied (as
        a float) into a padding slot of the gradient buffer behind the clip-norm slot, summed
        with everything else, and ``guard_view`` -- that slot's bits as int32, non-zero iff any
        rank's word was -- is what the optimizer must use as its guard (``TFAdam.guard``).  No
        extra collective per step."""
        self.store = store
        self.world = world_size
        self.group = group
        self.enabled = (world_size > 1) if enabled is None else enabled
        self.wire_bf16 = wire_dtype == "bf16"
        self.guard = guard
        self.guard_slot = store.norm_slot + 1
        if self.guard_slot >= store.numel:
            raise ValueError("no padding slot for the error word behind the clip-norm slot")
        self.guard_view = (store.grad[self.guard_slot:self.guard_slot + 1].view(torch.int32)
                           if guard is not None else None)
        self.buckets = self._make_buckets(bucket_mb)
        self._next = 0
        self._work: List[Tuple[object, int, int, Optional[torch.Tensor]]] = []
        # bf16 wire: per-bucket send / receive / gather buffers, allocated once
        self._wire_bufs: dict = {}
        # --profile: CUDA events at the step start, at each bucket's release (its gradients are
        # final on the compute stream) and at the end of the backward (finish), see windows()
        self.timing = timing and store.flat.device.type == "cuda"
        self._ev_start = None
        self._ev_ready: List[Tuple[int, object]] = []
        self._ev_end = None

    def _make_buckets(self, bucket_mb: float) -> List[Tuple[int, int]]:
        """Cut the flat buffer at tensor boundaries into ~bucket_mb slices.  The last tensor
        (the embedding, plus the clip-norm slot behind it) always forms its own final bucket:
        it is the last gradient the backward finalises (after the layer-0 weight gradients, the
        embedding GEMM and the token-norm GEMM), so only its few hundred KB -- not a whole
        layer's ~8 MB -- are all-reduced after the backward with nothing left to overlap."""
        cap = max(1, int(bucket_mb * (1 << 20) / 4))
        cuts, lo, cur = [], 0, 0
        specs = self.store.specs
        for i, s in enumerate(specs):
            if i == len(specs) - 1 and len(specs) > 1 and cur > lo:
                cuts.append((lo, cur))  # close the bucket before the final tensor
                lo = cur
            end = s.offset + s.numel
            cur = end
            if cur - lo >= cap:
                cuts.append((lo, cur))
                lo = cur
        if cur > lo:
            cuts.append((lo, cur))
        # a sliver left before the final bucket (a bias) joins its predecessor: one RCCL call
        # fewer, and it is final no later than the predecessor's last tensor
        merged = []
        for i, (a, b) in enumerate(cuts):
            if merged and i < len(cuts) - 1 and b - a < cap // 16:
                merged[-1] = (merged[-1][0], b)
            else:
                merged.append((a, b))
        cuts = merged
        # the flat buffer may have alignment padding at the end: cover it in the last bucket
        if cuts:
            cuts[-1] = (cuts[-1][0], self.store.numel)
        return cuts

    def reset(self):
        self._next = 0
        self._work.clear()
        if self.timing:
            self._ev_start = torch.cuda.Event(enable_timing=True)
            self._ev_start.record()
            self._ev_ready = []
            self._ev_end = None

    def launches_at(self, upto: Optional[int] = None) -> bool:
        """Whether ``ready(upto)`` would launch a bucket (the backward skips its deferred-sum
        flush for a readiness report that completes none: one tail launch fewer)."""
        if not self.enabled:
            return False
        lim = self.store.numel if upto is None else upto
        return self._next < len(self.buckets) and self.buckets[self._next][1] <= lim

    def ready(self, upto: Optional[int] = None, sync: bool = False):
        """Launch every not-yet-launched bucket that ends at or below flat offset ``upto``
        (``None`` = everything).  ``sync``: as blocking collectives (c10d still runs them on
        ProcessGroupNCCL's internal stream; ``async_op=False`` makes the current stream wait on
        the collective's completion, with no Work object kept here), for buckets whose exchange
        nothing is left to overlap, after every earlier asynchronous one has been waited for."""
        if not self.enabled:
            return
        lim = self.store.numel if upto is None else upto
        while self._next < len(self.buckets) and self.buckets[self._next][1] <= lim:
            lo, hi = self.buckets[self._next]
            g = self.store.grad[lo:hi]
            if self.guard is not None and lo <= self.guard_slot < hi:
                self.store.grad[self.guard_slot:self.guard_slot + 1].copy_(self.guard)
            if self.timing:
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()
                self._ev_ready.append((self._next, ev))
            if self.wire_bf16:
                # bf16 on the wire, fp32 accumulation: the bucket's world chunks travel once
                # through an all_to_all, each rank sums its chunk in fp32, the sums come back
                # through an all_gather (finish).  A bf16 all-reduce would round after every
                # ring hop: N-1 roundings of partial sums at N ranks.
                send, recv = self._bufs_for(lo, hi, g.device)[:2]
                send[: hi - lo].copy_(g)  # the tail padding stays zero (allocated zeroed)
                w = dist.all_to_all_single(recv, send, group=self.group, async_op=not sync)
                self._work.append((w, lo, hi, recv))
            else:
                w = dist.all_reduce(g, group=self.group, async_op=not sync)
                self._work.append((w, lo, hi, None))
            self._next += 1

    def finish(self, defer_scale: bool = False) -> float:
        """Wait for all buckets and average (sum / world).  With ``defer_scale`` the buffer is
        left holding the sum and the returned factor (1/world) is meant for
        ``TFAdam.step(lr, grad_scale=...)``, which folds it into its clip/update pass (one fewer
        pass over the gradient buffer)."""
        if not self.enabled:
            return 1.0
        if self.timing:
            self._ev_end = torch.cuda.Event(enable_timing=True)
            self._ev_end.record()
        # the buckets the backward launched first, then the rest as blocking collectives (the
        # current stream waits on them; nothing is left to overlap them with -- the measured
        # gain of this form comes from launch and wait ordering, not from where RCCL runs)
        for w, lo, hi, recv in self._work:
            w.wait()
        self.ready(None, sync=True)
        for w, lo, hi, recv in self._work:
            if recv is not None:  # bf16 wire: fp32 sum of my chunk, then gather every chunk
                _, _, mine, mine16, full = self._bufs_for(lo, hi, recv.device)
                torch.sum(recv.view(self.world, -1), 0, dtype=torch.float32, out=mine)
                mine16.copy_(mine)
                dist.all_gather_into_tensor(full, mine16, group=self.group)
                self.store.grad[lo:hi].copy_(full[: hi - lo])
        self._work.clear()
        self._next = 0
        if self.guard is not None and self.guard_view is not None and self.world > 1:
            # fold the reduced guard (non-zero iff any rank's word was) back into this rank's
            # own error word: every rank then raises on the same step (trainer poll).  One
            # bitwise OR (the slot's bits are non-zero iff any rank's word was)
            self.guard.bitwise_or_(self.guard_view)
        if defer_scale:
            return 1.0 / self.world
        self.store.grad.mul_(1.0 / self.world)  # (the guard slot stays non-zero iff it was)
        # the clip-norm slot holds a SUM OF SQUARES (TF's per-token embedding term, summed over
        # ranks): averaging the gradients scales it by 1/world^2, not 1/world
        self.store.norm_slot_view().mul_(1.0 / self.world)
        return 1.0

    def windows(self) -> List[Tuple[int, int, float, float]]:
        """(bucket, bytes on the wire, release time from the step start [ms], overlap window =
        end of the backward - release [ms]) of the last step; synchronises.  Buckets released
        by ``finish`` itself have a zero window."""
        if not (self.timing and self._ev_start is not None and self._ev_end is not None):
            return []
        torch.cuda.synchronize()
        out = []
        esz = 2 if self.wire_bf16 else 4
        for i, ev in self._ev_ready:
            lo, hi = self.buckets[i]
            t = self._ev_start.elapsed_time(ev)
            out.append((i, (hi - lo) * esz, t, max(0.0, self._ev_start.elapsed_time(self._ev_end) - t)))
        return out

    @staticmethod
    def exposed_ms(windows, world: int, busbw_gbps: float, latency_us: float = 25.0) -> float:
        """Communication time left after the backward ends, for a ring all-reduce of each bucket
        at ``busbw_gbps`` bus bandwidth (2(N-1)/N·S / busbw + latency per call), buckets issued in
        order on one stream, each no earlier than its release."""
        if world <= 1 or not windows:
            return 0.0
        end_bwd = max(t + w for _, _, t, w in windows)
        tnow = 0.0
        for _, nbytes, t, _ in windows:
            cost = 2.0 * (world - 1) / world * nbytes / (busbw_gbps * 1e9) * 1e3 + latency_us * 1e-3
            tnow = max(tnow, t) + cost
        return max(0.0, tnow - end_bwd)

    def _bufs_for(self, lo: int, hi: int, device) -> tuple:
        """bf16-wire buffers of bucket [lo, hi): (send, recv) of world·c bf16 elements, the
        chunk sum [c] in fp32 and bf16, and the gathered bf16 [world·c]; allocated on first use
        and reused every step (no allocator traffic on the step's critical path)."""
        key = (lo, hi)
        b = self._wire_bufs.get(key)
        if b is None:
            c = -(-(hi - lo) // self.world)
            b = (torch.zeros(self.world * c, dtype=torch.bfloat16, device=device),
                 torch.empty(self.world * c, dtype=torch.bfloat16, device=device),
                 torch.empty(c, dtype=torch.float32, device=device),
                 torch.empty(c, dtype=torch.bfloat16, device=device),
                 torch.empty(self.world * c, dtype=torch.bfloat16, device=device))
            self._wire_bufs[key] = b
        return b

    def broadcast_params(self, src: int = 0):
        if self.enabled:
            dist.broadcast(self.store.flat, src, group=self.group)
