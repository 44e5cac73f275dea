"""Sharded data-parallel optimizer step (ZeRO stage 1) over the flat buffers, bucketed and
overlapped with the backward.

The replicated path (grad_sync.GradSync) all-reduces the whole fp32 gradient and every rank
applies the identical clipped TF-Adam update to every parameter.  Here the flat buffer is cut
into buckets (``--bucket_mb``, cut at tensor boundaries rounded down to ``world·64`` elements),
and every bucket is split evenly over the ranks: rank r owns chunk r of every bucket.

1. ``ready(upto)`` -- called by the backward as gradient ranges become final, exactly like
   ``GradSync.ready`` -- launches each complete bucket's reduce-scatter at once (async, on
   RCCL's stream), so the head's and the upper layers' exchange overlaps the rest of the
   backward (``wire="fp32"``: ``reduce_scatter_tensor``; ``wire="bf16"``: the chunks travel as
   bf16 through one ``all_to_all`` and are summed in fp32 by their owner -- half the bytes, one
   rounding per value instead of one per ring hop of a bf16 reduction);
2. ``step(lr)``: the error words are MAX-reduced (a rank whose recurrence timed out poisoned
   the sums: every rank then skips the update), each rank's sum of squares of the norm terms it
   owns (the TF per-token embedding slot included where it lives) is all-reduced as one
   scalar -- the global clip norm;
3. clip + TF-Adam on the owned chunks only (Adam slots are touched only there);
4. one all-gather per bucket of the updated parameter chunks into every rank's flat buffer.

Wire bytes equal the fp32 all-reduce's with fp32 (2·(N-1)/N·S), 3/4 of it with the bf16
exchange; the optimizer's memory traffic drops to 1/world.  ``gather_slots()`` assembles the
full Adam slots before a checkpoint.  Reference: the PS applied Adam once per gradient push
(model.py:98 under replica_device_setter); SURVEY.md §2.4.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

from ..engine.optim import TFAdam
from ..models.params import ParamStore


def shard_buckets(store: ParamStore, world: int, bucket_mb: float) -> List[Tuple[int, int]]:
    """Bucket cuts of the flat buffer for the sharded step: ~``bucket_mb`` slices cut at tensor
    boundaries rounded DOWN to a multiple of ``world·64`` elements (a bucket is then complete as
    soon as the backward reports that boundary), the last one ending at ``store.numel``."""
    unit = world * 64
    if store.numel % unit:
        raise ValueError(f"sharded optimizer: {store.numel} elements do not split into "
                         f"{world} 64-aligned shards (use a world size dividing 64)")
    cap = max(unit, int(bucket_mb * (1 << 20) / 4))
    cuts, lo = [], 0
    for s in store.specs:
        end = (s.offset + s.numel) // unit * unit
        if end - lo >= cap:
            cuts.append((lo, end))
            lo = end
    if store.numel > lo:
        cuts.append((lo, store.numel))
    return cuts


class ShardedStep:
    def __init__(self, store: ParamStore, opt: TFAdam, world: int, rank: int,
                 wire: str = "fp32", group=None, bucket_mb: float = 8.0,
                 guard: Optional[torch.Tensor] = None):
        self.store, self.opt, self.world, self.rank = store, opt, world, rank
        self.group, self.wire, self.guard = group, wire, guard
        self.enabled = True  # the backward's readiness callbacks drive ready()
        self.buckets = shard_buckets(store, world, bucket_mb)
        # this rank's chunk of every bucket, and where it sits in the packed owned vector
        self.own: List[Tuple[int, int]] = []
        self.pos: List[int] = []
        p = 0
        for lo, hi in self.buckets:
            c = (hi - lo) // world
            self.own.append((lo + rank * c, lo + (rank + 1) * c))
            self.pos.append(p)
            p += c
        self.shard = p  # = store.numel // world
        dev = store.flat.device
        self.gown = torch.empty(self.shard, dtype=torch.float32, device=dev)   # reduced grads
        self.pown = torch.empty(self.shard, dtype=torch.float32, device=dev)   # gather staging
        self.sumsq = torch.zeros(1, dtype=torch.float32, device=dev)
        self._wire16: Optional[Tuple[torch.Tensor, torch.Tensor]] = None
        if wire == "bf16":
            self._wire16 = (torch.empty(store.numel, dtype=torch.bfloat16, device=dev),
                            torch.empty(store.numel, dtype=torch.bfloat16, device=dev))
        self.n_norm, self.use_slot = store.norm_terms()
        self._next = 0
        self._work: list = []
        # bucket indices in launch order of the current step (tests, --profile reports)
        self.launched: List[int] = []

    # -- the GradSync-compatible interface the backward drives ------------------------------
    def reset(self) -> None:
        self._next = 0
        self._work.clear()
        self.launched = []

    def ready(self, upto: Optional[int] = None) -> None:
        """Launch the reduce-scatter of every not-yet-launched bucket ending at or below flat
        offset ``upto`` (None = everything)."""
        lim = self.store.numel if upto is None else upto
        g = self.store.grad
        while self._next < len(self.buckets) and self.buckets[self._next][1] <= lim:
            i = self._next
            lo, hi = self.buckets[i]
            c = (hi - lo) // self.world
            out = self.gown[self.pos[i]:self.pos[i] + c]
            if self._wire16 is not None:
                send, recv = (b[lo:hi] for b in self._wire16)
                send.copy_(g[lo:hi])
                w = dist.all_to_all_single(recv, send, group=self.group, async_op=True)
                self._work.append((w, i, recv))
            else:
                w = dist.reduce_scatter_tensor(out, g[lo:hi], op=dist.ReduceOp.SUM,
                                               group=self.group, async_op=True)
                self._work.append((w, i, None))
            self.launched.append(i)
            self._next += 1

    # -- the optimizer step ----------------------------------------------------------------
    def _owned_sumsq(self) -> None:
        """Sum of squares of the norm terms this rank owns (reduced gradients), all-reduced."""
        acc = torch.zeros((), dtype=torch.float64, device=self.gown.device)
        for (a, b), p in zip(self.own, self.pos):
            e = min(b, self.n_norm)
            if e > a:
                part = self.gown[p:p + (e - a)].double()
                acc = acc + (part * part).sum()
        slot = self.store.norm_slot
        if self.use_slot:
            for (a, b), p in zip(self.own, self.pos):
                if a <= slot < b:
                    acc = acc + self.gown[p + slot - a].double()
        self.sumsq.copy_(acc.float().reshape(1))
        dist.all_reduce(self.sumsq, group=self.group)

    @torch.no_grad()
    def step(self, lr: float) -> torch.Tensor:
        """Gradients of this rank's batch are complete in ``store.grad`` (buckets already
        launched by the backward are not relaunched): finish the exchange, update the owned
        chunks, gather the parameters.  Returns the pre-clip global norm (device tensor)."""
        self.ready(None)
        for w, i, recv in self._work:
            w.wait()
            if recv is not None:  # bf16 wire: the owner sums the world copies of its chunk
                c = (self.buckets[i][1] - self.buckets[i][0]) // self.world
                torch.sum(recv.view(self.world, c), 0, dtype=torch.float32,
                          out=self.gown[self.pos[i]:self.pos[i] + c])
        self._work.clear()
        self._next = 0
        g = self.store.grad
        for (a, b), p in zip(self.own, self.pos):
            g[a:b].copy_(self.gown[p:p + (b - a)])
        if self.guard is not None:
            dist.all_reduce(self.guard, op=dist.ReduceOp.MAX, group=self.group)
        self._owned_sumsq()
        norm = self.opt.step_ranges(lr, self.own, self.sumsq, grad_scale=1.0 / self.world)
        flat = self.store.flat
        for (lo, hi), (a, b), p in zip(self.buckets, self.own, self.pos):
            stage = self.pown[p:p + (b - a)]
            stage.copy_(flat[a:b])
            dist.all_gather_into_tensor(flat[lo:hi], stage, group=self.group)
        return norm

    @torch.no_grad()
    def gather_slots(self) -> None:
        """Every rank's Adam slot chunks into the full m / v buffers (before a checkpoint)."""
        for buf in (self.opt.m, self.opt.v):
            for (lo, hi), (a, b), p in zip(self.buckets, self.own, self.pos):
                stage = self.pown[p:p + (b - a)]
                stage.copy_(buf[a:b])
                dist.all_gather_into_tensor(buf[lo:hi], stage, group=self.group)
