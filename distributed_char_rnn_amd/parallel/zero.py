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
        # RCCL runs the step's per-bucket all-gathers as ONE grouped launch (c10d coalescing);
        # gloo has no coalesced all-gather, it keeps one call per bucket
        self._coalesce = (dist.is_initialized() and dist.get_backend(group) == "nccl"
                          and hasattr(dist, "_coalescing_manager"))
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
        # the owned chunks of the parameters and of Adam's slots, packed like gown: the update
        # is ONE fused launch over them, and the packed parameters are the all-gathers' inputs
        # (no staging copies); opt.m / opt.v hold full copies only after gather_slots
        self.pown = torch.empty(self.shard, dtype=torch.float32, device=dev)
        self.mown = torch.empty(self.shard, dtype=torch.float32, device=dev)
        self.vown = torch.empty(self.shard, dtype=torch.float32, device=dev)
        # [owned sum of squares, this rank's error word as a float]: ONE all-reduce (SUM) gives
        # the global sum of squares and a guard that is non-zero iff any rank's word was
        self.red = torch.zeros(2, dtype=torch.float32, device=dev)
        self.sumsq = self.red[:1]
        self._wire16: Optional[Tuple[torch.Tensor, torch.Tensor]] = None
        if wire == "bf16":
            self._wire16 = (torch.empty(store.numel, dtype=torch.bfloat16, device=dev),
                            torch.empty(store.numel, dtype=torch.bfloat16, device=dev))
        self.n_norm, self.use_slot = store.norm_terms()
        # The norm terms this rank owns are ONE prefix gown[:P] of the packed owned vector: the
        # buckets are in flat order and the norm terms are the flat prefix [0, n_norm) (+ the
        # TF-mode slot, one element holding a sum of squares) -- so the owned sum of squares is
        # one native launch instead of a loop of float64 torch ops per bucket
        self._pre, self._slot_pos, prefix_ok = 0, -1, True
        for (a, b), p in zip(self.own, self.pos):
            e = min(b, self.n_norm)
            if e > a:
                prefix_ok &= p == self._pre
                self._pre = p + (e - a)
            if self.use_slot and a <= store.norm_slot < b:
                self._slot_pos = p + store.norm_slot - a
        # ... and the owned parameters (flat [0, norm_slot): the slot and the tail padding are
        # not parameters) the prefix pown[:Q]
        self._q = 0
        for (a, b), p in zip(self.own, self.pos):
            e = min(b, store.norm_slot)
            if e > a:
                prefix_ok &= p == self._q
                self._q = p + (e - a)
        if not prefix_ok:
            raise AssertionError("sharded optimizer: owned norm terms are not a prefix")
        self.refresh()
        self._ops = None
        if dev.type == "cuda":
            from ..ops import native

            self._ops = native.ops()
            self._npart = torch.empty(max(1, int(self._ops.opt_num_partials(max(self._pre, 1)))),
                                      dtype=torch.float32, device=dev)
            self._ntick = torch.zeros(1, dtype=torch.int32, device=dev)  # the kernel resets it
        self._next = 0
        self._work: list = []
        # bucket indices in launch order of the current step (tests, --profile reports)
        self.launched: List[int] = []
        self.early = 0

    @torch.no_grad()
    def refresh(self) -> None:
        """(Re)pack the owned chunks of the parameters and Adam's slots from the full buffers
        (construction; after a checkpoint restore or broadcast changed them)."""
        for (a, b), p in zip(self.own, self.pos):
            self.pown[p:p + (b - a)].copy_(self.store.flat[a:b])
            self.mown[p:p + (b - a)].copy_(self.opt.m[a:b])
            self.vown[p:p + (b - a)].copy_(self.opt.v[a:b])
        # the packed copies are authoritative from here on: a later change of the full buffers
        # (restore, broadcast: both bump store.version) is picked up by step()'s version check
        self._ver = self.store.version

    # -- the GradSync-compatible interface the backward drives ------------------------------
    def reset(self) -> None:
        self._next = 0
        self._work.clear()
        self.launched = []

    def launches_at(self, upto: Optional[int] = None) -> bool:
        """Whether ``ready(upto)`` would launch a bucket (the backward skips its deferred-sum
        flush for a readiness report that completes none: one tail launch fewer)."""
        if not self.enabled:
            return False
        lim = self.store.numel if upto is None else upto
        return self._next < len(self.buckets) and self.buckets[self._next][1] <= lim

    def ready(self, upto: Optional[int] = None, sync: bool = False) -> None:
        """Launch the reduce-scatter of every not-yet-launched bucket ending at or below flat
        offset ``upto`` (None = everything); ``sync`` as blocking collectives on the caller's
        stream (GradSync.ready)."""
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
                w = dist.all_to_all_single(recv, send, group=self.group, async_op=not sync)
                self._work.append((w, i, recv))
            else:
                w = dist.reduce_scatter_tensor(out, g[lo:hi], op=dist.ReduceOp.SUM,
                                               group=self.group, async_op=not sync)
                self._work.append((w, i, None))
            self.launched.append(i)
            self._next += 1

    # -- the optimizer step ----------------------------------------------------------------
    def _owned_sumsq(self) -> None:
        """Sum of squares of the norm terms this rank owns (reduced gradients), all-reduced:
        one native sumsq launch over the owned prefix gown[:P] (csrc/optim.hip, one-launch
        form), plus the slot element if this rank owns it."""
        pre = self.gown[:self._pre]
        slot = self.gown[self._slot_pos:self._slot_pos + 1] if self._slot_pos >= 0 else None
        if self._pre > 0 and self._ops is not None:
            # the slot term and the error word (as a float value in red[1]) ride in the same
            # launch: no separate add / copy kernels in front of the all-reduce
            self._ops.sumsq(pre, self._npart, self.red, self._ntick, slot, self.guard)
        else:
            if self._pre == 0:
                self.sumsq.zero_()
            else:
                self.sumsq.copy_((pre.double() * pre.double()).sum().float().reshape(1))
            if slot is not None:
                self.sumsq.add_(slot)
            if self.guard is not None:
                self.red[1:].copy_(self.guard)
        dist.all_reduce(self.red, group=self.group)
        if self.guard is not None and self.world > 1:
            # every rank's own word folded in (all ranks skip the update and raise together;
            # at world 1 the reduced word is the rank's own)
            self.guard.bitwise_or_(self.red[1:].view(torch.int32))

    @torch.no_grad()
    def step(self, lr: float) -> torch.Tensor:
        """Gradients of this rank's batch are complete in ``store.grad`` (buckets already
        launched by the backward are not relaunched): finish the exchange, update the owned
        chunks, gather the parameters.  Returns the pre-clip global norm (device tensor)."""
        self.early = len(self.launched)  # buckets the backward launched (reports)
        if self.store.version != self._ver:
            # the full parameter buffer changed since the owned chunks were packed (a restore or
            # broadcast after construction): re-pack, or the all-gather below would overwrite it
            self.refresh()
        # the backward's buckets first, then the rest as blocking collectives (RCCL's internal
        # stream; the current stream waits on them -- nothing is left to overlap)
        for w, i, recv in self._work:
            w.wait()
        self.ready(None, sync=True)
        for w, i, recv in self._work:
            if recv is not None:  # bf16 wire: the owner sums the world copies of its chunk
                c = (self.buckets[i][1] - self.buckets[i][0]) // self.world
                torch.sum(recv.view(self.world, c), 0, dtype=torch.float32,
                          out=self.gown[self.pos[i]:self.pos[i] + c])
        self._work.clear()
        self._next = 0
        self._owned_sumsq()  # (also reduces the error words)
        q = self._q
        norm = self.opt.step_packed(lr, self.pown[:q], self.gown[:q], self.mown[:q],
                                    self.vown[:q], self.sumsq, grad_scale=1.0 / self.world)
        flat = self.store.flat
        # one all-gather per bucket straight from the packed parameters (RCCL: one coalesced
        # group), blocking (the current stream waits on it): the next forward reads the parameters
        if self._coalesce:
            with dist._coalescing_manager(self.group, async_ops=False):
                for (lo, hi), (a, b), p in zip(self.buckets, self.own, self.pos):
                    dist.all_gather_into_tensor(flat[lo:hi], self.pown[p:p + (b - a)],
                                                group=self.group)
        else:
            for (lo, hi), (a, b), p in zip(self.buckets, self.own, self.pos):
                dist.all_gather_into_tensor(flat[lo:hi], self.pown[p:p + (b - a)],
                                            group=self.group)
        self._ver = self.store.version  # (the update above bumped it; flat now matches pown)
        return norm

    @torch.no_grad()
    def gather_slots(self) -> None:
        """Every rank's Adam slot chunks into the full m / v buffers (before a checkpoint)."""
        for buf, own in ((self.opt.m, self.mown), (self.opt.v, self.vown)):
            for (lo, hi), (a, b), p in zip(self.buckets, self.own, self.pos):
                dist.all_gather_into_tensor(buf[lo:hi], own[p:p + (b - a)], group=self.group)
