"""Sharded data-parallel optimizer step (ZeRO stage 1) over the flat buffers.

The replicated path (grad_sync.GradSync) all-reduces the whole fp32 gradient and every rank
applies the identical clipped TF-Adam update to every parameter.  Here, after the backward:

1. reduce-scatter the flat gradient: rank r receives the sum over ranks of its 1/world shard
   (``wire="fp32"``: ``reduce_scatter_tensor``; ``wire="bf16"``: the shards travel as bf16 through
   one ``all_to_all`` and are summed in fp32 on the receiving rank -- half the bytes of the fp32
   exchange, one rounding per value instead of one per ring hop of a bf16 all-reduce);
2. the clip norm: each rank's sum of squares of the norm terms in its shard (the TF per-token
   embedding slot included where it lives), all-reduced as one scalar;
3. clip + TF-Adam on the shard only (Adam slots are touched only there);
4. all-gather the updated parameter shards into every rank's full flat buffer.

Wire bytes equal the fp32 all-reduce's with fp32 (2·(N-1)/N·S), 3/4 of it with the bf16
reduce-scatter; the optimizer's memory traffic drops to 1/world.  ``gather_slots()`` assembles
the full Adam slots before a checkpoint.  Reference: the PS applied Adam once per gradient push
(model.py:98 under replica_device_setter); SURVEY.md §2.4.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from ..engine.optim import TFAdam
from ..models.params import ParamStore


class ShardedStep:
    def __init__(self, store: ParamStore, opt: TFAdam, world: int, rank: int,
                 wire: str = "fp32", group=None):
        if store.numel % (world * 64):
            raise ValueError(f"sharded optimizer: {store.numel} elements do not split into "
                             f"{world} 64-aligned shards (use a world size dividing 64)")
        self.store, self.opt, self.world, self.rank = store, opt, world, rank
        self.group, self.wire = group, wire
        self.shard = store.numel // world
        self.lo, self.hi = rank * self.shard, (rank + 1) * self.shard
        dev = store.flat.device
        self.gshard = torch.empty(self.shard, dtype=torch.float32, device=dev)
        self.sumsq = torch.zeros(1, dtype=torch.float32, device=dev)
        self._recv: Optional[torch.Tensor] = None
        n_norm, use_slot = store.norm_terms()
        self.n_norm, self.use_slot = n_norm, use_slot

    def _reduce_scatter(self) -> None:
        g = self.store.grad
        if self.wire == "bf16":
            send = g.view(self.world, self.shard).to(torch.bfloat16)
            if self._recv is None:
                self._recv = torch.empty_like(send)
            dist.all_to_all_single(self._recv, send, group=self.group)
            torch.sum(self._recv.float(), 0, out=self.gshard)
        else:
            dist.reduce_scatter_tensor(self.gshard, g, op=dist.ReduceOp.SUM, group=self.group)
        self.store.grad[self.lo:self.hi].copy_(self.gshard)

    def _shard_sumsq(self) -> None:
        g = self.store.grad
        a, b = self.lo, min(self.hi, self.n_norm)
        part = g[a:b] if b > a else g[:0]
        self.sumsq.copy_((part.double() * part.double()).sum().float().reshape(1))
        slot = self.store.norm_slot
        if self.use_slot and self.lo <= slot < self.hi:
            self.sumsq += g[slot:slot + 1]
        dist.all_reduce(self.sumsq, group=self.group)

    @torch.no_grad()
    def step(self, lr: float) -> torch.Tensor:
        """Gradients of this rank's batch are complete in ``store.grad``: exchange, update the
        shard, gather the parameters.  Returns the pre-clip global norm (device tensor)."""
        self._reduce_scatter()
        self._shard_sumsq()
        norm = self.opt.step_range(lr, self.lo, self.hi, self.sumsq, grad_scale=1.0 / self.world)
        flat = self.store.flat
        dist.all_gather_into_tensor(flat, flat[self.lo:self.hi].clone(), group=self.group)
        return norm

    @torch.no_grad()
    def gather_slots(self) -> None:
        """Every rank's Adam slot shards into the full m / v buffers (before a checkpoint)."""
        for buf in (self.opt.m, self.opt.v):
            dist.all_gather_into_tensor(buf, buf[self.lo:self.hi].clone(), group=self.group)
