"""Whole-training-step hipGraph (``--graph``): forward, fused head, BPTT, weight gradients and
the fused clip + TF-Adam update captured once and replayed every step.

A step of a small configuration -- the reference's default 2-layer LSTM-128, B = 50, T = 50
(train.py:37-61) -- is ~40 short launches whose host-side cost (Python dispatch + launch)
exceeds the GPU time; a replayed graph issues them with one call.  The reference pays the
same per-step host cost in TF's ``Session.run`` (train.py:199).

What changes from step to step is kept in device memory the graph reads:

* the token ids: copied into static [B, T] buffers before a replay;
* the TBPTT carry: the captured step ends by copying its final state into the static state
  tensors it read at the start, which are returned as the new state (passing them back in
  costs nothing; any other state -- an epoch's zero state, a restored carry -- is copied in);
* the learning rate: Adam reads lr_t = lr·sqrt(1-b2^t)/(1-b1^t) from a device scalar written
  before the replay; the step counter t and the parameter version advance on the host;
* the loss: cloned out of the graph's buffer after the replay.

Not captured (``GraphedStep.supported`` says why): data parallelism (the all-reduce buckets are
released by host callbacks), dropout (its mask seeds are per-step host values) and summary steps
that want the logits (run eagerly).  The persistent kernels' error word is polled outside the
graph (a non-blocking copy every ERR_POLL_EVERY-th replay, read one replay later), as in eager
mode.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch


class GraphedStep:
    def __init__(self, model, opt, log=print):
        self.model, self.opt, self.log = model, opt, log
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.failed = False
        self.shape: Optional[Tuple[int, int]] = None
        self.x = self.y = None
        self.state_in: List[Tuple[torch.Tensor, ...]] = []
        self.loss = None
        self.lr_dev = torch.zeros(1, dtype=torch.float32, device=model.device)
        self.replays = 0
        self.warm = 0  # eager steps before the capture (library handles, workspaces, buffers)

    @staticmethod
    def supported(model, world: int) -> Tuple[bool, str]:
        from .native import NativeBackend

        if model.device.type != "cuda" or not isinstance(model.backend, NativeBackend):
            return False, "needs the native GPU backend (rnn_size a multiple of 32)"
        if world > 1:
            return False, "data parallel: the all-reduce buckets are released by host callbacks"
        c = model.cfg
        if c.input_keep_prob < 1.0 or c.output_keep_prob < 1.0:
            return False, "dropout masks are seeded per step on the host"
        return True, ""

    def _capture(self, x, y, state, lr: float) -> None:
        be = self.model.backend
        B, T = x.shape
        self.shape = (B, T)
        self.x, self.y = x.clone(), y.clone()
        self.state_in = [tuple(t.clone() for t in layer) for layer in state]
        torch.cuda.synchronize()
        if (getattr(self.opt, "fused", None) is be and be._wver == self.model.store.version
                and be.knobs.dbg("graph_refresh", "0") != "1"):
            # the fused Adam writes every layout itself: the captured prep launch carries only
            # what it leaves behind (GRU: the fp32 concatenations; nothing for LSTM / RNN)
            be._post_adam = list(getattr(be, "_gru_f32_tasks", []))
        else:
            be._wver = None  # the captured prep launch must refresh the layouts every replay
        g = torch.cuda.CUDAGraph()
        # the capture records one optimizer step without running it: its host counters (Adam's
        # t, the parameter version, the backend's step count) are restored whether or not the
        # capture succeeds -- an eager fallback after a failed capture would otherwise apply
        # Adam's bias correction one step off for the rest of the run
        t0, v0, s0 = self.opt.t, self.model.store.version, be._steps
        be.capturing = True
        try:
            with torch.cuda.graph(g):
                loss, new_state, _ = be.train_step(self.x, self.y, self.state_in)
                self.opt.step(lr, lr_dev=self.lr_dev)
                for dst, src in zip(self.state_in, new_state):
                    for d, s in zip(dst, src):
                        d.copy_(s)
        finally:
            be.capturing = False
            self.opt.t, self.model.store.version, be._steps = t0, v0, s0
            be._wver = None  # the captured layout refresh has not run: an eager step redoes it
        self.loss = loss
        self.graph = g

    def __call__(self, x, y, state, lr: float):
        """One training step; returns (loss tensor, new state).  Falls back to the eager step
        if the capture fails (logged once)."""
        xi = x if isinstance(x, torch.Tensor) else torch.from_numpy(x)
        yi = y if isinstance(y, torch.Tensor) else torch.from_numpy(y)
        xi = xi.to(self.model.device, torch.int32, non_blocking=True)
        yi = yi.to(self.model.device, torch.int32, non_blocking=True)
        if self.failed or self.warm < 1:
            self.warm += 1
            return self._eager(xi, yi, state, lr)
        if self.graph is None or self.shape != tuple(xi.shape):
            try:
                self._capture(xi, yi, state, lr)
            except RuntimeError as e:  # capture unsupported on this build / op
                self.failed, self.graph = True, None
                self.log(f"--graph: capture failed ({e}); running the step eagerly")
                torch.cuda.synchronize()
                return self._eager(xi, yi, state, lr)
        else:
            self.x.copy_(xi)
            self.y.copy_(yi)
        for dst, src in zip(self.state_in, state):
            for d, s in zip(dst, src):
                if d.data_ptr() != s.data_ptr():
                    d.copy_(s)
        self.lr_dev.fill_(self.opt.lr_t(lr))
        self.graph.replay()
        self.opt.t += 1
        self.model.store.version += 1
        self.replays += 1
        # the replay ran a training step: count it, so _poll_errors' every-k-th non-blocking
        # copy of the error word happens during replays as in eager mode
        be = self.model.backend
        be._steps += 1
        be._poll_errors()
        return self.loss.clone(), self.state_in

    def _eager(self, x, y, state, lr):
        loss, new_state, _ = self.model.train_step(x, y, state)
        self.opt.step(lr)
        return loss, new_state
