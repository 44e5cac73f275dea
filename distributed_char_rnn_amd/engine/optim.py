"""TF-1.x-compatible Adam with global-norm clipping over the flat parameter buffer.

Reference: ``grads, _ = clip_by_global_norm(tf.gradients(cost, tvars), grad_clip)`` then
``AdamOptimizer(lr).apply_gradients(...)`` (model.py:88-98), lr assigned per epoch as
``learning_rate * decay_rate ** epoch`` (train.py:146-148, 187).  TF's Adam uses the
"epsilon-hat" form: ``lr_t = lr * sqrt(1 - b2^t) / (1 - b1^t)``,
``theta -= lr_t * m / (sqrt(v) + eps)`` with ``b1 = .9, b2 = .999, eps = 1e-8`` [TF-ext].
The embedding's IndexedSlices update in TF decays m/v densely and updates every row, which is
exactly dense Adam with a zero gradient for unseen rows, so one dense kernel matches it.  The
global norm, however, sees the IndexedSlices *values* (one row per token, duplicates not yet
summed), so with ``ModelConfig.clip_norm == "tf"`` the dense embedding gradient is left out of
the norm and the per-token sum of squares in ``ParamStore.norm_slot`` (written by the backend's
backward) is added instead.

On the GPU the whole update is the two-launch fused kernel in ``csrc/optim.hip``; on CPU the
same math runs as torch ops.
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from ..models.params import ParamStore


def lr_for_epoch(learning_rate: float, decay_rate: float, epoch: int) -> float:
    return float(learning_rate) * float(decay_rate) ** int(epoch)


class TFAdam:
    def __init__(self, store: ParamStore, beta1: float = 0.9, beta2: float = 0.999,
                 eps: float = 1e-8, clip: float = 5.0, bf16_mirror: bool = False,
                 guard: Optional[torch.Tensor] = None):
        """``guard``: a device error word (the persistent kernels' timeout word); while it is
        non-zero the fused kernel skips the update on device, so a timed-out step never
        corrupts the weights or the Adam slots."""
        self.store = store
        self.guard = guard
        self.b1, self.b2, self.eps, self.clip = beta1, beta2, eps, clip
        self.m = torch.zeros_like(store.flat)
        self.v = torch.zeros_like(store.flat)
        # number of update STEPS taken (TF beta{1,2}_power = b^t after t steps).  A step whose
        # update the guard skipped (a persistent-kernel timeout) still counts: the skip is
        # decided on the device and the host cannot know it without a sync, so t -- and with it
        # Adam's bias correction -- then runs one step ahead of the updates actually applied
        # (the CPU path counts the same way, so both paths agree).  A timed-out step raises at
        # the next error poll anyway; resuming from the last checkpoint restores t exactly.
        self.t = 0
        self.native = store.device.type == "cuda"
        self.last_norm = torch.zeros(1, device=store.device)
        self.mirror: Optional[torch.Tensor] = None
        # a backend that runs the update as its fused step-tail launch (csrc/tail.hip: Adam +
        # the bf16 weight layouts + the gather table in one pass), bound by
        # CharRNN.bind_optimizer; None: the two-launch kernel below
        self.fused = None
        if bf16_mirror:
            self.mirror = store.flat.to(torch.bfloat16)
        if self.native:
            from ..ops import native

            self._ops = native.ops()
            self._partials = torch.zeros(self._ops.opt_num_partials(store.numel),
                                         device=store.device)

    def lr_t(self, lr: float) -> float:
        t = self.t + 1
        return lr * math.sqrt(1.0 - self.b2 ** t) / (1.0 - self.b1 ** t)

    @torch.no_grad()
    def step(self, lr: float, grad_scale: float = 1.0,
             lr_dev: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Clip the flat gradient (times ``grad_scale``: 1/world when the data-parallel average
        is folded in here, see ``GradSync.finish(defer_scale=True)``) by global norm and apply
        one update.  Returns the pre-clip global norm as a 1-element device tensor (no host
        sync).  ``lr_dev``: a device fp32 scalar the kernel reads lr_t from (a step captured in
        a hipGraph; the caller writes ``lr_t(lr)`` into it before every replay)."""
        lr_t = self.lr_t(lr)
        st = self.store
        if self.fused is not None and self.fused.fused_adam(self, lr_t, grad_scale, lr_dev):
            self.t += 1
            st.version += 1
            self.fused.fused_adam_done()
            return self.last_norm
        n = st.norm_slot  # every parameter; the norm slot and the padding after it are not
        p, g, m, v = (b.narrow(0, 0, n) for b in (st.flat, st.grad, self.m, self.v))
        n_norm, use_slot = st.norm_terms()
        slot = st.norm_slot_view() if use_slot else None
        if self.native:
            mirror = self.mirror.narrow(0, 0, n) if self.mirror is not None else None
            self._ops.adam_clip(p, g, m, v, mirror, self._partials, self.last_norm, lr_t,
                                self.b1, self.b2, self.eps, self.clip, float(grad_scale), n_norm,
                                slot, self.guard, lr_dev)
        else:
            gn = g.narrow(0, 0, n_norm).double()
            sq = (gn * gn).sum() + (slot.double().sum() if slot is not None else 0.0)
            norm = torch.sqrt(sq).float() * grad_scale
            s = self.clip / torch.clamp(norm, min=self.clip) if self.clip > 0 else torch.ones(())
            self.last_norm.copy_(norm.reshape(1))
            if not self._guard_set():
                gs = g * (s * grad_scale)
                m.mul_(self.b1).add_(gs, alpha=1 - self.b1)
                v.mul_(self.b2).addcmul_(gs, gs, value=1 - self.b2)
                p.sub_(lr_t * m / (v.sqrt() + self.eps))
            if self.mirror is not None:
                self.mirror.copy_(st.flat)
        self.t += 1
        self.store.version += 1
        return self.last_norm

    @torch.no_grad()
    def step_packed(self, lr: float, p: torch.Tensor, g: torch.Tensor, m: torch.Tensor,
                    v: torch.Tensor, sumsq: torch.Tensor, grad_scale: float = 1.0) -> torch.Tensor:
        """One update (Adam step t -> t+1) of a packed parameter vector ``p`` with its own packed
        gradient / slot vectors (the sharded step's owned chunks, parallel/zero.py), clipped by
        the GLOBAL norm sqrt(``sumsq``) * grad_scale: ONE fused launch however many buckets the
        chunks come from."""
        lr_t = self.lr_t(lr)
        if p.numel() and self.native:
            self._ops.adam_clip(p, g, m, v, None, self._partials, self.last_norm, lr_t, self.b1,
                                self.b2, self.eps, self.clip, float(grad_scale), 0, sumsq,
                                self.guard)
        else:
            norm = torch.sqrt(sumsq.double().sum()).float() * grad_scale
            self.last_norm.copy_(norm.reshape(1))
            if p.numel() and not self._guard_set():
                s = self.clip / torch.clamp(norm, min=self.clip) if self.clip > 0 else torch.ones(())
                gs = g * (s * grad_scale)
                m.mul_(self.b1).add_(gs, alpha=1 - self.b1)
                v.mul_(self.b2).addcmul_(gs, gs, value=1 - self.b2)
                p.sub_(lr_t * m / (v.sqrt() + self.eps))
        self.t += 1
        self.store.version += 1
        return self.last_norm

    @torch.no_grad()
    def step_range(self, lr: float, lo: int, hi: int, sumsq: torch.Tensor,
                   grad_scale: float = 1.0) -> torch.Tensor:
        """One update of the parameters [lo, hi) only, clipped by the GLOBAL norm
        sqrt(``sumsq``) * grad_scale (a 1-element device tensor: the sum of squares of every
        norm term, already reduced over ranks)."""
        return self.step_ranges(lr, [(lo, hi)], sumsq, grad_scale)

    @torch.no_grad()
    def step_ranges(self, lr: float, ranges, sumsq: torch.Tensor,
                    grad_scale: float = 1.0) -> torch.Tensor:
        """One update (one Adam step t -> t+1) of the parameters in each [lo, hi) of
        ``ranges``, clipped by the GLOBAL norm sqrt(``sumsq``) * grad_scale.  The sharded
        data-parallel step (parallel/zero.py) calls this with the chunks a rank owns."""
        lr_t = self.lr_t(lr)
        applied = False
        for lo, hi in ranges:
            hi = min(hi, self.store.norm_slot)  # the norm slot and the tail padding: not params
            if hi <= lo:
                continue
            applied = True
            p, g, m, v = (b[lo:hi] for b in (self.store.flat, self.store.grad, self.m, self.v))
            if self.native:
                self._ops.adam_clip(p, g, m, v, None, self._partials, self.last_norm, lr_t,
                                    self.b1, self.b2, self.eps, self.clip, float(grad_scale), 0,
                                    sumsq, self.guard)
            else:
                norm = torch.sqrt(sumsq.double().sum()).float() * grad_scale
                self.last_norm.copy_(norm.reshape(1))
                if self._guard_set():
                    continue
                s = self.clip / torch.clamp(norm, min=self.clip) if self.clip > 0 else torch.ones(())
                gs = g * (s * grad_scale)
                m.mul_(self.b1).add_(gs, alpha=1 - self.b1)
                v.mul_(self.b2).addcmul_(gs, gs, value=1 - self.b2)
                p.sub_(lr_t * m / (v.sqrt() + self.eps))
        if not applied:  # a rank owning only the norm slot / tail padding: nothing to update
            self.last_norm.copy_((torch.sqrt(sumsq.sum()) * grad_scale).reshape(1))
        self.t += 1
        self.store.version += 1
        return self.last_norm

    def _guard_set(self) -> bool:
        """CPU path: the error word is set (the GPU kernel reads it on device instead)."""
        return self.guard is not None and bool(int(self.guard.reshape(-1)[0]))

    # -- checkpoint support (TF slot names) ----------------------------------------------
    def slot_state(self):
        """TF-named Adam slots + beta powers for the checkpoint."""
        out = {}
        for s in self.store.specs:
            out[f"{s.name}/Adam"] = self.store.view(s.name, self.m).detach().cpu().clone()
            out[f"{s.name}/Adam_1"] = self.store.view(s.name, self.v).detach().cpu().clone()
        out["beta1_power"] = torch.tensor(self.b1 ** (self.t + 1), dtype=torch.float32)
        out["beta2_power"] = torch.tensor(self.b2 ** (self.t + 1), dtype=torch.float32)
        return out

    def load_slot_state(self, sd) -> None:
        for s in self.store.specs:
            if f"{s.name}/Adam" in sd:
                self.store.view(s.name, self.m).copy_(torch.as_tensor(sd[f"{s.name}/Adam"]))
                self.store.view(s.name, self.v).copy_(torch.as_tensor(sd[f"{s.name}/Adam_1"]))
        if "beta1_power" in sd:
            bp = float(torch.as_tensor(sd["beta1_power"]))
            # TF stores b1^(t+1) after t updates; invert (robust to float rounding)
            self.t = max(0, int(round(math.log(bp) / math.log(self.b1))) - 1)
        if self.mirror is not None:
            self.mirror.copy_(self.store.flat)
