"""Inference of the native backend: next-step logits, evaluation loss and the device-side
sampling loop (the reference's Model.sample, model.py:105-140)."""
from __future__ import annotations

import torch


class InferenceMixin:
    @torch.no_grad()
    def step_logits(self, x_t: torch.Tensor, state):
        ids_tm = x_t.t().contiguous()
        bufs, O, logits, new_state = self._forward(ids_tm, state, False)
        T, B = ids_tm.shape
        lg = logits.view(T, B, self.V)[-1].clone()
        return lg, new_state

    @torch.no_grad()
    def eval_loss(self, x, y, state):
        ids_tm = x.t().contiguous()
        tgt = y.t().contiguous().view(-1)
        bufs, O, logits, new_state = self._forward(ids_tm, state, False,
                                                   want_logits=not (self.fused_head
                                                                    or self.wide_head))
        if self.wide_head:
            self.ops.head_wide(O, self._head["WsTw"], self._head["bs"], tgt, 1.0, None, None,
                               None, None, None, bufs["hw_part"], bufs["loss"][0, :1])
        elif self.fused_head:
            hd = self._head
            self.ops.head(O, hd["WsT"], None, hd["bs"], tgt, 1.0, None, None, None, None, None,
                          bufs["head_part"], bufs["loss"][0, :1])
        else:
            self.ops.xent(logits, tgt, 1.0, None, None, bufs["xpart"], bufs["loss"][0, :1])
        return bufs["loss"][0, 0].clone(), new_state

    @torch.no_grad()
    def sample_sequence(self, prime_ids, num: int, sampling_type: int, seed: int, num_samples: int,
                        space_id: int = -1, use_graph: bool = True):
        """Device-side autoregressive sampling (model.py:105-140); returns [S][num] ids.

        Every generated character is [recurrent step kernels of all layers, ``dcr::sample_step``]
        (csrc/sample.hip: softmax head + argmax / inverse-CDF draw, the pick written straight
        into the next step's input id).  The step is captured once into a hipGraph and replayed
        ``num - 1`` times, so the loop runs without a host round trip or per-kernel launch
        cost; the host reads the ids once at the end."""
        from ...models.reference import zero_state

        S = num_samples
        if num <= 0:
            return [[] for _ in range(S)]
        if not self.ops.sample_supported(self.V, self.H):
            return self._sample_sequence_torch(prime_ids, num, sampling_type, seed, S, space_id)
        state = zero_state(self.cfg, S, self.dev)
        for cid in prime_ids[:-1]:  # warm the state on prime[:-1] (model.py:107-111)
            x = torch.full((S, 1), cid, dtype=torch.int32, device=self.dev)
            _, state = self.step_logits(x, state)
        i32 = dict(dtype=torch.int32, device=self.dev)
        cur = torch.full((S,), int(prime_ids[-1]), **i32)
        out = torch.zeros(S, num, **i32)
        pos = torch.zeros(S, **i32)
        ctr = torch.zeros(S, **i32)
        st = [tuple(t.clone() for t in layer) for layer in state]
        self._run_prep(self._prep())
        WsT = self._head["Ws"].t().contiguous()            # [V, H] bf16, fixed while sampling
        bs = self._head["bs"]
        seed = int(seed) & ((1 << 63) - 1)

        def one():
            _, O, _, new = self._forward(cur.view(1, S), st, False, want_logits=False)
            self.ops.sample_step(O, WsT, bs, cur, out, pos, ctr, None, None, int(sampling_type),
                                 int(space_id), seed)
            for a, b in zip(st, new):
                for x, y in zip(a, b):
                    x.copy_(y)

        one()  # first character eagerly (also allocates the step's buffers)
        if num > 1:
            graph = None
            if use_graph and self.knobs.on("sample_graph"):
                try:
                    graph = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(graph):
                        one()
                except RuntimeError:
                    graph = None
            for _ in range(num - 1):
                if graph is not None:
                    graph.replay()
                else:
                    one()
        return out.cpu().tolist()

    @torch.no_grad()
    def _sample_sequence_torch(self, prime_ids, num, sampling_type, seed, S, space_id):
        """Library-op sampling loop for shapes the sampling kernel does not cover."""
        from ...models.reference import zero_state

        state = zero_state(self.cfg, S, self.dev)
        g = torch.Generator(device=self.dev)
        g.manual_seed(int(seed))
        for cid in prime_ids[:-1]:
            x = torch.full((S, 1), cid, dtype=torch.int32, device=self.dev)
            _, state = self.step_logits(x, state)
        cur = torch.full((S, 1), prime_ids[-1], dtype=torch.int32, device=self.dev)
        out = torch.empty(S, num, dtype=torch.int32, device=self.dev)
        for i in range(num):
            logits, state = self.step_logits(cur, state)
            p = torch.softmax(logits, -1)
            cdf = torch.cumsum(p, -1)
            r = torch.rand(S, 1, device=self.dev, generator=g) * cdf[:, -1:]
            pick = torch.searchsorted(cdf, r).clamp_(max=self.V - 1).to(torch.int32)
            if sampling_type == 0:
                pick = p.argmax(-1, keepdim=True).to(torch.int32)
            elif sampling_type == 2:
                am = p.argmax(-1, keepdim=True).to(torch.int32)
                pick = torch.where(cur == space_id, pick, am)
            out[:, i: i + 1] = pick
            cur = pick
        return out.cpu().tolist()
