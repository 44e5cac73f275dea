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
                        space_id: int = -1, use_graph: bool = True, use_generator: bool = True):
        """Device-side autoregressive sampling (model.py:105-140); returns [S][num] ids.

        LSTM models take the single-launch generator (``generate``); otherwise, or with
        ``use_generator=False``:

        Every generated character is [recurrent step kernels of all layers, ``dcr::sample_step``]
        (csrc/sample.hip: softmax head + argmax / inverse-CDF draw, the pick written straight
        into the next step's input id).  The step is captured once into a hipGraph and replayed
        ``num - 1`` times, so the loop runs without a host round trip or per-kernel launch
        cost; the host reads the ids once at the end."""
        from ...models.reference import zero_state

        S = num_samples
        if num <= 0:
            return [[] for _ in range(S)]
        if use_generator and self._generate_ok(S):
            return self.generate(prime_ids, num, sampling_type, seed, S, space_id)[0]
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

    def _generate_ok(self, S: int) -> bool:
        """The single-launch generator (csrc/generate.hip) covers LSTM stacks of up to 4 layers
        with H a multiple of 128 up to 4 x the CU count, up to 16 streams."""
        return (self.cfg.model == "lstm" and self.knobs.on("generate")
                and bool(self.ops.generate_supported(self.L, self.H, self.V, S)))

    @torch.no_grad()
    def generate(self, prime_ids, num: int, sampling_type: int, seed: int, S: int = 1,
                 space_id: int = -1, want_logits: bool = False):
        """Every character of Model.sample (model.py:105-140) in ONE launch: the recurrence of
        all layers, the softmax head and the draw, with the weights resident in LDS across the
        grid (csrc/generate.hip); prime[:-1] warms the zero state inside the launch.  Returns
        (ids [S][num], final state, logits [num, S, V] or None)."""
        from .forward import FORGET_BIAS

        self._run_prep(self._prep())  # weight layouts + the layer-0 gather table current
        hd, dev, L, H = self._head, self.dev, self.L, self.H
        if self._head.get("WsT_gen") is None or self._gen_ver != self._wver:
            self._head["WsT_gen"] = hd["Ws"].t().contiguous()
            self._gen_ver = self._wver
        f32 = dict(dtype=torch.float32, device=dev)
        h0 = torch.zeros(L, S, H, **f32)
        c0 = torch.zeros(L, S, H, **f32)
        h1, c1 = torch.empty_like(h0), torch.empty_like(c0)
        prime = torch.tensor([int(i) for i in prime_ids], dtype=torch.int32, device=dev)
        out = torch.empty(S, num, dtype=torch.int32, device=dev)
        hx = torch.empty(L * 2 * S * H, dtype=torch.int64, device=dev)
        ctr0 = torch.zeros(S, dtype=torch.int32, device=dev)
        lg = torch.empty(num, S, self.V, **f32) if want_logits else None
        w = self._w
        self.ops.generate([lw.Wh for lw in w], [lw.Wx for lw in w], [lw.bias for lw in w],
                          hd["table"], hd["WsT_gen"], hd["bs"], FORGET_BIAS, h0, c0, h1, c1,
                          prime, int(num), out, hx, int(sampling_type), int(space_id),
                          int(seed) & ((1 << 63) - 1), ctr0, lg, self.err, self.spin_limit,
                          getattr(self, "gen_stamps", None))
        ids = out.cpu().tolist()
        self.check_errors()
        state = [(c1[l], h1[l]) for l in range(L)]
        return ids, state, lg

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
