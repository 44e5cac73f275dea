"""Pure-PyTorch (autograd) char-RNN with TensorFlow 1.x cell semantics.

This is the numerical oracle for the HIP kernels and the CPU execution path (tests, gloo
plumbing).  It mirrors the reference graph (model.py:8-103):

* embedding lookup [V,H] -> optional ``dropout(output_keep_prob)`` on the embeddings
  (model.py:58-59, quirk A-13 kept);
* ``num_layers`` cells, each wrapped in ``DropoutWrapper(input_keep_prob, output_keep_prob)``
  when training with a keep-prob < 1 (model.py:27-36);
* static time unroll with shared weights (legacy_seq2seq.rnn_decoder, model.py:72); outputs
  flattened batch-major, row ``b*T + t`` (model.py:73);
* ``logits = out @ softmax_w + softmax_b`` (model.py:76), per-position sparse softmax CE and
  ``cost = sum / B / T`` (model.py:79-85).

Cell math [TF-ext, TF 1.8 rnn_cell_impl / contrib.rnn]:

* LSTMCell: ``[i,j,f,o] = [x,h] @ W + b``; ``c' = s(f+1) c + s(i) tanh(j)``;
  ``h' = s(o) tanh(c')``; state ``(c, h)``.
* GRUCell: ``[r,u] = s([x,h] @ Wg + bg)``; ``c~ = tanh([x, r*h] @ Wc + bc)``;
  ``h' = u h + (1-u) c~``.
* BasicRNNCell: ``h' = tanh([x,h] @ W + b)`` (the reference maps ``rnn`` to the abstract
  ``RNNCell``, bug A-3; we implement the intended BasicRNNCell).
* NASCell (8 branches, no biases): see :func:`nas_cell`.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

from .params import ModelConfig, ParamStore

State = List[Tuple[torch.Tensor, ...]]
LSTM_FORGET_BIAS = 1.0


class _RoundGrad(torch.autograd.Function):
    """Identity forward; the incoming gradient rounded to bf16 (the native backward stores the
    pre-activation gradient dZ in bf16 before its GEMMs)."""

    @staticmethod
    def forward(ctx, z):
        return z.view_as(z)

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).float()


class _RoundVal(torch.autograd.Function):
    """Operand rounded to bf16 forward (the MFMA operands); gradient passed through."""

    @staticmethod
    def forward(ctx, a):
        return a.to(torch.bfloat16).float()

    @staticmethod
    def backward(ctx, g):
        return g


_BF16_OPERANDS = [False]


def _mm(a, b):
    """Every GEMM of the oracle.  Under :func:`bf16_operands` both operands are rounded to bf16
    and the product's incoming gradient too: fp32 math on exactly the operands the native
    kernels feed their bf16 MFMAs, which separates kernel error from operand rounding."""
    if not _BF16_OPERANDS[0]:
        return a @ b
    return _RoundGrad.apply(_RoundVal.apply(a) @ _RoundVal.apply(b))


class bf16_operands:
    """Context manager: the oracle's GEMMs take bf16-rounded operands (see :func:`_mm`)."""

    def __enter__(self):
        self._prev = _BF16_OPERANDS[0]
        _BF16_OPERANDS[0] = True
        return self

    def __exit__(self, *exc):
        _BF16_OPERANDS[0] = self._prev
        return False


def lstm_cell(x, state, kernel, bias):
    c, h = state
    z = _mm(torch.cat([x, h], 1), kernel) + bias
    i, j, f, o = z.chunk(4, 1)
    c2 = torch.sigmoid(f + LSTM_FORGET_BIAS) * c + torch.sigmoid(i) * torch.tanh(j)
    h2 = torch.sigmoid(o) * torch.tanh(c2)
    return h2, (c2, h2)


def gru_cell(x, state, gk, gb, ck, cb):
    (h,) = state
    H = h.shape[1]
    rv = torch.sigmoid(_mm(torch.cat([x, h], 1), gk) + gb)
    r, u = rv[:, :H], rv[:, H:]
    c = torch.tanh(_mm(torch.cat([x, r * h], 1), ck) + cb)
    h2 = u * h + (1 - u) * c
    return h2, (h2,)


def rnn_cell(x, state, kernel, bias):
    (h,) = state
    h2 = torch.tanh(_mm(torch.cat([x, h], 1), kernel) + bias)
    return h2, (h2,)


def nas_preacts(x_proj, m_proj):
    """Combine the 8 input/recurrent branch pre-activations (split 3 is multiplicative)."""
    xs = x_proj.chunk(8, 1)
    ms = m_proj.chunk(8, 1)
    return [xs[k] * ms[k] if k == 3 else xs[k] + ms[k] for k in range(8)]


def nas_pointwise(p, c_prev):
    l1_0 = torch.sigmoid(p[0])
    l1_1 = F.relu(p[1])
    l1_2 = torch.sigmoid(p[2])
    l1_3 = F.relu(p[3])
    l1_4 = torch.tanh(p[4])
    l1_5 = torch.sigmoid(p[5])
    l1_6 = torch.tanh(p[6])
    l1_7 = torch.sigmoid(p[7])
    l2_0 = torch.tanh(l1_0 * l1_1)
    l2_1 = torch.tanh(l1_2 + l1_3)
    l2_2 = torch.tanh(l1_4 * l1_5)
    l2_3 = torch.sigmoid(l1_6 + l1_7)
    l2_0 = torch.tanh(l2_0 + c_prev)  # inject the cell
    new_c = l2_0 * l2_1
    l3_1 = torch.tanh(l2_2 + l2_3)
    new_m = torch.tanh(new_c * l3_1)
    return new_c, new_m


def nas_cell(x, state, kernel, recurrent_kernel):
    c, m = state
    p = nas_preacts(_mm(x, kernel), _mm(m, recurrent_kernel))
    new_c, new_m = nas_pointwise(p, c)
    return new_m, (new_c, new_m)


def cell_step(cfg: ModelConfig, x, state, w: Sequence[torch.Tensor]):
    if cfg.model == "lstm":
        return lstm_cell(x, state, *w)
    if cfg.model == "gru":
        return gru_cell(x, state, *w)
    if cfg.model == "rnn":
        return rnn_cell(x, state, *w)
    return nas_cell(x, state, *w)


def zero_state(cfg: ModelConfig, batch: int, device="cpu", dtype=torch.float32) -> State:
    z = lambda: torch.zeros(batch, cfg.rnn_size, device=device, dtype=dtype)  # noqa: E731
    return [tuple(z() for _ in range(cfg.state_arity)) for _ in range(cfg.num_layers)]


def _dropout(x, keep: float, gen: Optional[torch.Generator]):
    if keep >= 1.0:
        return x
    mask = (torch.rand(x.shape, generator=gen, device=x.device) < keep).to(x.dtype)
    return x * mask / keep


def forward(cfg: ModelConfig, params: dict, x: torch.Tensor, state: State, training: bool = True,
            gen: Optional[torch.Generator] = None, taps: Optional[dict] = None,
            masks: Optional[dict] = None):
    """x: int [B, T].  Returns (logits [B*T, V] batch-major, final_state, outputs [B, T, H]).
    ``taps["emb"]`` receives the embedding_lookup output (the tensor whose gradient TF
    represents as IndexedSlices).  ``masks`` (tests): explicit, already scaled dropout masks in
    the native backend's composed form -- ``in[l]`` [B, T, H] on layer l's input (layer 0:
    embedding x input dropout, l > 0: layer l-1's output x layer l's input dropout) and ``out``
    on the top layer's output -- instead of drawing them here."""
    B, T = x.shape
    emb = params["embedding"][x.long()]  # [B, T, H]
    if taps is not None:
        taps["emb"] = emb
    if masks is not None:
        return _forward_masked(cfg, params, emb, state, masks)
    if training and cfg.output_keep_prob:
        emb = _dropout(emb, cfg.output_keep_prob, gen)
    wrap = training and (cfg.output_keep_prob < 1.0 or cfg.input_keep_prob < 1.0)
    layer_w = [layer_weights(cfg, params, layer) for layer in range(cfg.num_layers)]
    state = [tuple(s) for s in state]
    outs = []
    for t in range(T):
        inp = emb[:, t]
        for layer in range(cfg.num_layers):
            if wrap:
                inp = _dropout(inp, cfg.input_keep_prob, gen)
            out, st = cell_step(cfg, inp, state[layer], layer_w[layer])
            state[layer] = st
            if wrap:
                out = _dropout(out, cfg.output_keep_prob, gen)
            inp = out
        outs.append(inp)
    out = torch.stack(outs, 1)  # [B, T, H]
    logits = _mm(out.reshape(B * T, -1), params["rnnlm/softmax_w"]) + params["rnnlm/softmax_b"]
    return logits, state, out


def _forward_masked(cfg, params, emb, state, masks):
    B, T, _ = emb.shape
    layer_w = [layer_weights(cfg, params, layer) for layer in range(cfg.num_layers)]
    state = [tuple(s) for s in state]
    outs = []
    for t in range(T):
        inp = emb[:, t]
        for layer in range(cfg.num_layers):
            if masks["in"][layer] is not None:
                inp = inp * masks["in"][layer][:, t]
            out, st = cell_step(cfg, inp, state[layer], layer_w[layer])
            state[layer] = st
            inp = out
        if masks.get("out") is not None:
            inp = inp * masks["out"][:, t]
        outs.append(inp)
    out = torch.stack(outs, 1)
    logits = _mm(out.reshape(B * T, -1), params["rnnlm/softmax_w"]) + params["rnnlm/softmax_b"]
    return logits, state, out


def layer_weights(cfg: ModelConfig, params: dict, layer: int):
    from .params import cell_specs

    return [params[s.name] for s in cell_specs(cfg, layer)]


def loss_fn(logits: torch.Tensor, y: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Returns (cost = mean CE over B*T, per-position CE [B*T])."""
    per = F.cross_entropy(logits, y.reshape(-1).long(), reduction="none")
    return per.sum() / per.numel(), per


class ReferenceBackend:
    """Autograd execution of one TBPTT training step; writes grads into the flat buffer."""

    def __init__(self, store: ParamStore, seed: int = 0):
        self.store = store
        self.cfg = store.cfg
        self.gen = torch.Generator(device=store.device.type if store.device.type == "cpu" else "cpu")
        self.gen.manual_seed(seed)

    def _forward(self, cfg, params, x, state, training=True, gen=None, taps=None, masks=None):
        """The model's forward (engine/native/fp32.py swaps in the native fp32 recurrence)."""
        return forward(cfg, params, x, state, training=training, gen=gen, taps=taps, masks=masks)

    def params(self, requires_grad: bool):
        out = {}
        for n in self.store.names():
            v = self.store.view(n)
            out[n] = v.detach().requires_grad_(requires_grad) if requires_grad else v
        return out

    def train_step(self, x, y, state: State, on_bucket_ready=None, want_extras: bool = False,
                   masks: Optional[dict] = None):
        params = self.params(True)
        gen = self.gen if self.store.device.type == "cpu" else None
        taps = {}
        logits, new_state, _ = self._forward(self.cfg, params, x, state, training=True, gen=gen,
                                             taps=taps, masks=masks)
        cost, per = loss_fn(logits, y)
        names = self.store.names()
        grads = torch.autograd.grad(cost, [params[n] for n in names] + [taps["emb"]],
                                    allow_unused=True)
        # TF's clip norm term for the embedding: the per-token IndexedSlices values
        g_tok = grads[-1]
        slot = self.store.norm_slot_view()
        if self.cfg.clip_norm == "tf" and g_tok is not None:
            slot.copy_((g_tok.double() ** 2).sum().reshape(1))
        else:
            slot.zero_()
        # readiness reported tensor by tensor in the flat buffer's order (head, top layer, ...,
        # embedding), as the native backward does, so the data-parallel buckets launch one by
        # one on this path too
        for n, g in zip(names, grads):
            gv = self.store.gview(n)
            if g is None:
                gv.zero_()
            else:
                gv.copy_(g)
            if on_bucket_ready is not None and n != names[-1]:
                sp = self.store.by_name[n]
                on_bucket_ready(sp.offset + sp.numel)
        if on_bucket_ready is not None:
            on_bucket_ready(None)
        detached = [tuple(s.detach() for s in st) for st in new_state]
        return cost.detach(), detached, {"logits": logits.detach(), "loss": per.detach()}

    @torch.no_grad()
    def step_logits(self, x_t: torch.Tensor, state: State):
        """One inference step (B, 1) -> (logits [B, V], new_state); no dropout."""
        logits, new_state, _ = self._forward(self.cfg, self.params(False), x_t, state,
                                             training=False)
        return logits, new_state

    @torch.no_grad()
    def eval_loss(self, x, y, state: State):
        logits, new_state, _ = self._forward(self.cfg, self.params(False), x, state,
                                             training=False)
        cost, _ = loss_fn(logits, y)
        return cost, new_state
