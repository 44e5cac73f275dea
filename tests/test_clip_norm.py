"""TF 1.x clip-norm semantics for the embedding gradient (CPU).

The reference clips with ``tf.clip_by_global_norm(tf.gradients(cost, tvars), grad_clip)``
(model.py:91-92).  The embedding's gradient there is an IndexedSlices whose *values* are the
per-token rows of d cost / d embedding_lookup(...) -- duplicates not yet summed -- and
``global_norm`` squares those values [TF-ext].  ``clip_norm="tf"`` reproduces that (the backend
writes the per-token sum of squares into ParamStore.norm_slot, the optimizer swaps it in for
the dense embedding term); ``clip_norm="dense"`` is the norm of the summed gradient."""
import math

import pytest
import torch

from distributed_char_rnn_amd.engine.optim import TFAdam
from distributed_char_rnn_amd.models.params import ModelConfig, ParamStore
from distributed_char_rnn_amd.models.reference import ReferenceBackend, forward, loss_fn


def _setup(mode, V=11, H=16, L=2, B=4, T=7):
    cfg = ModelConfig(model="lstm", vocab_size=V, rnn_size=H, num_layers=L, clip_norm=mode)
    store = ParamStore(cfg, seed=2)
    g = torch.Generator().manual_seed(5)
    x = torch.randint(0, V, (B, T), generator=g, dtype=torch.int32)
    y = torch.randint(0, V, (B, T), generator=g, dtype=torch.int32)
    st = [tuple(torch.zeros(B, H) for _ in range(2)) for _ in range(L)]
    return cfg, store, x, y, st


def _tf_norm_brute(cfg, store, x, y, st):
    """IndexedSlices values = per-token gradients of the lookup output; dense grads for the
    rest -- computed independently of the backend."""
    params = {n: store.view(n).detach().clone().requires_grad_(True) for n in store.names()}
    taps = {}
    logits, _, _ = forward(cfg, params, x, st, training=True, taps=taps)
    cost, _ = loss_fn(logits, y)
    names = [n for n in store.names() if n != "embedding"]
    grads = torch.autograd.grad(cost, [params[n] for n in names] + [taps["emb"]])
    sq = sum((g.double() ** 2).sum() for g in grads)
    return math.sqrt(float(sq))


def test_tf_mode_norm_uses_per_token_values():
    cfg, store, x, y, st = _setup("tf")
    ReferenceBackend(store).train_step(x, y, st)
    assert float(store.norm_slot_view()) > 0
    want = _tf_norm_brute(cfg, store, x, y, st)  # (before the update changes the params)
    opt = TFAdam(store, clip=1e9)
    norm = float(opt.step(1e-3))
    assert norm == pytest.approx(want, rel=1e-5)


def test_dense_mode_norm_is_the_flat_gradient_norm():
    cfg, store, x, y, st = _setup("dense")
    ReferenceBackend(store).train_step(x, y, st)
    assert float(store.norm_slot_view()) == 0.0
    dense = float(torch.sqrt((store.grad.double() ** 2).sum()))
    norm = float(TFAdam(store, clip=1e9).step(1e-3))
    assert norm == pytest.approx(dense, rel=1e-5)


def test_modes_differ_with_repeated_tokens_and_clip_follows_the_norm():
    """Repeated ids: the summed row norm differs from the per-token norm, and the clip scale
    (hence the update) follows the selected definition."""
    res = {}
    for mode in ("tf", "dense"):
        cfg, store, x, y, st = _setup(mode, V=3)  # 3 symbols over 28 tokens: heavy collisions
        ReferenceBackend(store).train_step(x, y, st)
        opt = TFAdam(store, clip=1e-3)  # always clipping
        norm = float(opt.step(1e-2))
        res[mode] = (norm, opt.m.narrow(0, 0, store.norm_slot).clone())
    n_tf, m_tf = res["tf"]
    n_dense, m_dense = res["dense"]
    assert n_tf != pytest.approx(n_dense, rel=1e-3)
    # first Adam step: m = (1 - b1) * (clip / norm) * g, so the two m's differ by the norm ratio
    torch.testing.assert_close(m_tf * (n_tf / n_dense), m_dense, rtol=1e-4, atol=1e-12)


def test_norm_slot_is_never_updated_and_outside_every_tensor():
    cfg, store, x, y, st = _setup("tf")
    end = max(s.offset + s.numel for s in store.specs)
    assert store.norm_slot >= end
    ReferenceBackend(store).train_step(x, y, st)
    before = store.flat[store.norm_slot:].clone()
    TFAdam(store).step(1e-2)
    assert torch.equal(store.flat[store.norm_slot:], before)


def test_cli_flag_reaches_the_model_config():
    from distributed_char_rnn_amd.engine.trainer import build_model
    from distributed_char_rnn_amd.utils.config import train_parser

    for flag, want in (([], "tf"), (["--clip_norm", "dense"], "dense")):
        args = train_parser().parse_args(["--rnn_size", "16", "--num_layers", "1"] + flag)
        model = build_model(args, 7, "cpu")
        assert model.store.cfg.clip_norm == want
    with pytest.raises(SystemExit):
        train_parser().parse_args(["--clip_norm", "bogus"])
