"""Long-sequence numerics of the hand-written recurrences (the T x L dependent chain of the
reference, model.py:72, differentiated by tf.gradients, model.py:91).

* the headline shape (2-layer LSTM-512, T = 128, B = 256: the two-layer wavefront kernels)
  against the fp32 autograd oracle (ReferenceBackend, TF cell semantics): loss, final TBPTT
  state and the relative error of every gradient tensor;
* config 3's cell at T = 256 (3-layer GRU-1024, persistent GRU kernels), same comparison;
* a 300-step training run on tinyshakespeare (the reference defaults: 2-layer LSTM-128,
  B = 50, T = 50, Adam 2e-3, clip 5): the native and the oracle loss curves must agree.

The data is the real corpus (data/tinyshakespeare/input.txt, the reference's own file), so
the gradients have the structure of a real training step rather than of uniform noise."""
import os

import numpy as np
import pytest
import torch

from distributed_char_rnn_amd.engine.optim import TFAdam
from distributed_char_rnn_amd.models.char_rnn import CharRNN
from distributed_char_rnn_amd.models.params import ModelConfig
from distributed_char_rnn_amd.models.reference import ReferenceBackend
from distributed_char_rnn_amd.utils import data as D
from oracle import check_grads

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TEXT = os.path.join(ROOT, "data", "tinyshakespeare", "input.txt")


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


@pytest.fixture(scope="module")
def corpus():
    text = D.read_text(TEXT)
    chars, vocab = D.build_vocab(text)
    return D.encode(text, vocab), len(chars)


def _window(ids, B, T, offset=0):
    """B row streams of T+1 tokens (train.py's x / y shift), as [B, T] int32 cuda tensors."""
    n = B * (T + 1)
    w = np.asarray(ids[offset:offset + n]).reshape(B, T + 1)
    x = torch.from_numpy(np.ascontiguousarray(w[:, :T])).cuda()
    y = torch.from_numpy(np.ascontiguousarray(w[:, 1:])).cuda()
    return x, y


def _compare(cfg, B, T, ids, state_scale=0.3, tol_state=3e-2, grad_key="long_t", plan_key=None):
    nat = CharRNN(cfg, device="cuda", seed=17)
    if plan_key is not None:
        plan = nat.backend._persist_plan(B, True, T)
        assert getattr(plan, plan_key), ("not on the hand-written path", plan)
    ref = ReferenceBackend(nat.store)
    x, y = _window(ids, B, T)
    torch.manual_seed(2)
    arity = 2 if cfg.model == "lstm" else 1
    st0 = [tuple(torch.randn(B, cfg.rnn_size, device="cuda") * state_scale for _ in range(arity))
           for _ in range(cfg.num_layers)]
    loss_r, st_r, _ = ref.train_step(x, y, [tuple(s.clone() for s in t) for t in st0])
    g_ref = nat.store.grad.clone()
    nat.store.grad.zero_()
    loss_n, st_n, _ = nat.backend.train_step(x, y, [tuple(s.clone() for s in t) for t in st0])
    torch.cuda.synchronize()
    nat.backend.check_errors()
    assert abs(loss_n.item() - loss_r.item()) < 1e-2 * max(1.0, abs(loss_r.item())), \
        (loss_n.item(), loss_r.item())
    for a_r, a_n in zip(st_r, st_n):
        for s_r, s_n in zip(a_r, a_n):
            assert rel(s_n, s_r) < tol_state
    return check_grads(grad_key, nat.store, nat.store.grad, g_ref)


def test_headline_shape_t128_matches_oracle(corpus, monkeypatch):
    monkeypatch.setenv("DCR_SPIN_LIMIT", str(1 << 22))
    ids, V = corpus
    cfg = ModelConfig(model="lstm", vocab_size=V, rnn_size=512, num_layers=2)
    errs = _compare(cfg, 256, 128, ids, plan_key="pair")
    print({k: f"{v[0]:.2e}/{v[1]:.2e}" for k, v in errs.items()})


def test_gru_t256_matches_oracle(corpus, monkeypatch):
    monkeypatch.setenv("DCR_SPIN_LIMIT", str(1 << 22))
    ids, V = corpus
    cfg = ModelConfig(model="gru", vocab_size=V, rnn_size=1024, num_layers=3)
    errs = _compare(cfg, 64, 256, ids, plan_key="gru_persist")
    print({k: f"{v[0]:.2e}/{v[1]:.2e}" for k, v in errs.items()})


def test_300_step_training_tracks_oracle(corpus):
    """Reference defaults (train.py:37-61) on the real corpus: native bf16 kernels vs the fp32
    autograd oracle, each with its own TF-Adam and TBPTT carry, from the same init."""
    ids, V = corpus
    B, T, steps = 50, 50, 300
    cfg = ModelConfig(model="lstm", vocab_size=V, rnn_size=128, num_layers=2)
    xb, yb, nb, _ = D.make_batches(ids, B, T)
    curves = {}
    for backend in ("native", "reference"):
        m = CharRNN(cfg, device="cuda", seed=23, backend=backend)
        opt = TFAdam(m.store, clip=5.0, guard=m.error_word())
        st = m.zero_state(B)
        losses = []
        for i in range(steps):
            loss, st, _ = m.train_step(xb[i % nb], yb[i % nb], st)
            opt.step(2e-3)
            losses.append(float(loss))
        m.check_errors()
        curves[backend] = np.array(losses)
    a, b = curves["native"], curves["reference"]
    assert a[0] > 4.0 and a[-20:].mean() < 2.6, a[::50]   # it learns (unigram entropy ~3.3)
    # windowed means agree; bf16 trajectories diverge slowly, the curves must not
    for lo in range(0, steps, 50):
        ma, mb = a[lo:lo + 50].mean(), b[lo:lo + 50].mean()
        assert abs(ma - mb) < 0.03 * mb, (lo, ma, mb)
