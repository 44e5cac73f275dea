"""Config 4's large-batch step (BASELINE.json: 4-layer LSTM-2048, large-batch DP) pinned at
B = 1024 -- the batch whose 3-step bench run ends at loss 5.83, above ln 65.

At B = 1024 the plan runs the fused per-step forward kernels (csrc/lstm_gemm_step.hip) and the
library-form BPTT steps (engine/native/libstep.py).  Here, at T = 16:

- one step against the fp32 autograd oracle (models/reference.py, /root/reference/model.py:72,
  91): loss, TBPTT state and every gradient (tests/oracle.py);
- the same step on the all-library route (DCR_RECURRENCE=library);
- three optimizer steps of bench.py's TF-Adam (lr 2e-3, clip 5) on bench.py's synthetic tokens,
  native and oracle each with their own Adam from the same init: the loss curves agree step by
  step, so whatever the curve does at this learning rate is the model's, not the kernels'.
"""
import os

import numpy as np
import pytest
import torch

from distributed_char_rnn_amd.engine.optim import TFAdam
from distributed_char_rnn_amd.models.char_rnn import CharRNN
from distributed_char_rnn_amd.models.params import ModelConfig
from distributed_char_rnn_amd.models.reference import ReferenceBackend
from distributed_char_rnn_amd.utils.data import synthetic_tokens
from oracle import check_grads, rel

pytestmark = pytest.mark.gpu

B, T, H, L, V = 1024, 16, 2048, 4, 65


def _cfg():
    return ModelConfig(model="lstm", vocab_size=V, rnn_size=H, num_layers=L)


def _batches(n):
    toks = synthetic_tokens(n * B * T + 1, V, seed=1000)
    d = torch.from_numpy(toks).cuda()
    xs, ys = d[:-1].view(B, n * T), d[1:].view(B, n * T)
    return [(xs[:, i * T:(i + 1) * T].contiguous(), ys[:, i * T:(i + 1) * T].contiguous())
            for i in range(n)]


def _with_env(key, val, fn):
    old = os.environ.get(key)
    os.environ[key] = val
    try:
        return fn()
    finally:
        if old is None:
            os.environ.pop(key, None)
        else:
            os.environ[key] = old


def test_b1024_step_matches_oracle_and_library():
    x, y = _batches(1)[0]
    nat = CharRNN(_cfg(), device="cuda", seed=11)
    plan = nat.backend._persist_plan(B, True, T)
    assert not plan.persistent, plan  # the per-step route is what this pins
    torch.manual_seed(3)
    st0 = [tuple(torch.randn(B, H, device="cuda") * 0.3 for _ in range(2)) for _ in range(L)]
    cp = lambda: [tuple(s.clone() for s in t) for t in st0]  # noqa: E731
    ref = ReferenceBackend(nat.store)
    loss_r, st_r, _ = ref.train_step(x, y, cp())
    g_ref = nat.store.grad.clone()
    nat.store.grad.zero_()
    loss_n, st_n, _ = nat.backend.train_step(x, y, cp())
    torch.cuda.synchronize()
    nat.backend.check_errors()
    g_nat = nat.store.grad.clone()
    assert abs(loss_n.item() - loss_r.item()) < 1e-2 * abs(loss_r.item()), (loss_n, loss_r)
    for a_r, a_n in zip(st_r, st_n):
        for s_r, s_n in zip(a_r, a_n):
            assert rel(s_n, s_r) < 3e-2
    check_grads("big_batch", nat.store, g_nat, g_ref)

    def lib():
        m = CharRNN(_cfg(), device="cuda", seed=11)
        assert m.backend._lib_step("fwd", B) and m.backend._lib_step("bwd", B)
        loss, _, _ = m.backend.train_step(x, y, cp())
        torch.cuda.synchronize()
        return loss.item(), m.store.grad.clone()

    l_lib, g_lib = _with_env("DCR_RECURRENCE", "library", lib)
    assert abs(l_lib - loss_n.item()) < 1e-3 * abs(l_lib)
    assert rel(g_lib, g_nat) < 2e-2


def test_b1024_three_adam_steps_track_oracle():
    """bench.py's optimizer (TF-Adam lr 2e-3, clip 5) for three steps with the TBPTT carry."""
    batches = _batches(3)
    nat = CharRNN(_cfg(), device="cuda", seed=1234)
    orc = CharRNN(_cfg(), device="cuda", seed=1234)
    assert torch.equal(nat.store.flat, orc.store.flat)
    ref = ReferenceBackend(orc.store)
    opt_n = TFAdam(nat.store, clip=5.0, guard=nat.error_word())
    opt_r = TFAdam(orc.store, clip=5.0)
    sn, sr = nat.zero_state(B), orc.zero_state(B)
    curves = {"native": [], "oracle": []}
    for x, y in batches:
        nat.store.grad.zero_()
        ln, sn, _ = nat.train_step(x, y, sn)
        opt_n.step(2e-3)
        nat.params_changed()
        orc.store.grad.zero_()
        lr_, sr, _ = ref.train_step(x, y, sr)
        opt_r.step(2e-3)
        curves["native"].append(ln.item())
        curves["oracle"].append(lr_.item())
    torch.cuda.synchronize()
    nat.backend.check_errors()
    print({k: [f"{v:.4f}" for v in c] for k, c in curves.items()})
    a, b = np.array(curves["native"]), np.array(curves["oracle"])
    assert np.all(np.abs(a - b) < 2e-2 * np.abs(b)), curves
    assert rel(nat.store.flat, orc.store.flat) < 1e-2
