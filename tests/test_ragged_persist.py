"""Ragged batches (B % 16 != 0) on the persistent GRU and single-layer LSTM kernels
(csrc/gru_persist.hip, csrc/lstm_persist.hip): the batch is padded to whole 16-row tiles inside
the kernels (padded rows live only in the hand-off rings), so the reference default
``--batch_size 50`` (train.py:46) stays on the persistent path.  Checked against the fp32
autograd oracle (TF cell semantics) and against the per-step kernels."""
import pytest
import torch

from distributed_char_rnn_amd.models.char_rnn import CharRNN
from distributed_char_rnn_amd.models.params import ModelConfig
from distributed_char_rnn_amd.models.reference import ReferenceBackend
from oracle import check_grads

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


@pytest.fixture(autouse=True)
def _env(monkeypatch):
    monkeypatch.setenv("DCR_SPIN_LIMIT", str(1 << 20))
    monkeypatch.setenv("DCR_DEBUG", "persist_min_t=1")


def _oracle_check(nat, B, T, H, L, arity):
    ref = ReferenceBackend(nat.store)
    torch.manual_seed(B)
    x = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    y = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    st0 = [tuple(torch.randn(B, H, device="cuda") * 0.5 for _ in range(arity)) for _ in range(L)]
    loss_r, st_r, _ = ref.train_step(x, y, [tuple(s.clone() for s in t) for t in st0])
    g_ref = nat.store.grad.clone()
    nat.store.grad.zero_()
    loss_n, st_n, _ = nat.backend.train_step(x, y, [tuple(s.clone() for s in t) for t in st0])
    torch.cuda.synchronize()
    nat.backend.check_errors()
    assert abs(loss_n.item() - loss_r.item()) < 2e-2 * max(1.0, abs(loss_r.item()))
    for a_r, a_n in zip(st_r, st_n):
        for s_r, s_n in zip(a_r, a_n):
            assert rel(s_n, s_r) < 3e-2
    check_grads("ragged_persist", nat.store, nat.store.grad, g_ref)


@pytest.mark.parametrize("B,T,H,L", [(50, 6, 128, 2), (37, 5, 256, 1), (100, 4, 512, 2),
                                     (200, 3, 1024, 1)])
def test_gru_ragged_batch_on_persistent_kernels(B, T, H, L, dcr_ops):
    assert B % 16 != 0
    assert dcr_ops.gru_persist_ub(H, B) > 0
    cfg = ModelConfig(model="gru", vocab_size=65, rnn_size=H, num_layers=L)
    nat = CharRNN(cfg, device="cuda", seed=3)
    assert nat.backend._persist_plan(B, True, T).gru_persist
    _oracle_check(nat, B, T, H, L, 1)


def test_gru_reference_default_batch_equals_per_step_kernels(monkeypatch):
    """--model gru at the reference default B = 50, T = 50 (train.py:44-46): the persistent
    kernels against the per-step kernels over three carried-state steps."""
    B, T, H = 50, 50, 128
    cfg = ModelConfig(model="gru", vocab_size=65, rnn_size=H, num_layers=2)
    a = CharRNN(cfg, device="cuda", seed=5)
    monkeypatch.setenv("DCR_RECURRENCE", "step")
    b = CharRNN(cfg, device="cuda", seed=5)
    assert a.backend._persist_plan(B, True, T).gru_persist
    assert not b.backend._persist_plan(B, True, T).gru_persist
    g = torch.Generator().manual_seed(2)
    sa, sb = a.zero_state(B), b.zero_state(B)
    for _ in range(3):
        x = torch.randint(0, 65, (B, T), generator=g, dtype=torch.int32).cuda()
        y = torch.randint(0, 65, (B, T), generator=g, dtype=torch.int32).cuda()
        la, sa, _ = a.backend.train_step(x, y, sa)
        lb, sb, _ = b.backend.train_step(x, y, sb)
    torch.cuda.synchronize()
    a.backend.check_errors()
    assert abs(la.item() - lb.item()) < 2e-3
    assert rel(a.store.grad, b.store.grad) < 2e-2
    for u, v in zip(sa, sb):
        assert rel(u[0], v[0]) < 1e-2


@pytest.mark.parametrize("B,T,H,L", [(50, 6, 128, 3), (37, 5, 256, 1)])
def test_lstm_single_layer_persistent_ragged(B, T, H, L, monkeypatch, dcr_ops):
    """Odd layer counts put the top layer on the single-layer persistent kernel (3 layers =
    one pair + one single); L = 1 runs it alone."""
    assert dcr_ops.lstm_persist_supported(H, B)
    cfg = ModelConfig(model="lstm", vocab_size=65, rnn_size=H, num_layers=L)
    nat = CharRNN(cfg, device="cuda", seed=7)
    plan = nat.backend._persist_plan(B, True, T)
    assert plan.persist, plan
    _oracle_check(nat, B, T, H, L, 2)
