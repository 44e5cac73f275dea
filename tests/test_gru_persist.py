"""Persistent GRU kernels (csrc/gru_persist.hip) vs the fp32 autograd oracle (TF GRUCell
semantics: reset before the candidate matmul) and vs the per-step GRU kernels."""
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
def _short_spins(monkeypatch):
    monkeypatch.setenv("DCR_SPIN_LIMIT", str(1 << 20))
    monkeypatch.setenv("DCR_DEBUG", "persist_min_t=1")  # short test sequences still take these kernels


def _model(B, H, L, seed=3, **kw):
    cfg = ModelConfig(model="gru", vocab_size=65, rnn_size=H, num_layers=L, **kw)
    nat = CharRNN(cfg, device="cuda", seed=seed)
    return cfg, nat


@pytest.mark.parametrize("B,T,H,L", [(32, 6, 128, 2), (48, 5, 256, 1), (16, 4, 1024, 1),
                                     (128, 3, 1024, 2), (64, 7, 384, 3)])
def test_gru_persist_matches_reference(B, T, H, L):
    cfg, nat = _model(B, H, L)
    assert nat.backend._persist_plan(B, True).gru_persist, "expected the persistent path"
    ref = ReferenceBackend(nat.store)
    torch.manual_seed(1)
    x = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    y = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    st0 = [(torch.randn(B, H, device="cuda") * 0.5,) for _ in range(L)]
    loss_r, st_r, _ = ref.train_step(x, y, [tuple(s.clone() for s in t) for t in st0])
    g_ref = nat.store.grad.clone()
    nat.store.grad.zero_()
    loss_n, st_n, _ = nat.backend.train_step(x, y, [tuple(s.clone() for s in t) for t in st0])
    torch.cuda.synchronize()
    nat.backend.check_errors()
    assert abs(loss_n.item() - loss_r.item()) < 2e-2 * max(1.0, abs(loss_r.item()))
    for a_r, a_n in zip(st_r, st_n):
        assert rel(a_n[0], a_r[0]) < 3e-2
    check_grads("gru_persist", nat.store, nat.store.grad, g_ref)


def test_gru_persist_equals_per_step_kernels(monkeypatch):
    """Same bf16 math, different schedule: agreement to accumulation-order noise."""
    B, T, H = 64, 16, 256
    _, a = _model(B, H, 2, seed=5)
    monkeypatch.setenv("DCR_RECURRENCE", "step")
    _, b = _model(B, H, 2, seed=5)
    assert a.backend._persist_plan(B, True).gru_persist
    assert not b.backend._persist_plan(B, True).gru_persist
    x = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    la, sa, _ = a.backend.train_step(x, x, a.zero_state(B))
    lb, sb, _ = b.backend.train_step(x, x, b.zero_state(B))
    torch.cuda.synchronize()
    a.backend.check_errors()
    assert abs(la.item() - lb.item()) < 1e-3
    assert rel(a.store.grad, b.store.grad) < 1e-2
    assert rel(sa[1][0], sb[1][0]) < 1e-2
    # inference path (step_logits / eval) goes through the same persistent forward
    ea, _ = a.backend.eval_loss(x, x, a.zero_state(B))
    eb, _ = b.backend.eval_loss(x, x, b.zero_state(B))
    assert abs(ea.item() - eb.item()) < 1e-3


def test_gru_persist_dropout_and_long_sequence():
    B, T, H = 32, 96, 128
    _, m = _model(B, H, 2, input_keep_prob=0.9, output_keep_prob=0.8)
    x = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    st = m.zero_state(B)
    for _ in range(3):
        loss, st, _ = m.backend.train_step(x, x, st)
    torch.cuda.synchronize()
    m.backend.check_errors()
    assert torch.isfinite(loss) and torch.isfinite(m.store.grad).all()


@pytest.mark.parametrize("B,T,H,nt", [(64, 5, 256, 2), (64, 4, 512, 4), (96, 3, 1024, 2),
                                      (256, 3, 1024, 0)])
def test_gru_batch_tiles_per_workgroup(B, T, H, nt, monkeypatch):
    """NT batch tiles per workgroup (gru_nt forced; nt = 0: the planner's own choice, NT = 2 at
    B = 256, H = 1024) vs the fp32 oracle, and vs the NT = 1 schedule (same per-tile math)."""
    dbg = "persist_min_t=1" + (f",gru_nt={nt}" if nt else "")
    monkeypatch.setenv("DCR_DEBUG", dbg)
    cfg, nat = _model(B, H, 2, seed=7)
    plan = int(nat.backend.ops.gru_persist_ub(H, B))
    assert plan >> 4 == (nt or 2), plan
    ref = ReferenceBackend(nat.store)
    torch.manual_seed(2)
    x = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    y = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    st0 = [(torch.randn(B, H, device="cuda") * 0.5,) for _ in range(2)]
    loss_r, st_r, _ = ref.train_step(x, y, [tuple(s.clone() for s in t) for t in st0])
    g_ref = nat.store.grad.clone()
    nat.store.grad.zero_()
    loss_n, st_n, _ = nat.backend.train_step(x, y, [tuple(s.clone() for s in t) for t in st0])
    torch.cuda.synchronize()
    nat.backend.check_errors()
    g_nt = nat.store.grad.clone()
    assert abs(loss_n.item() - loss_r.item()) < 2e-2 * max(1.0, abs(loss_r.item()))
    for a_r, a_n in zip(st_r, st_n):
        assert rel(a_n[0], a_r[0]) < 3e-2
    check_grads("gru_persist_multi", nat.store, nat.store.grad, g_ref)
    if nt and B < 256:  # NT = 1 fits these grids: same schedule per tile
        monkeypatch.setenv("DCR_DEBUG", "persist_min_t=1,gru_nt=1")
        _, one = _model(B, H, 2, seed=7)
        assert int(one.backend.ops.gru_persist_ub(H, B)) >> 4 == 1
        loss_1, st_1, _ = one.backend.train_step(x, y, [tuple(s.clone() for s in t) for t in st0])
        torch.cuda.synchronize()
        assert abs(loss_1.item() - loss_n.item()) < 1e-4
        assert rel(g_nt, one.store.grad) < 1e-4
