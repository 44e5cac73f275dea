"""Persistent weights-resident LSTM for H = 2048 at small batch (csrc/lstm_persist_nt.hip):
16-unit workgroups over NT 16-row batch tiles, so BASELINE config 4 (4-layer LSTM-2048) at
B = 64 runs its recurrence on one launch per layer and direction instead of a library GEMM per
step.  Checked against the fp32 autograd oracle (TF cell semantics, model.py:61-73, 91) and
against the library-GEMM step path (DCR_RECURRENCE=library)."""
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


def _batch(B, T, H, L, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randint(0, 65, (B, T), generator=g, dtype=torch.int32).cuda()
    y = torch.randint(0, 65, (B, T), generator=g, dtype=torch.int32).cuda()
    st0 = [tuple(torch.randn(B, H, generator=g).cuda() * 0.5 for _ in range(2)) for _ in range(L)]
    return x, y, st0


@pytest.mark.parametrize("B,T,L,dbg", [(64, 6, 2, "nt_bwd=0"), (20, 5, 1, "nt_bwd=0"),
                                       (64, 6, 2, "nt_bwd=1"), (20, 5, 1, "nt_bwd=1"),
                                       (7, 4, 1, "nt_bwd=1"), (64, 6, 2, "lib"),
                                       (96, 4, 2, "lib,bigstep=2"),
                                       # NT = 4 batch tiles per workgroup (B = 65-128); 96:
                                       # the second batch group holds two tiles, 100: ragged rows
                                       (128, 5, 2, "nt_bwd=1"), (96, 4, 2, "nt_bwd=1"),
                                       (100, 4, 1, "nt_bwd=1")])
def test_nt_kernels_match_oracle(B, T, L, dbg, dcr_ops, monkeypatch):
    """Default: both directions persistent; nt_bwd=0: persistent forward, library BPTT steps;
    lib: the per-step library / fused step kernels (the upper layer's input bias added by
    their cell epilogues)."""
    lib = dbg.startswith("lib")
    monkeypatch.setenv("DCR_DEBUG", "persist_min_t=100000" + dbg[3:] if lib
                       else f"persist_min_t=1,{dbg}")
    H = 2048
    if not lib:
        assert int(dcr_ops.lstm_persist_nt_tiles(H, B)) in (1, 2, 4)
    cfg = ModelConfig(model="lstm", vocab_size=65, rnn_size=H, num_layers=L)
    nat = CharRNN(cfg, device="cuda", seed=5)
    # non-zero biases (TF initialises them to zero): the upper layers' input bias is added in
    # the persistent forward's epilogue, not by the input GEMM
    gb = torch.Generator().manual_seed(7)
    for sp in nat.store.specs:
        if sp.name.endswith("bias"):
            nat.store.view(sp.name).copy_(torch.randn(sp.shape, generator=gb) * 0.3)
    nat.params_changed()
    P = nat.backend._persist_plan(B, True, T)
    assert not P.pair
    assert P.persist == (not lib) and (lib or P.persist_bwd == (dbg == "nt_bwd=1"))
    x, y, st0 = _batch(B, T, H, L, B)
    ref = ReferenceBackend(nat.store)
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
    check_grads("persist_nt", nat.store, nat.store.grad, g_ref)


def test_nt_kernels_match_library_path(monkeypatch):
    """A 2-layer LSTM-2048 step at B = 64, T = 32 (NT = 2, 256 workgroups): the persistent
    kernels vs the library-GEMM + epilogue per-step path; same loss, gradients and state
    within bf16 noise."""
    B, T, H, L = 64, 32, 2048, 2
    cfg = ModelConfig(model="lstm", vocab_size=65, rnn_size=H, num_layers=L)
    x, y, st0 = _batch(B, T, H, L, 11)
    res = []
    for rec in ("auto", "library"):
        monkeypatch.setenv("DCR_RECURRENCE", rec)
        m = CharRNN(cfg, device="cuda:0", seed=0)
        assert m.backend._persist_plan(B, True, T).persist == (rec == "auto")
        loss, st, _ = m.train_step(x, y, [tuple(s.clone() for s in t) for t in st0])
        torch.cuda.synchronize()
        m.backend.check_errors()
        res.append((loss.item(), m.store.grad.clone(), st))
    (l1, g1, s1), (l0, g0, s0) = res
    assert abs(l1 - l0) < 1e-3
    assert rel(g1, g0) < 2e-2
    for a1, a0 in zip(s1, s0):
        for t1, t0 in zip(a1, a0):
            assert rel(t1, t0) < 1e-2


def test_nt_spin_timeout_drains_and_guards(monkeypatch):
    """A forced hand-off timeout (DCR_SPIN_LIMIT=1) in the H = 2048 persistent kernels: every
    workgroup still finishes (bounded polls, the grid drains), the error word is set, the
    guarded optimizer leaves the weights unchanged and check_errors raises."""
    from distributed_char_rnn_amd.engine.optim import TFAdam

    monkeypatch.setenv("DCR_SPIN_LIMIT", "1")
    B, T, H = 64, 32, 2048
    cfg = ModelConfig(model="lstm", vocab_size=65, rnn_size=H, num_layers=1)
    m = CharRNN(cfg, device="cuda", seed=2)
    assert m.backend._persist_plan(B, True, T).persist
    opt = TFAdam(m.store, clip=5.0, guard=m.error_word())
    x, y, _ = _batch(B, T, H, 1, 3)
    p0 = m.store.flat.clone()
    m.train_step(x, y, m.zero_state(B))
    opt.step(2e-3)
    torch.cuda.synchronize()
    assert int(m.backend.err.item()) != 0, "the forced timeout did not trigger"
    assert torch.equal(m.store.flat, p0)
    with pytest.raises(RuntimeError, match="timed out"):
        m.check_errors()


@pytest.mark.parametrize("B", [128, 100])
def test_nt4_dma_forward_bitwise_equals_register_form(B, monkeypatch):
    """The NT = 4 forward's h tiles by LDS-DMA (default) vs the register double buffer
    (DCR_DEBUG=nt_dma=0) over T = 48 steps: the same MFMA and partial-sum order, so loss, state
    and gradients must be bitwise equal -- a stale or misordered hand-off read in either form
    would change them (B = 100: a ragged second batch group)."""
    T, H, L = 48, 2048, 1
    cfg = ModelConfig(model="lstm", vocab_size=65, rnn_size=H, num_layers=L)
    x, y, st0 = _batch(B, T, H, L, 21)
    res = []
    for dma in ("1", "0"):
        monkeypatch.setenv("DCR_DEBUG", f"persist_min_t=1,nt_dma={dma}")
        m = CharRNN(cfg, device="cuda:0", seed=3)
        assert m.backend._persist_plan(B, True, T).persist
        loss, st, _ = m.train_step(x, y, [tuple(s.clone() for s in t) for t in st0])
        torch.cuda.synchronize()
        m.backend.check_errors()
        res.append((loss.item(), m.store.grad.clone(), [s.clone() for a in st for s in a]))
    (l1, g1, s1), (l0, g0, s0) = res
    assert l1 == l0
    assert torch.equal(g1, g0)
    for a, b in zip(s1, s0):
        assert torch.equal(a, b)
