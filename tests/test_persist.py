"""Persistent weights-resident LSTM kernels (csrc/lstm_persist.hip) vs the fp32 autograd oracle
and vs the per-step kernels; also checks that no hand-off ever timed out."""
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


@pytest.fixture(autouse=True, params=["auto", "single"])
def _short_spins(monkeypatch, request):
    """auto: layer pairs on the wavefront kernels; single: every layer on the single-layer
    kernels."""
    monkeypatch.setenv("DCR_SPIN_LIMIT", str(1 << 20))
    monkeypatch.setenv("DCR_DEBUG", "persist_min_t=1")  # short test sequences still qualify
    monkeypatch.setenv("DCR_RECURRENCE", request.param)


def _persist(backend, B):
    return backend._persist_plan(B, True).persist


@pytest.mark.parametrize("mode", ["exclusive", "overlap"])
@pytest.mark.parametrize("B,T,H,L", [(32, 5, 128, 2), (48, 7, 256, 1), (64, 9, 512, 2),
                                     (256, 4, 512, 2), (16, 3, 1024, 1), (128, 3, 1024, 2)])
def test_persist_matches_reference(B, T, H, L, mode, dcr_ops, monkeypatch):
    monkeypatch.setenv("DCR_MODE", mode)
    cfg = ModelConfig(model="lstm", vocab_size=65, rnn_size=H, num_layers=L)
    nat = CharRNN(cfg, device="cuda", seed=3)
    if not _persist(nat.backend, B):
        pytest.skip("grid not co-resident for this shape: per-step path")
    ref = ReferenceBackend(nat.store)
    torch.manual_seed(1)
    x = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    y = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    st0 = [tuple(torch.randn(B, H, device="cuda") * 0.5 for _ in range(2)) for _ in range(L)]
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
    check_grads("persist", nat.store, nat.store.grad, g_ref)


def test_persist_equals_per_step_kernels(monkeypatch):
    """Same bf16 math, different schedule: results agree to accumulation-order noise."""
    B, T, H = 64, 16, 256
    cfg = ModelConfig(model="lstm", vocab_size=65, rnn_size=H, num_layers=2)
    a = CharRNN(cfg, device="cuda", seed=5)
    monkeypatch.setenv("DCR_RECURRENCE", "step")
    b = CharRNN(cfg, device="cuda", seed=5)
    assert a.backend._persist_plan(B, True).persistent
    assert not b.backend._persist_plan(B, True).persistent
    x = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    la, sa, _ = a.backend.train_step(x, x, a.zero_state(B))
    lb, sb, _ = b.backend.train_step(x, x, b.zero_state(B))
    torch.cuda.synchronize()
    a.backend.check_errors()
    assert abs(la.item() - lb.item()) < 1e-3
    assert rel(a.store.grad, b.store.grad) < 1e-2
    for s1, s2 in zip(sa, sb):
        for u, v in zip(s1, s2):
            assert rel(u, v) < 1e-2


def test_persist_repeated_calls_stable():
    """Counters are re-zeroed per launch: many back-to-back launches stay correct."""
    B, T, H = 128, 8, 512
    cfg = ModelConfig(model="lstm", vocab_size=65, rnn_size=H, num_layers=2)
    m = CharRNN(cfg, device="cuda", seed=7)
    x = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    st = m.zero_state(B)
    l0, _, _ = m.backend.train_step(x, x, st)
    g0 = m.store.grad.clone()
    for _ in range(20):
        l1, _, _ = m.backend.train_step(x, x, st)
    torch.cuda.synchronize()
    m.backend.check_errors()
    assert abs(l0.item() - l1.item()) < 1e-5
    assert rel(m.store.grad, g0) < 1e-5


def test_residency_plan_and_refusal(dcr_ops):
    """A grid that cannot be co-resident is planned onto the per-step path, and the op itself
    refuses to launch it (instead of spinning into a timeout)."""
    cus = dcr_ops.num_cus()
    assert cus > 0
    # bench shape: 256 workgroups; the forward and both BPTT variants are co-resident (the
    # exclusive schedule the backend uses by default)
    H, B = 512, 256
    grid = dcr_ops.lstm_persist_grid(H, B)
    assert grid <= cus * dcr_ops.lstm_persist_occupancy(0, H, B, 0, 0)
    assert grid <= cus * dcr_ops.lstm_persist_occupancy(1, H, B, 65, 0)
    assert grid <= cus * dcr_ops.lstm_persist_occupancy(1, H, B, 65, 4)
    # H=1024, B=256: 512 workgroups of a one-per-CU kernel can never all be resident
    H, B, T = 1024, 256, 2
    if dcr_ops.lstm_persist_grid(H, B) <= cus * dcr_ops.lstm_persist_occupancy(0, H, B, 0, 0):
        pytest.skip("this GPU can hold the H=1024 grid")
    cfg = ModelConfig(model="lstm", vocab_size=65, rnn_size=H, num_layers=1)
    m = CharRNN(cfg, device="cuda", seed=1)
    assert not _persist(m.backend, B)
    dev = "cuda"
    WT = torch.zeros(4 * H, H, dtype=torch.bfloat16, device=dev)
    zx = torch.zeros(T, B, 4 * H, device=dev)
    hbuf = torch.zeros(T + 1, B, H, dtype=torch.bfloat16, device=dev)
    cbuf = torch.zeros(T + 1, B, H, device=dev)
    h32 = torch.zeros(B, H, device=dev)
    cnt = torch.zeros((B // 16) * (T + 1) * 4, dtype=torch.int32, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    with pytest.raises(RuntimeError, match="co-resident"):
        ring = torch.zeros(2 * B * H, dtype=torch.bfloat16, device=dev)
        dcr_ops.lstm_persist_fwd(WT, zx, None, hbuf, cbuf, None, h32, cnt, err, 1.0, 1 << 16, ring)
    # the model still trains through the per-step kernels
    x = torch.randint(0, 65, (B, T), device=dev, dtype=torch.int32)
    loss, _, _ = m.backend.train_step(x, x, m.zero_state(B))
    assert torch.isfinite(loss).item()


@pytest.mark.parametrize("B,T,H", [(32, 7, 128), (256, 12, 512), (64, 5, 384)])
def test_two_layer_wavefront_equals_single_layer_kernels(B, T, H, monkeypatch):
    """lstm2_persist.hip (layers 0 and 1 as one wavefront launch) vs two single-layer
    persistent launches: identical bf16 math, so agreement to accumulation-order noise."""
    cfg = ModelConfig(model="lstm", vocab_size=65, rnn_size=H, num_layers=2)
    monkeypatch.setenv("DCR_RECURRENCE", "auto")
    a = CharRNN(cfg, device="cuda", seed=9)
    monkeypatch.setenv("DCR_RECURRENCE", "single")
    b = CharRNN(cfg, device="cuda", seed=9)
    assert a.backend._persist_plan(B, True, T).pair
    assert not b.backend._persist_plan(B, True, T).pair
    x = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    sa, sb = a.zero_state(B), b.zero_state(B)
    for _ in range(2):  # carried state across steps
        la, sa, _ = a.backend.train_step(x, x, sa)
        lb, sb, _ = b.backend.train_step(x, x, sb)
    torch.cuda.synchronize()
    a.backend.check_errors()
    assert abs(la.item() - lb.item()) < 1e-4
    assert rel(a.store.grad, b.store.grad) < 1e-3
    for u, v in zip(sa, sb):
        for p, q in zip(u, v):
            assert rel(p, q) < 1e-3
    ea, _ = a.backend.eval_loss(x, x, a.zero_state(B))
    eb, _ = b.backend.eval_loss(x, x, b.zero_state(B))
    assert abs(ea.item() - eb.item()) < 1e-4


@pytest.mark.parametrize("B,T,H,L", [(32, 6, 128, 2), (256, 10, 512, 2), (64, 5, 384, 4),
                                     (96, 4, 256, 3)])
def test_two_layer_wavefront_bptt_equals_single_layer_kernels(B, T, H, L, monkeypatch):
    """lstm2_bwd_persist_kernel (layers l and l+1 in one reverse wavefront, layer l's dtop
    fused in-kernel) vs single-layer persistent BPTT launches + the dX GEMM."""
    cfg = ModelConfig(model="lstm", vocab_size=65, rnn_size=H, num_layers=L)
    monkeypatch.setenv("DCR_RECURRENCE", "auto")
    a = CharRNN(cfg, device="cuda", seed=5)
    monkeypatch.setenv("DCR_DEBUG", "persist_min_t=1,pair_bwd=0")
    b = CharRNN(cfg, device="cuda", seed=5)
    assert a.backend._persist_plan(B, True, T).pair_bwd
    assert not b.backend._persist_plan(B, True, T).pair_bwd
    torch.manual_seed(2)
    x = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    y = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    sa, sb = a.zero_state(B), b.zero_state(B)
    for _ in range(2):
        la, sa, _ = a.backend.train_step(x, y, sa)
        lb, sb, _ = b.backend.train_step(x, y, sb)
    torch.cuda.synchronize()
    a.backend.check_errors()
    assert abs(la.item() - lb.item()) < 1e-4
    for s in a.store.specs:
        e = rel(a.store.gview(s.name), b.store.gview(s.name))
        assert e < 2e-3, (s.name, e)
