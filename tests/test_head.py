"""Fused softmax head (csrc/head.hip) vs a plain PyTorch fp32 reference of the same ops:
logits = O·Ws + b, CE summed / N, dlogits = (softmax - onehot)/N, d softmax_b, dtop = dlog·Wsᵀ."""
import pytest
import torch
from oracle import check_grads

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def _pads(ops, V, H, Ws):
    VP, VK = ops.head_pads(V)
    WsT = torch.zeros(VP, H, dtype=torch.bfloat16, device="cuda")
    WsT[:V] = Ws.t().to(torch.bfloat16)
    Wsk = torch.zeros(H, VK, dtype=torch.bfloat16, device="cuda")
    Wsk[:, :V] = Ws.to(torch.bfloat16)
    return WsT, Wsk


@pytest.mark.parametrize("N,H,V", [(32768, 512, 65), (1000, 64, 1), (517, 128, 16),
                                   (777, 96, 100), (300, 256, 256), (64, 32, 33)])
def test_head_train_matches_fp32(N, H, V, dcr_ops):
    torch.manual_seed(0)
    O = (torch.randn(N, H, device="cuda") * 0.5).to(torch.bfloat16)
    Ws = torch.randn(H, V, device="cuda") * (1.0 / H ** 0.5)
    b = torch.randn(V, device="cuda") * 0.1
    y = torch.randint(0, V, (N,), device="cuda", dtype=torch.int32)
    WsT, Wsk = _pads(dcr_ops, V, H, Ws)
    logits = torch.empty(N, V, device="cuda")
    row_loss = torch.empty(N, device="cuda")
    dlog = torch.empty(N, V, dtype=torch.bfloat16, device="cuda")
    dtop = torch.empty(N, H, device="cuda")
    db = torch.empty(V, device="cuda")
    part = torch.empty(dcr_ops.head_workspace(N, V), device="cuda")
    loss = torch.empty(1, device="cuda")
    dcr_ops.head(O, WsT, Wsk, b, y, 1.0 / N, logits, row_loss, dlog, dtop, db, part, loss)
    torch.cuda.synchronize()
    # fp32 reference on the same bf16-rounded operands
    Of, Wf = O.float(), Ws.to(torch.bfloat16).float()
    lg = Of @ Wf + b
    lse = torch.logsumexp(lg, 1)
    rl = lse - lg.gather(1, y.long()[:, None])[:, 0]
    p = torch.softmax(lg, 1)
    d = p.clone()
    d[torch.arange(N), y.long()] -= 1.0
    d /= N
    assert rel(logits, lg) < 2e-3
    assert rel(row_loss, rl) < 2e-3
    assert abs(loss.item() - rl.mean().item()) < 2e-3 * max(1.0, abs(rl.mean().item()))
    assert rel(dlog.float(), d) < 1e-2
    assert rel(db, d.sum(0)) < 2e-2
    assert rel(dtop, dlog.float() @ Wf.t()) < 1e-2


def test_head_eval_and_logits_only(dcr_ops):
    N, H, V = 2000, 128, 65
    torch.manual_seed(1)
    O = torch.randn(N, H, device="cuda").to(torch.bfloat16)
    Ws = torch.randn(H, V, device="cuda") * 0.1
    b = torch.randn(V, device="cuda") * 0.1
    y = torch.randint(0, V, (N,), device="cuda", dtype=torch.int32)
    WsT, _ = _pads(dcr_ops, V, H, Ws)
    part = torch.empty(dcr_ops.head_workspace(N, V), device="cuda")
    loss = torch.empty(1, device="cuda")
    dcr_ops.head(O, WsT, None, b, y, 1.0, None, None, None, None, None, part, loss)
    lg = O.float() @ Ws.to(torch.bfloat16).float() + b
    ref = torch.nn.functional.cross_entropy(lg, y.long())
    assert abs(loss.item() - ref.item()) < 2e-3
    logits = torch.empty(N, V, device="cuda")
    dcr_ops.head(O, WsT, None, b, None, 1.0, logits, None, None, None, None, part, None)
    assert rel(logits, lg) < 2e-3


def test_model_fused_head_equals_library_head(monkeypatch):
    """Whole training step: fused head vs the library GEMM + xent path."""
    from distributed_char_rnn_amd.models.char_rnn import CharRNN
    from distributed_char_rnn_amd.models.params import ModelConfig

    B, T = 64, 16
    cfg = ModelConfig(model="lstm", vocab_size=65, rnn_size=256, num_layers=2)
    a = CharRNN(cfg, device="cuda", seed=11)
    monkeypatch.setenv("DCR_DEBUG", "fused_head=0")
    c = CharRNN(cfg, device="cuda", seed=11)
    assert a.backend.fused_head and not c.backend.fused_head
    x = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    y = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    la, _, ea = a.backend.train_step(x, y, a.zero_state(B), want_extras=True)
    lc, _, ec = c.backend.train_step(x, y, c.zero_state(B), want_extras=True)
    torch.cuda.synchronize()
    assert abs(la.item() - lc.item()) < 1e-3
    assert rel(ea["logits"], ec["logits"]) < 1e-3
    assert rel(a.store.grad, c.store.grad) < 1e-2
    for name in ("rnnlm/softmax_b", "rnnlm/softmax_w"):
        assert rel(a.store.gview(name), c.store.gview(name)) < 1e-2
    ev_a, _ = a.backend.eval_loss(x, y, a.zero_state(B))
    ev_c, _ = c.backend.eval_loss(x, y, c.zero_state(B))
    assert abs(ev_a.item() - ev_c.item()) < 1e-3


@pytest.mark.parametrize("N,V", [(1000, 8192), (333, 256), (70, 1028), (4100, 12288)])
def test_xent_wide_matches_torch(N, V, dcr_ops):
    torch.manual_seed(3)
    logits = torch.randn(N, V, device="cuda") * 4
    y = torch.randint(0, V, (N,), device="cuda", dtype=torch.int32)
    rl = torch.empty(N, device="cuda")
    dl = torch.empty(N, V, dtype=torch.bfloat16, device="cuda")
    colpart = torch.empty(dcr_ops.xent_wide_waves(N) * V, device="cuda")
    db = torch.empty(V, device="cuda")
    part = torch.empty(dcr_ops.xent_num_partials(N), device="cuda")
    loss = torch.empty(1, device="cuda")
    bias = torch.randn(V, device="cuda")
    dcr_ops.xent_wide(logits, bias, y, 1.0 / N, rl, dl, colpart, db, part, loss)
    lt = (logits + bias).clone().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(lt, y.long(), reduction="none")
    ref.mean().backward()
    torch.testing.assert_close(rl, ref.detach(), rtol=1e-5, atol=1e-4)
    assert abs(loss.item() - ref.mean().item()) < 1e-4
    assert rel(dl.float(), lt.grad) < 1e-2
    assert rel(db, dl.float().sum(0)) < 1e-5   # exactly the bf16 dlogits that the GEMMs see


def test_model_wide_vocab_matches_reference():
    """V=300: library logits GEMM + xent_wide + dense layer-0 embedding gradient route."""
    from distributed_char_rnn_amd.models.char_rnn import CharRNN
    from distributed_char_rnn_amd.models.params import ModelConfig
    from distributed_char_rnn_amd.models.reference import ReferenceBackend

    B, T, H, V = 32, 6, 128, 300
    cfg = ModelConfig(model="lstm", vocab_size=V, rnn_size=H, num_layers=2)
    nat = CharRNN(cfg, device="cuda", seed=4)
    assert not nat.backend.fused_head
    ref = ReferenceBackend(nat.store)
    x = torch.randint(0, V, (B, T), device="cuda", dtype=torch.int32)
    y = torch.randint(0, V, (B, T), device="cuda", dtype=torch.int32)
    st0 = nat.zero_state(B)
    loss_r, _, _ = ref.train_step(x, y, st0)
    g_ref = nat.store.grad.clone()
    nat.store.grad.zero_()
    loss_n, _, _ = nat.backend.train_step(x, y, nat.zero_state(B))
    torch.cuda.synchronize()
    assert abs(loss_n.item() - loss_r.item()) < 2e-2 * max(1.0, abs(loss_r.item()))
    check_grads("head", nat.store, nat.store.grad, g_ref)
