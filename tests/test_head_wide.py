"""Fused wide-vocabulary head (csrc/head_wide.hip) against the fp32 PyTorch oracle: logits ->
sequence loss (model.py:76-85) -> bf16 dlogits and d softmax_b in one launch, and the training
step that uses it at the 8k-token config's vocabulary (V = 8192) against the reference backend."""
import pytest
import torch
from oracle import check_grads

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("N,V", [(1000, 8192), (129, 256), (4100, 1024), (64, 64)])
def test_head_wide_matches_torch(N, V, dcr_ops):
    H = 512
    assert dcr_ops.head_wide_supported(V, H)
    g = torch.Generator(device="cuda").manual_seed(N + V)
    O = (torch.randn(N, H, device="cuda", generator=g) * 0.5).bfloat16()
    Ws = (torch.randn(H, V, device="cuda", generator=g) * 0.1)
    WsT = Ws.t().contiguous().bfloat16()
    bias = torch.randn(V, device="cuda", generator=g)
    y = torch.randint(0, V, (N,), device="cuda", dtype=torch.int32, generator=g)
    nb = dcr_ops.head_wide_blocks(N)
    rl = torch.empty(N, device="cuda")
    dl = torch.empty(N, V, dtype=torch.bfloat16, device="cuda")
    lg = torch.empty(N, V, device="cuda")
    colpart = torch.empty(dcr_ops.head_wide_colpart_rows(N) * V, device="cuda")
    db = torch.empty(V, device="cuda")
    part = torch.empty(dcr_ops.head_wide_workspace(N), device="cuda")
    loss = torch.empty(1, device="cuda")
    dcr_ops.head_wide(O, WsT, bias, y, 1.0 / N, rl, dl, lg, colpart, db, part, loss)
    torch.cuda.synchronize()
    lt = (O.float() @ WsT.float().t() + bias).requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(lt, y.long(), reduction="none")
    ref.mean().backward()
    assert rel(lg, lt.detach()) < 1e-5
    torch.testing.assert_close(rl, ref.detach(), rtol=1e-4, atol=1e-3)
    assert abs(loss.item() - ref.mean().item()) < 1e-4 * max(1.0, ref.mean().item())
    assert rel(dl.float(), lt.grad) < 1e-2
    assert rel(db, dl.float().sum(0)) < 1e-5   # exactly the bf16 dlogits the GEMMs see
    # eval form: loss only, nothing else written
    loss2 = torch.empty(1, device="cuda")
    dcr_ops.head_wide(O, WsT, bias, y, 1.0, None, None, None, None, None, part, loss2)
    assert abs(loss2.item() - loss.item()) < 1e-5 * max(1.0, loss.item())


@pytest.mark.parametrize("chunk", [1, 3])
def test_head_wide_chunked_identical(chunk, dcr_ops, monkeypatch):
    """Token counts whose [N, V] outputs pass the kernel's 32-bit buffer offsets run as chunks
    of whole 256-token blocks (launch_head_wide).  Forced small chunks (DCR_DEBUG hw_chunk)
    must give bitwise the same loss, row losses, dlogits, logits and d softmax_b as one launch."""
    H, V, N = 512, 1024, 256 * 7 + 77
    g = torch.Generator(device="cuda").manual_seed(7)
    O = (torch.randn(N, H, device="cuda", generator=g) * 0.5).bfloat16()
    WsT = (torch.randn(V, H, device="cuda", generator=g) * 0.1).bfloat16()
    bias = torch.randn(V, device="cuda", generator=g)
    y = torch.randint(0, V, (N,), device="cuda", dtype=torch.int32, generator=g)

    def run():
        rl = torch.empty(N, device="cuda")
        dl = torch.empty(N, V, dtype=torch.bfloat16, device="cuda")
        lg = torch.empty(N, V, device="cuda")
        colpart = torch.empty(dcr_ops.head_wide_colpart_rows(N) * V, device="cuda")
        db = torch.empty(V, device="cuda")
        part = torch.empty(dcr_ops.head_wide_workspace(N), device="cuda")
        loss = torch.empty(1, device="cuda")
        dcr_ops.head_wide(O, WsT, bias, y, 1.0 / N, rl, dl, lg, colpart, db, part, loss)
        torch.cuda.synchronize()
        return rl, dl, lg, db, loss

    one = run()
    monkeypatch.setenv("DCR_DEBUG", f"hw_chunk={chunk}")
    chunked = run()
    for a, b in zip(one, chunked):
        assert torch.equal(a, b)


def test_model_wide_head_matches_reference_v8192():
    """The 8k-token config's head shape (V = 8192, H = 512) through the training step: loss and
    every gradient against the fp32 autograd oracle, and against the library-logits route."""
    import os

    from distributed_char_rnn_amd.models.char_rnn import CharRNN
    from distributed_char_rnn_amd.models.params import ModelConfig
    from distributed_char_rnn_amd.models.reference import ReferenceBackend

    B, T, H, V = 32, 10, 512, 8192
    cfg = ModelConfig(model="lstm", vocab_size=V, rnn_size=H, num_layers=2)
    nat = CharRNN(cfg, device="cuda", seed=4)
    assert nat.backend.wide_head and not nat.backend.fused_head
    ref = ReferenceBackend(nat.store)
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randint(0, V, (B, T), device="cuda", dtype=torch.int32, generator=g)
    y = torch.randint(0, V, (B, T), device="cuda", dtype=torch.int32, generator=g)
    loss_r, _, _ = ref.train_step(x, y, nat.zero_state(B))
    g_ref = nat.store.grad.clone()
    nat.store.grad.zero_()
    loss_n, _, ex = nat.backend.train_step(x, y, nat.zero_state(B), want_extras=True)
    torch.cuda.synchronize()
    assert abs(loss_n.item() - loss_r.item()) < 1e-2 * max(1.0, abs(loss_r.item()))
    check_grads("head_wide", nat.store, nat.store.grad, g_ref)
    g_wide = nat.store.grad.clone()
    ev = nat.backend.eval_loss(x, y, nat.zero_state(B))[0]
    assert abs(ev.item() - loss_n.item()) < 1e-3
    # the library-logits route (DCR_DEBUG wide_head=0): same loss, same gradients
    os.environ["DCR_DEBUG"] = "wide_head=0"
    try:
        lib = CharRNN(cfg, device="cuda", seed=4)
    finally:
        del os.environ["DCR_DEBUG"]
    assert not lib.backend.wide_head
    loss_l, _, ex_l = lib.backend.train_step(x, y, lib.zero_state(B), want_extras=True)
    torch.cuda.synchronize()
    assert abs(loss_l.item() - loss_n.item()) < 2e-3
    assert rel(ex["logits"], ex_l["logits"]) < 1e-3
    assert rel(g_wide, lib.store.grad) < 2e-2


@pytest.mark.parametrize("M,N,K,lda", [(2048, 512, 8192, 8192), (1024, 512, 1024, 1032),
                                       (4096, 256, 256, 256)])
def test_gemm_nt_matches_torch(M, N, K, lda, dcr_ops):
    """gemm_nt (csrc/tokennorm.hip's pipeline storing its products): C = A · Bᵀ with both bf16
    operands K-contiguous -- config 5's dtop = dlogits · softmax_wᵀ -- against fp32 torch on the
    same bf16 operands (a row stride beyond K included)."""
    assert dcr_ops.gemm_nt_supported(M, N, K)
    g = torch.Generator(device="cuda").manual_seed(M + K)
    A = torch.randn(M, lda, device="cuda", generator=g).bfloat16()[:, :K]
    B = torch.randn(N, K, device="cuda", generator=g).bfloat16()
    C = torch.full((M, N), float("nan"), device="cuda")
    dcr_ops.gemm_nt(A, B, C)
    torch.cuda.synchronize()
    ref = A.float() @ B.float().t()
    assert rel(C, ref) < 1e-5
    assert not dcr_ops.gemm_nt_supported(M + 16, N, K)


def test_model_wide_head_dtop_nt_matches_library():
    """The wide head's dtop through gemm_nt (N = 1024 tokens tile it) against the library GEMM
    (DCR_DEBUG dtop_nt=0): same loss, gradients equal up to fp32 summation order."""
    import os

    from distributed_char_rnn_amd.models.char_rnn import CharRNN
    from distributed_char_rnn_amd.models.params import ModelConfig

    B, T, H, V = 64, 16, 512, 8192
    cfg = ModelConfig(model="lstm", vocab_size=V, rnn_size=H, num_layers=2)
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randint(0, V, (B, T), device="cuda", dtype=torch.int32, generator=g)
    y = torch.randint(0, V, (B, T), device="cuda", dtype=torch.int32, generator=g)
    res = []
    for dbg in (None, "dtop_nt=0"):
        if dbg:
            os.environ["DCR_DEBUG"] = dbg
        try:
            m = CharRNN(cfg, device="cuda", seed=5)
        finally:
            os.environ.pop("DCR_DEBUG", None)
        assert m.backend.wide_head
        loss, _, _ = m.backend.train_step(x, y, m.zero_state(B))
        torch.cuda.synchronize()
        res.append((loss.item(), m.store.grad.clone()))
    assert abs(res[0][0] - res[1][0]) < 1e-6
    assert rel(res[0][1], res[1][1]) < 1e-4


def test_head_wide_train_flags_kernel_identical(dcr_ops, monkeypatch):
    """The training step's flag combination (softmax_b, dlogits, colpart, no logits) runs the
    compile-time-flag kernels (constant counted waits, every wave DMAs the bias row); DCR_DEBUG
    hw_fl=0 forces the generic ones: bitwise the same outputs."""
    H, V, N = 512, 8192, 2048 + 77
    g = torch.Generator(device="cuda").manual_seed(11)
    O = (torch.randn(N, H, device="cuda", generator=g) * 0.5).bfloat16()
    WsT = (torch.randn(V, H, device="cuda", generator=g) * 0.1).bfloat16()
    bias = torch.randn(V, device="cuda", generator=g)
    y = torch.randint(0, V, (N,), device="cuda", dtype=torch.int32, generator=g)

    def run():
        rl = torch.empty(N, device="cuda")
        dl = torch.empty(N, V, dtype=torch.bfloat16, device="cuda")
        colpart = torch.empty(dcr_ops.head_wide_colpart_rows(N) * V, device="cuda")
        db = torch.empty(V, device="cuda")
        part = torch.empty(dcr_ops.head_wide_workspace(N), device="cuda")
        loss = torch.empty(1, device="cuda")
        dcr_ops.head_wide(O, WsT, bias, y, 1.0 / N, rl, dl, None, colpart, db, part, loss)
        torch.cuda.synchronize()
        return rl, dl, db, loss

    fast = run()
    monkeypatch.setenv("DCR_DEBUG", "hw_fl=0")
    generic = run()
    for a, b in zip(fast, generic):
        assert torch.equal(a, b)
