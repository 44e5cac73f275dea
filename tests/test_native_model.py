"""Native (HIP) model step vs the fp32 PyTorch autograd oracle with TF cell semantics.

Covers the fused recurrent kernels (csrc/rnn_step.hip) for every cell type, the fused
softmax-CE (csrc/xent.hip), the layer-0 E·W_x gather fusion and segment-sum backward
(csrc/embed.hip) and the backend's GEMM plumbing.  bf16 MFMA operands => compare with
relative-norm tolerances."""
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


def _oracle_ctx(model):
    """NAS gradients are checked against the oracle on bf16-rounded GEMM operands: the fp32
    oracle differs from ANY bf16-operand computation of NAS by ~8e-2 (its nested gate products
    amplify operand rounding), while the native kernels sit 3e-3 from the rounded-operand oracle
    (test_cell_error_is_bf16_operand_rounding measures both)."""
    import contextlib

    from distributed_char_rnn_amd.models.reference import bf16_operands

    return bf16_operands() if model == "nas" else contextlib.nullcontext()


def _pair(model, B, T, H, L, V=65, seed=0, **kw):
    cfg = ModelConfig(model=model, vocab_size=V, rnn_size=H, num_layers=L, **kw)
    nat = CharRNN(cfg, device="cuda", seed=seed)
    ref = ReferenceBackend(nat.store)  # same flat params, fp32 autograd on the GPU
    return cfg, nat, ref


@pytest.mark.parametrize("model", ["lstm", "gru", "rnn", "nas"])
@pytest.mark.parametrize("B,T,H,L", [(32, 6, 64, 2), (20, 5, 32, 1), (48, 4, 96, 3)])
def test_train_step_matches_reference(model, B, T, H, L):
    torch.manual_seed(0)
    cfg, nat, ref = _pair(model, B, T, H, L)
    x = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    y = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    st0 = [tuple(torch.randn(B, H, device="cuda") * 0.5 for _ in range(cfg.state_arity))
           for _ in range(L)]
    with _oracle_ctx(model):
        loss_r, st_r, _ = ref.train_step(x, y, [tuple(s.clone() for s in t) for t in st0])
    g_ref = nat.store.grad.clone()
    nat.store.grad.zero_()
    loss_n, st_n, _ = nat.backend.train_step(x, y, [tuple(s.clone() for s in t) for t in st0])
    torch.cuda.synchronize()
    assert abs(loss_n.item() - loss_r.item()) < 2e-2 * max(1.0, abs(loss_r.item())), (loss_n, loss_r)
    for (a_r, a_n) in zip(st_r, st_n):
        for s_r, s_n in zip(a_r, a_n):
            assert rel(s_n, s_r) < 3e-2
    check_grads("native_model_nas" if model == "nas" else "native_model", nat.store,
                nat.store.grad, g_ref)
    # TF clip-norm term: per-token sum of squares of the embedding-lookup gradient
    slot_r = nat.store.norm_slot_view(g_ref)
    slot_n = nat.store.norm_slot_view()
    assert slot_r.item() > 0 and rel(slot_n, slot_r) < 6e-2, (slot_n, slot_r)


@pytest.mark.parametrize("model", ["lstm", "gru"])
def test_dropout_path_runs_and_is_finite(model):
    cfg, nat, _ = _pair(model, 32, 4, 64, 2, input_keep_prob=0.8, output_keep_prob=0.7)
    x = torch.randint(0, 65, (32, 4), device="cuda", dtype=torch.int32)
    loss, st, _ = nat.backend.train_step(x, x, nat.zero_state(32))
    assert torch.isfinite(loss)
    assert torch.isfinite(nat.store.grad).all()
    assert nat.store.gview("embedding").abs().sum() > 0


@pytest.mark.parametrize("model", ["lstm", "gru", "rnn", "nas"])
def test_step_logits_matches_reference(model):
    cfg, nat, ref = _pair(model, 4, 1, 64, 2)
    st = nat.zero_state(4)
    x = torch.tensor([[1], [2], [3], [4]], device="cuda", dtype=torch.int32)
    for _ in range(3):
        ln, stn = nat.backend.step_logits(x, st)
        lr, str_ = ref.step_logits(x, st)
        assert rel(ln, lr) < 3e-2
        st = stn


def test_xent_kernel(dcr_ops):
    N, V = 1000, 65
    logits = torch.randn(N, V, device="cuda") * 3
    tgt = torch.randint(0, V, (N,), device="cuda", dtype=torch.int32)
    rl = torch.empty(N, device="cuda")
    dl = torch.empty(N, V, device="cuda", dtype=torch.bfloat16)
    part = torch.empty(dcr_ops.xent_num_partials(N), device="cuda")
    loss = torch.empty(1, device="cuda")
    dcr_ops.xent(logits, tgt, 1.0 / N, rl, dl, part, loss)
    lt = logits.clone().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(lt, tgt.long(), reduction="none")
    ref.mean().backward()
    torch.testing.assert_close(rl, ref.detach(), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(loss[0], ref.mean().detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dl.float(), lt.grad, rtol=1e-2, atol=1e-5)


@pytest.mark.parametrize("V,W,N,ld,dt", [
    (65, 256, 5000, 256, "bf16"), (1, 130, 777, 130, "bf16"), (200, 64, 300, 64, "bf16"),
    (1, 3072, 5000, 3072, "bf16"), (1, 520, 777, 520, "bf16"),
    # one-hot MFMA route (onehot_segsum_kernel): full strips, a ragged strip, strided rows
    (65, 512, 32768, 512, "bf16"), (96, 136, 1000, 136, "bf16"), (65, 2048, 4097, 2056, "bf16"),
    (65, 256, 5000, 256, "fp32")])
def test_segsum_kernel(dcr_ops, V, W, N, ld, dt):
    X = torch.randn(N, ld, device="cuda")
    X = (X.to(torch.bfloat16) if dt == "bf16" else X)[:, :W]
    ids = torch.randint(0, V, (N,), device="cuda", dtype=torch.int32) if V > 1 else None
    out = torch.empty(V, W, device="cuda")
    ws = torch.empty(max(1, dcr_ops.segsum_workspace(N, W, V)), device="cuda")
    dcr_ops.segsum(X, ids, V, out, ws, False)
    ref = torch.zeros(V, W, device="cuda", dtype=torch.float64)
    ref.index_add_(0, (ids if ids is not None else torch.zeros(N, device="cuda", dtype=torch.int32)).long(),
                   X.double())
    torch.testing.assert_close(out.double(), ref, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("N", [4100, 32768])
def test_segsum_atomic_wide_vocab_runs(dcr_ops, N):
    """Wide-vocabulary atomic route (V > 96) with fp32 rows and long runs of equal ids (the
    kernel sums a run in registers and flushes it with one atomic), ragged last chunk."""
    V, W = 8192, 512
    X = torch.randn(N, W, device="cuda")
    ids = torch.randint(0, V, (N,), device="cuda", dtype=torch.int32)
    ids[100:180] = 7        # a run crossing a 32-row chunk boundary
    ids[-5:] = ids[0]
    out = torch.empty(V, W, device="cuda")
    ws = torch.empty(max(1, dcr_ops.segsum_workspace(N, W, V)), device="cuda")
    dcr_ops.segsum(X, ids, V, out, ws, False)
    ref = torch.zeros(V, W, device="cuda", dtype=torch.float64)
    ref.index_add_(0, ids.long(), X.double())
    torch.testing.assert_close(out.double(), ref, rtol=1e-4, atol=1e-4)
    # sorted route: ids sorted + source-row permutation (engine/native/backward.py _embed_grad)
    sid, perm = torch.sort(ids)
    out2 = torch.empty(V, W, device="cuda")
    dcr_ops.segsum(X, sid, V, out2, ws, False, perm.int())
    torch.testing.assert_close(out2.double(), ref, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("dew,rec", [("segsum", "auto"), ("segsum", "single"),
                                     ("fused", "single")])
def test_embedding_table_gradient_routes_agree(dew, rec, monkeypatch):
    """The layer-0 dEW = onehot(ids)ᵀ·dZ0 routes (library one-hot GEMM, one-hot MFMA segment
    sum, LDS partials inside the single-layer BPTT) give the same gradients up to fp32
    summation order."""
    B, T, H = 64, 12, 128
    torch.manual_seed(3)
    x = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    y = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    monkeypatch.setenv("DCR_RECURRENCE", rec)
    grads = []
    for mode in ("gemm", dew):
        monkeypatch.setenv("DCR_DEBUG", f"persist_min_t=1,dew={mode}")
        cfg, nat, _ = _pair("lstm", B, T, H, 2, seed=4)
        nat.backend.train_step(x, y, nat.zero_state(B))
        torch.cuda.synchronize()
        grads.append(nat.store.grad.clone())
    assert rel(grads[1], grads[0]) < 1e-5


@pytest.mark.parametrize("nbt", ["2", "4"])
@pytest.mark.parametrize("model", ["lstm", "gru", "rnn", "nas"])
def test_per_step_batch_tiles_match_reference(model, nbt, monkeypatch):
    """Per-step kernels with several batch tiles per workgroup (weight slice read once per
    NBT x 16 rows; ragged last group) against the fp32 oracle."""
    monkeypatch.setenv("DCR_RECURRENCE", "step")
    monkeypatch.setenv("DCR_DEBUG", f"step_nbt={nbt}")
    B, T, H, L = 56, 5, 64, 2
    torch.manual_seed(2)
    cfg, nat, ref = _pair(model, B, T, H, L)
    x = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    y = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    st0 = [tuple(torch.randn(B, H, device="cuda") * 0.5 for _ in range(cfg.state_arity))
           for _ in range(L)]
    with _oracle_ctx(model):
        loss_r, _, _ = ref.train_step(x, y, [tuple(s.clone() for s in t) for t in st0])
    g_ref = nat.store.grad.clone()
    nat.store.grad.zero_()
    loss_n, _, _ = nat.backend.train_step(x, y, [tuple(s.clone() for s in t) for t in st0])
    torch.cuda.synchronize()
    assert abs(loss_n.item() - loss_r.item()) < 2e-2 * max(1.0, abs(loss_r.item()))
    check_grads("native_model_nas" if model == "nas" else "native_model", nat.store,
                nat.store.grad, g_ref)


# B = 512: the BPTT step product runs as split-K slabs summed by the cell kernel
@pytest.mark.parametrize("B,T,H,L", [(32, 5, 64, 2), (64, 4, 128, 1), (512, 3, 64, 1)])
def test_library_step_lstm_path_matches_reference(B, T, H, L, monkeypatch):
    """DCR_RECURRENCE=library: per-step library GEMM (h·W_h / dZ·W_hᵀ) + epilogue-only cell
    kernels (the H > 1024 LSTM path) against the fp32 oracle, persistent kernels off."""
    monkeypatch.setenv("DCR_RECURRENCE", "library")
    torch.manual_seed(5)
    cfg, nat, ref = _pair("lstm", B, T, H, L)
    assert nat.backend._lib_step("fwd", B) and nat.backend._lib_step("bwd", B)
    # a first step captures the T-step loops as graphs; the checked step replays them
    x0 = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    nat.backend.train_step(x0, x0, nat.zero_state(B))
    x = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    y = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    st0 = [tuple(torch.randn(B, H, device="cuda") * 0.5 for _ in range(2)) for _ in range(L)]
    loss_r, st_r, _ = ref.train_step(x, y, [tuple(s.clone() for s in t) for t in st0])
    g_ref = nat.store.grad.clone()
    nat.store.grad.zero_()
    loss_n, st_n, _ = nat.backend.train_step(x, y, [tuple(s.clone() for s in t) for t in st0])
    torch.cuda.synchronize()
    assert abs(loss_n.item() - loss_r.item()) < 2e-2 * max(1.0, abs(loss_r.item()))
    for (a_r, a_n) in zip(st_r, st_n):
        for s_r, s_n in zip(a_r, a_n):
            assert rel(s_n, s_r) < 3e-2
    check_grads("native_model_lib", nat.store, nat.store.grad, g_ref)


@pytest.mark.parametrize("model", ["nas", "lstm"])
def test_cell_error_is_bf16_operand_rounding(model):
    """Where the native error against the fp32 oracle comes from: the same oracle with every GEMM
    fed bf16-rounded operands (and a bf16 dZ, models/reference.py bf16_operands) -- fp32 math on
    the operands the kernels' MFMAs see -- must sit much closer to the native gradients than the
    fp32 oracle does.  For NAS this is what justifies its looser fp32-oracle tolerance."""
    from oracle import block_err
    from distributed_char_rnn_amd.models.reference import bf16_operands

    B, T, H, L = 48, 4, 96, 3
    torch.manual_seed(0)
    cfg, nat, ref = _pair(model, B, T, H, L)
    x = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    y = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    st0 = [tuple(torch.randn(B, H, device="cuda") * 0.5 for _ in range(cfg.state_arity))
           for _ in range(L)]
    cp = lambda: [tuple(s.clone() for s in t) for t in st0]  # noqa: E731
    ref.train_step(x, y, cp())
    g_f = nat.store.grad.clone()
    with bf16_operands():
        ref.train_step(x, y, cp())
    g_e = nat.store.grad.clone()
    nat.store.grad.zero_()
    nat.backend.train_step(x, y, cp())
    torch.cuda.synchronize()
    g_n = nat.store.grad.clone()
    worst_f = worst_e = 0.0
    for s in nat.store.specs:
        n, f, e = (nat.store.view(s.name, g) for g in (g_n, g_f, g_e))
        ef, ee = max(rel(n, f), block_err(n, f)), max(rel(n, e), block_err(n, e))
        print(f"{model} {s.name}: vs fp32 {ef:.2e}  vs bf16-operand oracle {ee:.2e}")
        worst_f, worst_e = max(worst_f, ef), max(worst_e, ee)
    print(f"{model} worst: vs fp32 {worst_f:.2e}  vs bf16-operand oracle {worst_e:.2e}")
    assert worst_e < 2e-2, worst_e
    if model == "nas":
        assert worst_e < worst_f / 3, (worst_e, worst_f)
