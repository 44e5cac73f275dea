"""CPU tests of the reference (oracle) model: TF cell semantics, parameter layout and
initialisers, gradient correctness (finite differences), TF-Adam + clipping, checkpoints."""
import math

import numpy as np
import pytest
import torch

from distributed_char_rnn_amd.engine.optim import TFAdam, lr_for_epoch
from distributed_char_rnn_amd.models import reference as R
from distributed_char_rnn_amd.models.char_rnn import CharRNN
from distributed_char_rnn_amd.models.params import ModelConfig, ParamStore, glorot_limit
from distributed_char_rnn_amd.utils import checkpoint as ckpt


def test_param_layout_names_and_shapes():
    cfg = ModelConfig(model="lstm", vocab_size=65, rnn_size=512, num_layers=2)
    st = ParamStore(cfg)
    names = st.names()
    assert names[:2] == ["rnnlm/softmax_w", "rnnlm/softmax_b"]
    assert names[-1] == "embedding"
    assert st.view("rnnlm/multi_rnn_cell/cell_0/lstm_cell/kernel").shape == (1024, 2048)
    # parameter count quoted in SURVEY.md §6: 4,265,025 for 2-layer LSTM-512, V=65
    assert sum(s.numel for s in st.specs) == 4265025
    # buckets: layer ranges are contiguous and ordered top layer first
    assert st.layer_range(1)[1] <= st.layer_range(0)[0]
    for s in st.specs:
        assert s.offset % 64 == 0


def test_initialisers():
    cfg = ModelConfig(model="gru", vocab_size=30, rnn_size=16, num_layers=1)
    st = ParamStore(cfg, seed=1)
    assert torch.all(st.view("rnnlm/multi_rnn_cell/cell_0/gru_cell/gates/bias") == 1.0)
    assert torch.all(st.view("rnnlm/multi_rnn_cell/cell_0/gru_cell/candidate/bias") == 0.0)
    w = st.view("embedding")
    assert w.abs().max() <= glorot_limit((30, 16)) + 1e-6
    b = st.view("rnnlm/softmax_b")
    assert b.abs().max() <= math.sqrt(3.0 / 30) + 1e-6 and b.abs().max() > 0


def test_lstm_cell_tf_semantics():
    torch.manual_seed(0)
    H, D = 3, 2
    x, c, h = torch.randn(4, D), torch.randn(4, H), torch.randn(4, H)
    k, b = torch.randn(D + H, 4 * H), torch.randn(4 * H)
    out, (c2, h2) = R.lstm_cell(x, (c, h), k, b)
    z = torch.cat([x, h], 1) @ k + b
    i, j, f, o = z[:, :H], z[:, H:2 * H], z[:, 2 * H:3 * H], z[:, 3 * H:]
    ce = torch.sigmoid(f + 1.0) * c + torch.sigmoid(i) * torch.tanh(j)
    torch.testing.assert_close(c2, ce)
    torch.testing.assert_close(h2, torch.sigmoid(o) * torch.tanh(ce))


def test_gru_reset_before_matmul():
    torch.manual_seed(0)
    H, D = 3, 2
    x, h = torch.randn(2, D), torch.randn(2, H)
    gk, gb, ck, cb = torch.randn(D + H, 2 * H), torch.randn(2 * H), torch.randn(D + H, H), torch.randn(H)
    out, (h2,) = R.gru_cell(x, (h,), gk, gb, ck, cb)
    ru = torch.sigmoid(torch.cat([x, h], 1) @ gk + gb)
    r, u = ru[:, :H], ru[:, H:]
    cc = torch.tanh(torch.cat([x, r * h], 1) @ ck + cb)
    torch.testing.assert_close(h2, u * h + (1 - u) * cc)


@pytest.mark.parametrize("model", ["lstm", "gru", "rnn", "nas"])
def test_reference_gradients_finite_difference(model):
    torch.manual_seed(0)
    cfg = ModelConfig(model=model, vocab_size=7, rnn_size=4, num_layers=2)
    st = ParamStore(cfg, seed=0)
    st.flat.data = st.flat.double()
    st.grad = torch.zeros_like(st.flat)
    be = R.ReferenceBackend(st)
    x = torch.randint(0, 7, (3, 4), dtype=torch.int32)
    y = torch.randint(0, 7, (3, 4), dtype=torch.int32)
    state = R.zero_state(cfg, 3, dtype=torch.float64)
    be.train_step(x, y, state)
    g = st.grad.clone()

    def f():
        p = {n: st.view(n) for n in st.names()}
        lg, _, _ = R.forward(cfg, p, x, state, training=False)
        return R.loss_fn(lg, y)[0].item()

    rng = np.random.default_rng(0)
    for idx in rng.choice(st.numel, 12, replace=False):
        old = st.flat[idx].item()
        st.flat[idx] = old + 1e-6
        fp = f()
        st.flat[idx] = old - 1e-6
        fm = f()
        st.flat[idx] = old
        assert abs((fp - fm) / 2e-6 - g[idx].item()) < 1e-5 * max(1, abs(g[idx].item()))


def test_tf_adam_matches_formula_and_clips():
    cfg = ModelConfig(model="rnn", vocab_size=5, rnn_size=4, num_layers=1, clip_norm="dense")
    st = ParamStore(cfg, seed=0)
    opt = TFAdam(st, clip=0.5)
    p0 = st.flat.clone()
    st.grad.normal_()
    n = st.norm_slot  # parameters end here; the norm slot block is neither measured nor updated
    g = st.grad[:n].clone()
    norm = g.norm().item()
    opt.step(0.01)
    gs = g * (0.5 / max(norm, 0.5))
    m = 0.1 * gs
    v = 0.001 * gs * gs
    lr_t = 0.01 * math.sqrt(1 - 0.999) / (1 - 0.9)
    torch.testing.assert_close(st.flat[:n], p0[:n] - lr_t * m / (v.sqrt() + 1e-8), rtol=1e-5,
                               atol=1e-7)
    assert torch.equal(st.flat[n:], p0[n:])
    assert abs(opt.last_norm.item() - norm) < 1e-4
    assert opt.t == 1
    assert lr_for_epoch(0.002, 0.97, 3) == pytest.approx(0.002 * 0.97 ** 3)


def test_charrnn_cpu_train_step_reduces_loss():
    torch.manual_seed(0)
    cfg = ModelConfig(model="lstm", vocab_size=10, rnn_size=16, num_layers=2)
    m = CharRNN(cfg, device="cpu", seed=0)
    opt = TFAdam(m.store, clip=5.0)
    x = np.tile(np.arange(10, dtype=np.int32), (4, 2))[:, :12]
    y = np.roll(x, -1, axis=1)
    st = m.zero_state(4)
    losses = []
    for _ in range(60):
        loss, st, _ = m.train_step(x, y, m.zero_state(4))
        opt.step(0.01)
        losses.append(loss.item())
    assert losses[-1] < 0.5 * losses[0]


def test_checkpoint_roundtrip_and_max_to_keep(tmp_path):
    saver = ckpt.Saver(max_to_keep=2)
    t = {"a": torch.randn(3, 4), "b/Adam": np.arange(5, dtype=np.float32),
         "global_step": np.array(7, dtype=np.int64)}
    for step in (0, 5, 9):
        saver.save(str(tmp_path), t, step)
    st = ckpt.get_checkpoint_state(str(tmp_path))
    assert st["model_checkpoint_path"].endswith("model.ckpt-9")
    assert len(st["all_model_checkpoint_paths"]) == 2
    assert not (tmp_path / "model.ckpt-0.index").exists()
    assert (tmp_path / "model.ckpt-9.data-00000-of-00001").exists()
    got = ckpt.Saver.restore(ckpt.latest_checkpoint(str(tmp_path)))
    np.testing.assert_array_equal(got["a"], t["a"].numpy())
    assert int(got["global_step"]) == 7
    # corruption is detected
    data = tmp_path / "model.ckpt-9.data-00000-of-00001"
    b = bytearray(data.read_bytes())
    b[-1] ^= 0xFF
    data.write_bytes(bytes(b))
    with pytest.raises(IOError):
        ckpt.Saver.restore(str(tmp_path / "model.ckpt-9"))


def test_adam_slot_checkpoint_roundtrip():
    cfg = ModelConfig(model="lstm", vocab_size=6, rnn_size=4, num_layers=1)
    st = ParamStore(cfg, seed=0)
    opt = TFAdam(st)
    for _ in range(3):
        st.grad.normal_()
        opt.step(1e-3)
    slots = opt.slot_state()
    assert "rnnlm/multi_rnn_cell/cell_0/lstm_cell/kernel/Adam_1" in slots
    st2 = ParamStore(cfg, seed=1)
    opt2 = TFAdam(st2)
    opt2.load_slot_state(slots)
    assert opt2.t == 3
    for s in st.specs:
        torch.testing.assert_close(st2.view(s.name, opt2.m), st.view(s.name, opt.m))
        torch.testing.assert_close(st2.view(s.name, opt2.v), st.view(s.name, opt.v))


def test_tf_adam_grad_scale_equals_averaged_gradient():
    from distributed_char_rnn_amd.engine.optim import TFAdam
    cfg = ModelConfig(model="lstm", vocab_size=11, rnn_size=8, num_layers=1)
    a = CharRNN(cfg, device="cpu", seed=0)
    b = CharRNN(cfg, device="cpu", seed=0)
    g = torch.randn(a.store.numel) * 3.0
    a.store.grad.copy_(g / 4)
    b.store.grad.copy_(g)
    # the norm slot holds a SUM OF SQUARES (TF per-token embedding term): the all-reduced
    # slot of 4 ranks is averaged by 1/4^2, exactly what the folded grad_scale does to it
    slot = a.store.norm_slot
    a.store.grad[slot:] = 0.0
    b.store.grad[slot:] = 0.0
    a.store.grad[slot] = 7.0 / 16
    b.store.grad[slot] = 7.0
    oa, ob = TFAdam(a.store, clip=1.0), TFAdam(b.store, clip=1.0)
    na = oa.step(1e-2)
    nb = ob.step(1e-2, grad_scale=0.25)
    torch.testing.assert_close(nb, na)
    torch.testing.assert_close(b.store.flat, a.store.flat)


def test_bf16_operand_oracle_rounds_gemm_operands_and_dz():
    """models/reference.py bf16_operands: fp32 GEMMs of bf16-rounded operands, a bf16-rounded
    incoming gradient, and the switch restored on exit."""
    from distributed_char_rnn_amd.models import reference as R

    g = torch.Generator().manual_seed(0)
    a = torch.randn(8, 16, generator=g, requires_grad=True)
    b = torch.randn(16, 4, generator=g, requires_grad=True)
    up = torch.randn(8, 4, generator=g)
    with R.bf16_operands():
        out = R._mm(a, b)
        out.backward(up)
    ab, bb, ub = (t.detach().bfloat16().float() for t in (a, b, up))
    assert torch.equal(out, ab @ bb)
    torch.testing.assert_close(a.grad, ub @ bb.t())
    torch.testing.assert_close(b.grad, ab.t() @ ub)
    assert not R._BF16_OPERANDS[0]
    assert torch.equal(R._mm(a, b), a @ b)
