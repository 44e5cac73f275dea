"""rnn_size not a multiple of the kernels' tiles (the reference accepts any size,
model.py:30): the native backend runs a zero-padded model (engine/native/padded.py).  CPU: the
index map places every real parameter element at its padded position; GPU: the padded run on
the hand-written kernels matches the fp32 oracle of the unpadded model."""
import pytest
import torch

from distributed_char_rnn_amd.engine.native.padded import _index_map, _real_offsets, padded_size
from distributed_char_rnn_amd.models.params import ModelConfig, ParamStore, cell_specs
from oracle import check_grads


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("model", ["lstm", "gru", "rnn"])
def test_index_map_places_every_block(model):
    cfg = ModelConfig(model=model, vocab_size=11, rnn_size=5, num_layers=2)
    st = ParamStore(cfg, "cpu", seed=1)
    Hp = padded_size(5)
    assert Hp == 128
    from dataclasses import replace

    ps = ParamStore(replace(cfg, rnn_size=Hp), "cpu", seed=None)
    ps.flat.zero_()
    ps.flat.index_copy_(0, _index_map(st, ps), st.flat.index_select(0, _real_offsets(st)))
    H = 5
    assert torch.equal(ps.view("embedding")[:, :H], st.view("embedding"))
    assert ps.view("embedding")[:, H:].abs().sum() == 0
    assert torch.equal(ps.view("rnnlm/softmax_w")[:H], st.view("rnnlm/softmax_w"))
    assert torch.equal(ps.view("rnnlm/softmax_b"), st.view("rnnlm/softmax_b"))
    for layer in range(2):
        for sp in cell_specs(cfg, layer):
            real, pad = st.view(sp.name), ps.view(sp.name)
            if real.dim() == 1:
                k = real.shape[0] // H
                for g in range(k):
                    assert torch.equal(pad[g * Hp: g * Hp + H], real[g * H:(g + 1) * H])
                continue
            kr, kc = real.shape[0] // H, real.shape[1] // H
            for a in range(kr):
                for b in range(kc):
                    assert torch.equal(pad[a * Hp: a * Hp + H, b * Hp: b * Hp + H],
                                       real[a * H:(a + 1) * H, b * H:(b + 1) * H]), (sp.name, a, b)
    # every padding position stays zero
    assert int((ps.flat != 0).sum()) == int((st.flat != 0).sum())


@pytest.mark.gpu
@pytest.mark.parametrize("model,H,B,T,L", [("lstm", 100, 50, 12, 2), ("lstm", 200, 64, 9, 3),
                                           ("gru", 100, 48, 10, 2), ("rnn", 50, 32, 8, 2)])
def test_padded_native_matches_oracle(model, H, B, T, L, monkeypatch):
    from distributed_char_rnn_amd.models.char_rnn import CharRNN
    from distributed_char_rnn_amd.models.reference import ReferenceBackend

    monkeypatch.setenv("DCR_DEBUG", "persist_min_t=1")
    cfg = ModelConfig(model=model, vocab_size=65, rnn_size=H, num_layers=L)
    nat = CharRNN(cfg, device="cuda", seed=6)
    assert type(nat.backend).__name__ == "PaddedNativeBackend"
    if model == "lstm":
        assert nat.backend._persist_plan(B, True, T).persistent
    ref = ReferenceBackend(nat.store)
    g = torch.Generator().manual_seed(H)
    x = torch.randint(0, 65, (B, T), generator=g, dtype=torch.int32).cuda()
    y = torch.randint(0, 65, (B, T), generator=g, dtype=torch.int32).cuda()
    torch.manual_seed(1)
    st0 = [tuple(torch.randn(B, H, device="cuda") * 0.5 for _ in range(cfg.state_arity))
           for _ in range(L)]
    loss_r, st_r, _ = ref.train_step(x, y, [tuple(s.clone() for s in t) for t in st0])
    g_ref = nat.store.grad.clone()
    nat.store.grad.zero_()
    loss_n, st_n, _ = nat.train_step(x, y, [tuple(s.clone() for s in t) for t in st0])
    torch.cuda.synchronize()
    nat.check_errors()
    assert abs(loss_n.item() - loss_r.item()) < 2e-2 * max(1.0, abs(loss_r.item()))
    for a_r, a_n in zip(st_r, st_n):
        for s_r, s_n in zip(a_r, a_n):
            assert s_n.shape == s_r.shape
            assert rel(s_n, s_r) < 3e-2
    check_grads("padded", nat.store, nat.store.grad, g_ref)
    lg, _ = nat.step_logits(x[:, :1], [tuple(s.clone() for s in t) for t in st0])
    lr, _ = ref.step_logits(x[:, :1], [tuple(s.clone() for s in t) for t in st0])
    assert rel(lg, lr) < 3e-2
