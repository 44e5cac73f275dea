"""Dropout at speed (DropoutWrapper + embedding dropout, model.py:31-34, 58-59).

The native backend draws one bit mask per layer input plus one on the top output per step
(csrc/dropout.hip); the two-layer wavefront kernels apply theirs to MFMA fragments and to the
stashed dtop in-kernel.  The oracle here is the fp32 autograd model run with *the kernel's own
masks* (expanded from the bits), so forward, loss, final state and every gradient must agree to
bf16 noise -- on the pair kernels, the single-layer / per-step kernels and the GRU route."""
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


def expand(bits, scale):
    """[T, B, H/8] uint8 -> [B, T, H] float mask (scaled), batch-major for the oracle."""
    T, B, K8 = bits.shape
    sh = torch.arange(8, device=bits.device, dtype=torch.uint8)
    m = ((bits.unsqueeze(-1) >> sh) & 1).reshape(T, B, K8 * 8).float() * scale
    return m.transpose(0, 1).contiguous()


def _run(model, B, T, H, L, ikp, okp, env=None, monkeypatch=None, key="dropout"):
    for k, v in (env or {}).items():
        monkeypatch.setenv(k, v)
    cfg = ModelConfig(model=model, vocab_size=65, rnn_size=H, num_layers=L,
                      input_keep_prob=ikp, output_keep_prob=okp)
    nat = CharRNN(cfg, device="cuda", seed=3)
    g = torch.Generator().manual_seed(B + T)
    x = torch.randint(0, 65, (B, T), generator=g, dtype=torch.int32).cuda()
    y = torch.randint(0, 65, (B, T), generator=g, dtype=torch.int32).cuda()
    torch.manual_seed(1)
    arity = 2 if model in ("lstm", "nas") else 1
    st0 = [tuple(torch.randn(B, H, device="cuda") * 0.5 for _ in range(arity)) for _ in range(L)]
    loss_n, st_n, _ = nat.backend.train_step(x, y, [tuple(s.clone() for s in t) for t in st0])
    torch.cuda.synchronize()
    nat.backend.check_errors()
    g_nat = nat.store.grad.clone()
    dm = nat.backend.last_dropout_masks
    assert dm is not None
    masks = {"in": [expand(b, dm["sin"]) if b is not None else None for b in dm["inb"]],
             "out": expand(dm["out"], dm["sout"]) if dm["out"] is not None else None}
    ref = ReferenceBackend(nat.store)
    loss_r, st_r, _ = ref.train_step(x, y, [tuple(s.clone() for s in t) for t in st0],
                                     masks=masks)
    assert abs(loss_n.item() - loss_r.item()) < 2e-2 * max(1.0, abs(loss_r.item()))
    for a_r, a_n in zip(st_r, st_n):
        for s_r, s_n in zip(a_r, a_n):
            assert rel(s_n, s_r) < 3e-2
    check_grads(key, nat.store, g_nat, nat.store.grad)
    return nat, dm


@pytest.mark.parametrize("B,T,H,L", [(64, 6, 128, 2), (256, 5, 512, 2), (50, 4, 256, 4),
                                     (512, 3, 512, 2)])
def test_dropout_on_pair_kernels_matches_oracle(B, T, H, L, monkeypatch):
    nat, _ = _run("lstm", B, T, H, L, 0.8, 0.7)
    assert nat.backend._persist_plan(B, True, T).pair


@pytest.mark.parametrize("ikp,okp", [(0.5, 1.0), (1.0, 0.6)])
def test_dropout_single_keep_prob(ikp, okp):
    _run("lstm", 64, 5, 256, 2, ikp, okp)


def test_dropout_per_step_and_single_layer_kernels(monkeypatch):
    _run("lstm", 48, 5, 128, 3, 0.8, 0.7)                                   # pair + single
    _run("lstm", 32, 4, 128, 2, 0.8, 0.7, {"DCR_RECURRENCE": "step"}, monkeypatch)  # per-step


def test_dropout_gru():
    _run("gru", 64, 5, 128, 2, 0.8, 0.7)


def test_dropout_masks_statistics_and_fresh_per_step():
    cfg = ModelConfig(model="lstm", vocab_size=65, rnn_size=512, num_layers=2,
                      input_keep_prob=0.8, output_keep_prob=0.5)
    m = CharRNN(cfg, device="cuda", seed=5)
    B, T = 256, 32
    x = torch.randint(0, 65, (B, T), dtype=torch.int32, device="cuda")
    m.backend.train_step(x, x, m.zero_state(B))
    d1 = m.backend.last_dropout_masks
    frac_in = expand(d1["inb"][1], 1.0).mean().item()
    frac_out = expand(d1["out"], 1.0).mean().item()
    assert abs(frac_in - 0.4) < 0.01 and abs(frac_out - 0.5) < 0.01
    first = d1["inb"][0].clone()
    m.backend.train_step(x, x, m.zero_state(B))
    assert not torch.equal(first, m.backend.last_dropout_masks["inb"][0])


@pytest.mark.parametrize("B,H,L", [(256, 512, 2), (50, 256, 4)])
def test_dropout_library_input_projection_matches_oracle(B, H, L, monkeypatch):
    """DCR_DEBUG=xin=0: the masked embedding rows (and layer 2's masked input) through the library
    zx GEMM instead of the two-layer forward's in-kernel projection (the default, covered by the
    tests above)."""
    nat, _ = _run("lstm", B, 5, H, L, 0.8, 0.7, env={"DCR_DEBUG": "persist_min_t=1,xin=0"},
                  monkeypatch=monkeypatch)
    assert nat.backend._persist_plan(B, True, 5).pair


@pytest.mark.parametrize("B,T", [(256, 24), (256, 130), (200, 24)])
def test_pair_forward_masked_rows_match_mask_pass(B, T, monkeypatch):
    """The G = 1 two-layer dropout forward writes layer l+1's masked input rows itself
    (Lstm2Args.xdst) and the top layer's output-dropout rows (odst): bitwise the rows of the
    separate mask passes (DCR_DEBUG=xdst=0), so the step's gradients match."""
    cfg = ModelConfig(model="lstm", vocab_size=65, rnn_size=512, num_layers=2,
                      input_keep_prob=0.8, output_keep_prob=0.7)
    x = torch.randint(0, 65, (B, T), dtype=torch.int32, device="cuda")
    y = torch.randint(0, 65, (B, T), dtype=torch.int32, device="cuda")
    out = []
    for knob in ("xdst=0", ""):
        monkeypatch.setenv("DCR_DEBUG", knob)
        m = CharRNN(cfg, device="cuda", seed=9)
        assert m.backend._persist_plan(B, True, T).pair_g == 1
        m.backend.train_step(x, y, m.zero_state(B))
        torch.cuda.synchronize()
        m.backend.check_errors()
        bufs = m.backend._bufs[(B, T, True)]
        out.append((bufs["layers"][1].x_drop.clone(), bufs["o_drop"].clone(),
                    m.store.grad.clone()))
    (xa, oa, ga), (xb, ob, gb) = out
    assert torch.equal(xa, xb)
    assert torch.equal(oa, ob)
    assert float((ga - gb).norm() / gb.norm()) < 1e-6


def test_bits_launch_writes_embedding_rows(monkeypatch):
    """Layer 0's masked embedding rows written by the dropout-bits launch itself equal the
    separate embed_dropout launch's (DCR_DEBUG=bits_embed=0), with the same masks."""
    cfg = ModelConfig(model="lstm", vocab_size=65, rnn_size=256, num_layers=2,
                      input_keep_prob=0.8, output_keep_prob=0.7)
    B, T = 64, 12
    x = torch.randint(0, 65, (B, T), dtype=torch.int32, device="cuda")
    out = []
    for knob in ("bits_embed=0", ""):
        monkeypatch.setenv("DCR_DEBUG", knob)
        m = CharRNN(cfg, device="cuda", seed=4)
        m.backend.train_step(x, x, m.zero_state(B))
        torch.cuda.synchronize()
        bufs = m.backend._bufs[(B, T, True)]
        dm = m.backend.last_dropout_masks
        out.append((bufs["layers"][0].x_drop.clone(), dm["inb"][0].clone(), m.store.grad.clone()))
    (xa, ma, ga), (xb, mb, gb) = out
    assert torch.equal(ma, mb)
    assert torch.equal(xa, xb)
    assert float((ga - gb).norm() / gb.norm()) < 1e-6


def _mix64(z):
    import numpy as np
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def test_dropout_bits_match_host_hash(dcr_ops):
    """The mask words against a host (numpy uint64) evaluation of the same counter hash: word i
    of segment m = 8 hashes of (seed ^ mix64(stream_m * C)) + 8 i + q, four 16-bit uniforms
    each against keep * 65536 (csrc/dropout.hip)."""
    import numpy as np
    nseg, nw = 3, 1000
    bits = torch.empty(nseg, nw * 4, dtype=torch.uint8, device="cuda")
    seed, streams, keeps = 12345, [7, 8, 255], [0.8, 0.5, 0.64]
    dcr_ops.dropout_bits_multi(bits, seed, streams, keeps)
    got = bits.view(torch.int32).cpu().numpy().view(np.uint32)
    with np.errstate(over="ignore"):
        for m in range(nseg):
            key = np.uint64(seed) ^ _mix64(np.uint64(streams[m]) * np.uint64(0x632BE59BD9B4E019))
            kt = int(keeps[m] * 65536.0 + 0.5)
            li = np.arange(nw, dtype=np.uint64)
            w = np.zeros(nw, dtype=np.uint64)
            for q in range(8):
                r = _mix64(key + li * np.uint64(8) + np.uint64(q))
                for e in range(4):
                    u = (r >> np.uint64(16 * e)) & np.uint64(0xFFFF)
                    w |= (u < np.uint64(kt)).astype(np.uint64) << np.uint64(4 * q + e)
            assert np.array_equal(got[m], w.astype(np.uint32))
