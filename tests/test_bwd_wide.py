"""The 32-unit x 16-row two-layer BPTT (csrc/lstm2_bwd_wide.hip) against the 16-unit x 32-row
kernel it replaces at G = 1 (csrc/lstm2_persist.hip, ``DCR_DEBUG=wide=0``) and the fp32 oracle.

Both kernels split K = 4H over the same wave quarters in the same k order and sum the four
partials in the same order, so every dZ -- hence every weight gradient, the TBPTT state and the
loss -- is bitwise identical; only the in-kernel bias-gradient partials are summed in another
order (rows per tick, then time, instead of time per lane, then rows)."""
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


def _run(cfg, B, T, wide, monkeypatch, steps=2, pf=None, rs=False):
    monkeypatch.setenv("DCR_SPIN_LIMIT", str(1 << 20))
    monkeypatch.setenv("DCR_DEBUG", "persist_min_t=1" + ("" if wide else ",wide=0") +
                       (f",wide_pf={pf}" if pf is not None else "") + (",bwd_rs=1" if rs else ""))
    m = CharRNN(cfg, device="cuda", seed=21)
    plan = m.backend._persist_plan(B, True, T)
    assert plan.pair_bwd and plan.pair_g == 1, plan
    g = torch.Generator().manual_seed(B + T)
    st = m.zero_state(B)
    for _ in range(steps):
        x = torch.randint(0, cfg.vocab_size, (B, T), generator=g, dtype=torch.int32).cuda()
        y = torch.randint(0, cfg.vocab_size, (B, T), generator=g, dtype=torch.int32).cuda()
        loss, st, _ = m.backend.train_step(x, y, st)
    torch.cuda.synchronize()
    m.backend.check_errors()
    return m, loss.item(), [s.clone() for t in st for s in t]


@pytest.mark.parametrize("pf", [None, 0, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("B,T,H,drop", [(256, 8, 512, False), (50, 7, 128, False),
                                        (37, 6, 512, False), (100, 5, 256, True),
                                        (256, 6, 512, True)])
def test_wide_bptt_equals_narrow(B, T, H, drop, pf, monkeypatch, dcr_ops):
    """Every operand-prefetch mode of the wide kernel (``wide_pf``, None = the default)."""
    assert dcr_ops.lstm2_bwd_wide_ok(H, B)
    kp = 0.8 if drop else 1.0
    cfg = ModelConfig(model="lstm", vocab_size=65, rnn_size=H, num_layers=2,
                      input_keep_prob=kp, output_keep_prob=kp)
    a, la, sa = _run(cfg, B, T, True, monkeypatch, pf=pf)
    b, lb, sb = _run(cfg, B, T, False, monkeypatch)
    assert la == lb
    for u, v in zip(sa, sb):
        assert torch.equal(u, v)
    for s in a.store.specs:
        ga, gb = a.store.gview(s.name), b.store.gview(s.name)
        if s.name.endswith("/bias"):
            assert rel(ga, gb) < 1e-5, s.name
        else:
            assert torch.equal(ga, gb), s.name


@pytest.mark.parametrize("rs", [False, True])
def test_wide_bptt_matches_oracle_headline_shape(rs, monkeypatch, dcr_ops):
    """H = 512, B = 256 (the headline's 256-workgroup grid) against the fp32 autograd oracle:
    the all-gather kernel (lstm2_bwd_wide.hip) and the reduce-scatter one (lstm2_bwd_rs.hip)."""
    B, T, H = 256, 16, 512
    assert dcr_ops.lstm2_bwd_wide_ok(H, B) and dcr_ops.lstm2_bwd_rs_ok(H, B)
    monkeypatch.setenv("DCR_DEBUG", "persist_min_t=1" + (",bwd_rs=1" if rs else ""))
    cfg = ModelConfig(model="lstm", vocab_size=65, rnn_size=H, num_layers=2)
    nat = CharRNN(cfg, device="cuda", seed=4)
    ref = ReferenceBackend(nat.store)
    g = torch.Generator().manual_seed(0)
    x = torch.randint(0, 65, (B, T), generator=g, dtype=torch.int32).cuda()
    y = torch.randint(0, 65, (B, T), generator=g, dtype=torch.int32).cuda()
    torch.manual_seed(2)
    st0 = [tuple(torch.randn(B, H, device="cuda") * 0.5 for _ in range(2)) for _ in range(2)]
    loss_r, _, _ = ref.train_step(x, y, [tuple(s.clone() for s in t) for t in st0])
    g_ref = nat.store.grad.clone()
    nat.store.grad.zero_()
    loss_n, _, _ = nat.backend.train_step(x, y, [tuple(s.clone() for s in t) for t in st0])
    torch.cuda.synchronize()
    nat.backend.check_errors()
    assert abs(loss_n.item() - loss_r.item()) < 2e-2
    check_grads("bwd_wide", nat.store, nat.store.grad, g_ref)


def test_wide_plan_limits(dcr_ops):
    """Where the wide kernel applies: grids of (H/32) x ceil(B/16) <= one workgroup per CU."""
    cus = dcr_ops.num_cus()
    for H, B in ((512, 256), (512, 1), (256, 512), (128, 1024)):
        assert dcr_ops.lstm2_bwd_wide_ok(H, B) == ((H // 32) * ((B + 15) // 16) <= cus), (H, B)
    assert not dcr_ops.lstm2_bwd_wide_ok(1024, 64)


@pytest.mark.parametrize("B,T,H", [(256, 8, 512), (50, 7, 128), (37, 6, 512), (100, 12, 256),
                                   (256, 130, 512), (16, 2, 512), (40, 1, 256)])
def test_rs_bptt_matches_all_gather(B, T, H, monkeypatch, dcr_ops):
    """The reduce-scatter BPTT (csrc/lstm2_bwd_rs.hip, opt-in) against the all-gather one over two steps
    (TBPTT carry, ragged batches, T = 1 and 2, the XCD-local form from T = 8): the same products
    summed in another order, so a few ulp apart -- a wrong slice, slot or tick would be O(1)."""
    assert dcr_ops.lstm2_bwd_rs_ok(H, B)
    cfg = ModelConfig(model="lstm", vocab_size=65, rnn_size=H, num_layers=2)
    a, la, sa = _run(cfg, B, T, True, monkeypatch, rs=True)
    assert a.backend._bufs[(B, T, True)]["prs"] is not None
    b, lb, sb = _run(cfg, B, T, True, monkeypatch, rs=False)
    assert abs(la - lb) < 1e-4 * max(1.0, abs(lb))
    for u, v in zip(sa, sb):
        assert rel(u, v) < 2e-3
    for s in a.store.specs:
        assert rel(a.store.gview(s.name), b.store.gview(s.name)) < 5e-3, s.name
