"""XCD-resident hand-offs (csrc/persist_common.h, ``DCR_DEBUG xcdloc``) against the write-through
protocol they replace on single-XCD columns.

The local form keeps a column's ring lines and per-workgroup flags in one XCD's L2 (plain payload
stores, plain flag stores, sc1 loads); the write-through form stores sc1 and signals with atomic
counters.  Both compute exactly the same products in the same order, so every result -- losses,
the TBPTT state and every gradient -- must be bitwise identical.  A stale hand-off read (a value
of the ring slot's previous occupant, two ticks old) would change them, so long sequences over
several steps are the in-situ stale-read check (the tagged-line stress test is
scripts/micro/handoff_xcd.hip).  Each run also asserts that the local form actually engaged: the
kernels mark a column that ran XCD-local in its counter region (slot 0, dword 1)."""
import pytest
import torch

from distributed_char_rnn_amd.models.char_rnn import CharRNN
from distributed_char_rnn_amd.models.params import ModelConfig

pytestmark = pytest.mark.gpu


def _run(cfg, B, T, loc, monkeypatch, steps):
    monkeypatch.setenv("DCR_SPIN_LIMIT", str(1 << 22))
    monkeypatch.setenv("DCR_DEBUG", "xcdloc=1" if loc else "xcdloc=0")
    m = CharRNN(cfg, device="cuda", seed=5)
    plan = m.backend._persist_plan(B, True, T)
    if cfg.model == "gru":
        assert plan.gru_persist, plan
    else:
        assert plan.pair and plan.pair_bwd, plan
    g = torch.Generator().manual_seed(B * 7 + T)
    st = m.zero_state(B)
    losses = []
    for _ in range(steps):
        x = torch.randint(0, cfg.vocab_size, (B, T), generator=g, dtype=torch.int32).cuda()
        y = torch.randint(0, cfg.vocab_size, (B, T), generator=g, dtype=torch.int32).cuda()
        loss, st, _ = m.backend.train_step(x, y, st)
        losses.append(loss.item())
    torch.cuda.synchronize()
    m.backend.check_errors()
    cnt = m.backend._bufs[(B, T, True)]["cnt"]
    L = cfg.num_layers
    bwd_mark = 1
    if cfg.model == "gru":  # the bwd's mark sits in its second counter set (dZg)
        ops = m.backend.ops
        nt = int(ops.gru_persist_ub(cfg.rnn_size, B)) >> 4
        ncol = -(-B // (16 * nt))  # 16 nt-row batch groups
        bwd_mark = ncol * (T + 1) * 4 + 1
    # column 0 of the first layer (pair) forward / BPTT
    marks = (int(cnt[0][1].item()), int(cnt[L][bwd_mark].item()))
    return m, losses, [s.clone() for t in st for s in t], marks


# `local`: whether every column's workgroups sit on one XCD (the XCD-padded grid,
# persist_common.h xcd_grid, also covers fewer than 8 columns)
@pytest.mark.parametrize("model,B,T,H,drop,steps,local", [
    ("lstm", 256, 1024, 512, False, 4, 1),  # headline shape: fwd G = 1 + wide BPTT, 4 x 1026 ticks
    ("lstm", 512, 64, 512, False, 2, 1),    # forward G = 2 + the 16 x 32 BPTT at G = 2
    ("lstm", 50, 40, 128, False, 2, 1),     # ragged batch, H = 128: 2 columns (padded grid)
    ("lstm", 256, 64, 512, True, 2, 1),     # dropout instantiations
    ("gru", 128, 512, 1024, False, 3, 1),   # config 3's GRU-1024 shape: 2 hand-offs per step
    ("gru", 50, 40, 256, False, 2, 1),      # ragged GRU batch: 4 columns (padded grid)
])
def test_local_handoff_bitwise(model, B, T, H, drop, steps, local, monkeypatch):
    kp = 0.8 if drop else 1.0
    cfg = ModelConfig(model=model, vocab_size=65, rnn_size=H, num_layers=2,
                      input_keep_prob=kp, output_keep_prob=kp)
    a, la, sa, ma = _run(cfg, B, T, True, monkeypatch, steps)
    b, lb, sb, mb = _run(cfg, B, T, False, monkeypatch, steps)
    assert ma == (local, local), ma  # the local form ran where it can (one XCD per column)
    assert mb == (0, 0), mb
    assert la == lb
    for u, v in zip(sa, sb):
        assert torch.equal(u, v)
    for s in a.store.specs:
        assert torch.equal(a.store.gview(s.name), b.store.gview(s.name)), s.name
