"""--graph: the whole training step replayed from one captured hipGraph
(engine/graph_step.py) must follow the eager step exactly -- same kernels, same order."""
import pytest
import torch

from distributed_char_rnn_amd.engine.graph_step import GraphedStep
from distributed_char_rnn_amd.engine.optim import TFAdam
from distributed_char_rnn_amd.models.char_rnn import CharRNN
from distributed_char_rnn_amd.models.params import ModelConfig


def test_graph_step_unsupported_cases_cpu():
    cfg = ModelConfig(model="lstm", vocab_size=20, rnn_size=16, num_layers=2)
    m = CharRNN(cfg, device="cpu", seed=0)
    ok, why = GraphedStep.supported(m, 1)
    assert not ok and "native" in why


def _run(graph, cfg, B, T, steps, lr=2e-3, fused=False):
    m = CharRNN(cfg, device="cuda", seed=21)
    opt = TFAdam(m.store, clip=5.0, guard=m.error_word())
    if fused:  # the fused Adam tail (as bench.py / train.py bind it)
        m.bind_optimizer(opt)
        assert opt.fused is not None
    gstep = GraphedStep(m, opt) if graph else None
    g = torch.Generator().manual_seed(4)
    data = [(torch.randint(0, cfg.vocab_size, (B, T), generator=g, dtype=torch.int32),
             torch.randint(0, cfg.vocab_size, (B, T), generator=g, dtype=torch.int32))
            for _ in range(steps)]
    st = m.zero_state(B)
    losses = []
    for i, (x, y) in enumerate(data):
        if i == 3:
            st = m.zero_state(B)  # an epoch boundary: a foreign state is copied in
        if gstep is not None:
            loss, st = gstep(x.cuda(), y.cuda(), st, lr)
        else:
            loss, st, _ = m.train_step(x.cuda(), y.cuda(), st)
            opt.step(lr)
        losses.append(loss.clone())  # (eager losses are views of a ping-pong buffer)
    torch.cuda.synchronize()
    m.check_errors()
    return [float(v) for v in losses], m.store.flat.clone(), opt, gstep, st


@pytest.mark.gpu
@pytest.mark.parametrize("kind,B,T,H,L,fused", [
    ("lstm", 50, 50, 128, 2, False), ("lstm", 64, 16, 256, 3, False),
    ("lstm", 50, 50, 128, 2, True), ("gru", 50, 50, 128, 2, True),
    ("gru", 64, 16, 256, 3, False)])
def test_graph_step_equals_eager(kind, B, T, H, L, fused):
    """Fused: the captured step's prep launch carries only what the fused Adam leaves behind
    (GRU: the fp32 concatenations), not the whole layout refresh."""
    cfg = ModelConfig(model=kind, vocab_size=65, rnn_size=H, num_layers=L)
    le, pe, oe, _, se = _run(False, cfg, B, T, 7, fused=fused)
    lg, pg, og, gs, sg = _run(True, cfg, B, T, 7, fused=fused)
    assert gs.graph is not None and not gs.failed and gs.replays >= 4
    assert og.t == oe.t == 7
    assert lg == le
    assert torch.equal(pg, pe)
    assert torch.equal(og.m, oe.m) and torch.equal(og.v, oe.v)
    for a, b in zip(sg, se):
        for u, v in zip(a, b):
            assert torch.equal(u, v)


@pytest.mark.gpu
def test_graph_replays_poll_the_error_word():
    """A persistent-kernel error raised while the step is graph-replayed is reported within a
    few replays (the replays count as steps for the every-k-th non-blocking error-word copy),
    not silently skipped until the next checkpoint."""
    cfg = ModelConfig(model="lstm", vocab_size=65, rnn_size=128, num_layers=2)
    B, T = 32, 16
    m = CharRNN(cfg, device="cuda", seed=5)
    opt = TFAdam(m.store, clip=5.0, guard=m.error_word())
    gstep = GraphedStep(m, opt)
    g = torch.Generator().manual_seed(1)
    x = torch.randint(0, 65, (B, T), generator=g, dtype=torch.int32).cuda()
    y = torch.randint(0, 65, (B, T), generator=g, dtype=torch.int32).cuda()
    st = m.zero_state(B)
    for _ in range(4):
        _, st = gstep(x, y, st, 2e-3)
    torch.cuda.synchronize()
    assert gstep.graph is not None and gstep.replays >= 2
    m.error_word().fill_(7)  # as a spin timeout inside a replay would
    raised = False
    for _ in range(2 * m.backend.ERR_POLL_EVERY + 2):
        try:
            _, st = gstep(x, y, st, 2e-3)
        except RuntimeError as e:
            assert "code 7" in str(e)
            raised = True
            break
    assert raised
