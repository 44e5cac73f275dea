"""The data-parallel machinery on a real GPU and a real RCCL communicator (one rank: the
one-GPU box cannot host two ranks on separate devices, and RCCL refuses two ranks on one).

* a 1-rank ``nccl`` process group with ``GradSync(enabled=True)`` in the headline configuration
  (two-layer wavefront kernels, exclusive schedule, deferred 1/world scaling): RCCL's stream
  ordering against the persistent grids and the bucket releases must leave the gradients and
  the updated weights equal to the run without a process group (to the last bits: the
  weight-gradient launches are grouped by bucket release there);
* a forced persistent-kernel spin timeout (tiny DCR_SPIN_LIMIT) must leave the weights and the
  Adam slots unchanged (the optimizer reads the error word on device) and raise on the host.
"""
import socket

import pytest
import torch
import torch.distributed as dist

from distributed_char_rnn_amd.engine.optim import TFAdam
from distributed_char_rnn_amd.models.char_rnn import CharRNN
from distributed_char_rnn_amd.models.params import ModelConfig
from distributed_char_rnn_amd.parallel.grad_sync import GradSync

pytestmark = pytest.mark.gpu

CFG = dict(model="lstm", vocab_size=65, rnn_size=512, num_layers=2)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _steps(model, opt, sync, x, y, n):
    st = model.zero_state(x.shape[0])
    norms = []
    for _ in range(n):
        if sync is not None:
            sync.reset()
        loss, st, _ = model.train_step(x, y, st, sync)
        gs = sync.finish(defer_scale=True) if sync is not None else 1.0
        opt.step(2e-3, grad_scale=gs)
        norms.append(float(opt.last_norm))
    torch.cuda.synchronize()
    return loss.item(), norms


def test_rccl_one_rank_grad_sync_matches_no_sync(monkeypatch):
    monkeypatch.setenv("DCR_SPIN_LIMIT", str(1 << 22))
    B, T = 256, 32
    g = torch.Generator().manual_seed(0)
    x = torch.randint(0, 65, (B, T), generator=g, dtype=torch.int32).cuda()
    y = torch.randint(0, 65, (B, T), generator=g, dtype=torch.int32).cuda()
    a = CharRNN(ModelConfig(**CFG), device="cuda", seed=1)
    oa = TFAdam(a.store, clip=5.0, guard=a.error_word())
    la, na = _steps(a, oa, None, x, y, 3)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0,
                            world_size=1, device_id=torch.device("cuda", 0))
    try:
        b = CharRNN(ModelConfig(**CFG), device="cuda", seed=1)
        plan = b.backend._persist_plan(B, True, T)
        assert plan.pair and plan.mode == "exclusive"
        ob = TFAdam(b.store, clip=5.0, guard=b.error_word())
        sync = GradSync(b.store, 1, bucket_mb=1.0, enabled=True)  # several buckets
        assert len(sync.buckets) >= 3
        sync.broadcast_params(0)
        lb, nb = _steps(b, ob, sync, x, y, 3)
    finally:
        dist.destroy_process_group()
    a.check_errors()
    b.check_errors()
    # the hand-written weight-gradient GEMM picks its split-K slab count for the problems of
    # one launch, and under data parallelism the launches follow the bucket releases (the
    # layer-1 and layer-0 gradients in separate launches instead of one): the same products
    # summed in another order, last-bit differences in the first step's gradients (its norm
    # agrees to 1e-6); Adam's m / sqrt(v) turns last-bit differences of near-zero gradients into
    # lr-sized update differences, so later steps agree to ~1e-5.  A stream-ordering race
    # would show as stale or partial gradients, orders of magnitude above this.
    assert abs(na[0] - nb[0]) <= 1e-6 * abs(na[0]), (na, nb)
    assert all(abs(x - y) <= 1e-3 * abs(x) for x, y in zip(na, nb)), (na, nb)
    assert abs(la - lb) <= 1e-4 * abs(la), (la, lb)
    d = ((a.store.flat - b.store.flat).norm() / a.store.flat.norm()).item()
    assert d < 1e-4, d
    assert ((oa.m - ob.m).norm() / oa.m.norm()).item() < 1e-3
    assert ((oa.v - ob.v).norm() / oa.v.norm()).item() < 1e-3


def test_spin_timeout_leaves_weights_unchanged(monkeypatch):
    B, T = 256, 64
    m = CharRNN(ModelConfig(**CFG), device="cuda", seed=2)
    opt = TFAdam(m.store, clip=5.0, guard=m.error_word())
    x = torch.randint(0, 65, (B, T), dtype=torch.int32, device="cuda")
    st = m.zero_state(B)
    m.train_step(x, x, st)
    opt.step(2e-3)
    m.check_errors()
    p0, m0, v0, t0 = m.store.flat.clone(), opt.m.clone(), opt.v.clone(), opt.t
    monkeypatch.setenv("DCR_SPIN_LIMIT", "1")
    m2 = CharRNN(ModelConfig(**CFG), device="cuda", seed=2)  # reads the spin limit
    m2.store.flat.copy_(m.store.flat)
    m2.params_changed()
    opt2 = TFAdam(m2.store, clip=5.0, guard=m2.error_word())
    opt2.m.copy_(opt.m)
    opt2.v.copy_(opt.v)
    opt2.t = t0
    m2.train_step(x, x, st)
    opt2.step(2e-3)
    torch.cuda.synchronize()
    assert int(m2.backend.err.item()) != 0, "the forced timeout did not trigger"
    assert torch.equal(m2.store.flat, p0)
    assert torch.equal(opt2.m, m0) and torch.equal(opt2.v, v0)
    with pytest.raises(RuntimeError, match="timed out"):
        m2.check_errors()


def test_rccl_one_rank_sharded_step_matches_replicated(monkeypatch):
    """parallel/zero.py over a real 1-rank RCCL communicator (reduce-scatter, scalar
    all-reduce, all-gather on the persistent-kernel headline path): the shard is the whole
    buffer, so the update equals the plain fused clip + Adam step up to the norm's summation
    order."""
    from distributed_char_rnn_amd.parallel.zero import ShardedStep

    monkeypatch.setenv("DCR_SPIN_LIMIT", str(1 << 22))
    B, T = 256, 32
    g = torch.Generator().manual_seed(1)
    x = torch.randint(0, 65, (B, T), generator=g, dtype=torch.int32).cuda()
    y = torch.randint(0, 65, (B, T), generator=g, dtype=torch.int32).cuda()
    a = CharRNN(ModelConfig(**CFG), device="cuda", seed=3)
    oa = TFAdam(a.store, clip=0.01, guard=a.error_word())
    la, na = _steps(a, oa, None, x, y, 3)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0,
                            world_size=1, device_id=torch.device("cuda", 0))
    try:
        b = CharRNN(ModelConfig(**CFG), device="cuda", seed=3)
        ob = TFAdam(b.store, clip=0.01, guard=b.error_word())
        zs = ShardedStep(b.store, ob, 1, 0)
        st = b.zero_state(B)
        nb = []
        for _ in range(3):
            lb, st, _ = b.train_step(x, y, st)
            nb.append(float(zs.step(2e-3)))
        zs.gather_slots()
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()
    b.check_errors()
    assert na[0] > 0.01  # clipping active
    assert abs(lb.item() - la) < 1e-6 * max(1.0, abs(la))
    for u, v in zip(nb, na):
        assert abs(u - v) < 1e-4 * v
    assert ((b.store.flat - a.store.flat).norm() / a.store.flat.norm()).item() < 1e-5
