"""The native GPU data-parallel path across processes: 2 ranks on cuda:0 (gloo: RCCL refuses
two ranks on one device; DCR_RECURRENCE=step: no persistent grids, which must not share CUs
with another process -- or DCR_GPU_SHARE: the headline shape on the persistent kernels, their
launches serialised across the processes), replicated and sharded (ZeRO-1) steps with clipping active, the TF
per-token norm slot and the fused step tail, against ONE process on the 2x batch; and a forced
error word on one rank makes every rank skip the update and raise on the same step.

Reference: sync DP replaces the parameter server of train.py:117-135 (model.py:98); the
replicas must stay identical and equal to the single-process step on the concatenated batch."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CFG = dict(model="lstm", vocab_size=65, rnn_size=128, num_layers=2)
CLIP = 0.01
B, T, STEPS = 16, 16, 3
# the headline's model shape on the persistent kernels (two-layer wavefront forward, wide BPTT,
# exclusive-mode bucket release, per-bucket wgrad / FINALIZE launches): DCR_GPU_SHARE serialises
# the two processes' persistent launches with a file lock (engine/native/backend.py)
CFG_HL = dict(model="lstm", vocab_size=65, rnn_size=512, num_layers=2)
B_HL = 64


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(rows):
    rng = np.random.default_rng(5)
    return rng.integers(0, 65, size=(STEPS, rows, T + 1)).astype(np.int32)


def _model(cfg=None):
    from distributed_char_rnn_amd.engine.optim import TFAdam
    from distributed_char_rnn_amd.models.char_rnn import CharRNN
    from distributed_char_rnn_amd.models.params import ModelConfig

    m = CharRNN(ModelConfig(**(cfg or CFG)), device="cuda:0", seed=4)
    opt = TFAdam(m.store, clip=CLIP, guard=m.error_word())
    m.bind_optimizer(opt)
    return m, opt


def _worker(rank, world, port, mode, fault_step, q, share=None):
    env = dict(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    if share:
        env["DCR_GPU_SHARE"] = share
    else:
        env["DCR_RECURRENCE"] = "step"
    os.environ.update(env)
    global B, CFG
    if share:
        B, CFG = B_HL, CFG_HL
    import torch.distributed as dist

    from distributed_char_rnn_amd.parallel.grad_sync import GradSync
    from distributed_char_rnn_amd.parallel.zero import ShardedStep

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m, opt = _model()
        guard = m.error_word()
        dist.broadcast(m.store.flat, 0)
        m.params_changed()
        if mode == "replicated":
            sync = GradSync(m.store, world, 0.05, "fp32", guard=guard)
            opt.guard = sync.guard_view
        else:
            sync = ShardedStep(m.store, opt, world, rank, wire="fp32", bucket_mb=0.05, guard=guard)
        m.backend.defer_err_poll = True
        if share:  # the persistent wavefront kernels ran (not the per-step fallback)
            P = m.backend._persist_plan(B, True, T)
            assert P.pair and P.pair_bwd and P.persistent, P
        data = _data(B * world)
        st = m.zero_state(B)
        snaps, norms, raised = [], [], []
        for s in range(STEPS):
            blk = torch.from_numpy(data[s, rank * B:(rank + 1) * B]).cuda()
            sync.reset()
            if s == fault_step and rank == 1:
                guard.fill_(7)  # this rank's recurrence "times out" during the step's backward
            _, st, _ = m.train_step(blk[:, :-1], blk[:, 1:], st, sync)
            if mode == "replicated":
                gs = sync.finish(defer_scale=True)
                norms.append(float(opt.step(0.01, grad_scale=gs)))
            else:
                norms.append(float(sync.step(0.01)))
            try:
                m.check_errors()
                raised.append(False)
            except RuntimeError:
                raised.append(True)
            snaps.append(m.store.flat.cpu().numpy().copy())
        q.put((rank, snaps, norms, raised))
    finally:
        dist.destroy_process_group()


def _run(mode, fault_step=-1, world=2, share=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, mode, fault_step, q, share))
          for r in range(world)]
    for p in ps:
        p.start()
    out = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    return sorted(out, key=lambda o: o[0])


def _single(world=2, persistent=False):
    b = B_HL if persistent else B
    if not persistent:
        os.environ["DCR_RECURRENCE"] = "step"
    try:
        m, opt = _model(CFG_HL if persistent else None)
        data = _data(b * world)
        st = m.zero_state(b * world)
        snaps, norms = [], []
        for s in range(STEPS):
            blk = torch.from_numpy(data[s]).cuda()
            _, st, _ = m.train_step(blk[:, :-1], blk[:, 1:], st)
            norms.append(float(opt.step(0.01)))
            snaps.append(m.store.flat.cpu().numpy().copy())
        return snaps, norms
    finally:
        os.environ.pop("DCR_RECURRENCE", None)


@pytest.mark.parametrize("mode", ["replicated", "sharded"])
def test_two_gpu_ranks_equal_single_process(mode):
    ref, ref_norms = _single()
    assert all(n > CLIP for n in ref_norms), ("clipping must be active", ref_norms)
    out = _run(mode)
    for rank, snaps, norms, raised in out:
        assert not any(raised)
        np.testing.assert_allclose(norms, ref_norms, rtol=2e-3)
        d = np.abs(snaps[-1] - ref[-1]).max() / np.abs(ref[-1]).max()
        assert d < 2e-3, d
        np.testing.assert_array_equal(snaps[-1], out[0][1][-1])  # replicas identical


@pytest.mark.parametrize("mode", ["replicated", "sharded"])
def test_error_word_on_one_rank_stops_every_rank(mode):
    out = _run(mode, fault_step=1)
    for rank, snaps, norms, raised in out:
        assert raised == [False, True, False], (rank, raised)
        np.testing.assert_array_equal(snaps[1], snaps[0])  # the faulted step was skipped
        np.testing.assert_array_equal(snaps[-1], out[0][1][-1])


@pytest.mark.parametrize("mode", ["replicated", "sharded"])
def test_two_ranks_headline_shape_persistent(mode, tmp_path):
    """The code the benchmark runs, across two processes: H = 512, L = 2 on the persistent
    two-layer wavefront kernels, exclusive-mode bucket release after the BPTT launch, the
    per-bucket weight-gradient / FINALIZE flushes, the TF norm slot and the error-word guard
    riding the last bucket -- against ONE process on the 2x batch (also persistent)."""
    ref, ref_norms = _single(persistent=True)
    assert all(n > CLIP for n in ref_norms), ("clipping must be active", ref_norms)
    out = _run(mode, share=str(tmp_path / "gpu.lock"))
    for rank, snaps, norms, raised in out:
        assert not any(raised)
        np.testing.assert_allclose(norms, ref_norms, rtol=3e-3)
        d = np.abs(snaps[-1] - ref[-1]).max() / np.abs(ref[-1]).max()
        assert d < 3e-3, d
        np.testing.assert_array_equal(snaps[-1], out[0][1][-1])  # replicas identical
