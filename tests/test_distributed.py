"""Synchronous data parallelism on the gloo backend (CPU, world size 2): the DP step must equal a
single-process step on the concatenated batch; topology mapping of the reference's PS flags;
bucket layout of the gradient all-reduce; the ps-role rendezvous."""
import argparse
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from distributed_char_rnn_amd.engine.optim import TFAdam
from distributed_char_rnn_amd.models.char_rnn import CharRNN
from distributed_char_rnn_amd.models.params import ModelConfig, ParamStore
from distributed_char_rnn_amd.parallel import topology
from distributed_char_rnn_amd.parallel.grad_sync import GradSync


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


CFG = dict(model="lstm", vocab_size=11, rnn_size=8, num_layers=2)


def _data(B, T, steps):
    rng = np.random.default_rng(0)
    return rng.integers(0, 11, size=(steps, B, T + 1)).astype(np.int32)


CLIP = 0.05  # small enough that every step clips (the clip norm itself is then under test)


def _worker(rank, world, port, B, T, steps, out_q, bucket_mb, wire, defer=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = ModelConfig(**CFG)
        m = CharRNN(cfg, device="cpu", seed=123)
        opt = TFAdam(m.store, clip=CLIP)
        sync = GradSync(m.store, world, bucket_mb, wire)
        sync.broadcast_params(0)
        data = _data(B * world, T, steps)
        state = m.zero_state(B)
        losses, norms = [], []
        for s in range(steps):
            blk = data[s, rank * B:(rank + 1) * B]
            sync.reset()
            loss, state, _ = m.train_step(blk[:, :-1], blk[:, 1:], state, sync)
            gs = sync.finish(defer_scale=defer)
            opt.step(0.01, grad_scale=gs)
            losses.append(loss.item())
            norms.append(float(opt.last_norm))
        if rank == 0:
            out_q.put((m.store.flat.clone().numpy(), losses, norms))
    finally:
        dist.destroy_process_group()


def _single(B, T, steps):
    cfg = ModelConfig(**CFG)
    m = CharRNN(cfg, device="cpu", seed=123)
    opt = TFAdam(m.store, clip=CLIP)
    data = _data(B, T, steps)
    state = m.zero_state(B)
    norms = []
    for s in range(steps):
        loss, state, _ = m.train_step(data[s, :, :-1], data[s, :, 1:], state)
        opt.step(0.01)
        norms.append(float(opt.last_norm))
    return m.store.flat.clone().numpy(), norms


@pytest.mark.parametrize("bucket_mb,wire,defer", [(8.0, "fp32", False), (0.0005, "fp32", False),
                                                  (8.0, "fp32", True)])
def test_dp_two_ranks_equals_single_process_double_batch(bucket_mb, wire, defer):
    """Both averaging paths of GradSync.finish (scale in place / folded into the optimizer),
    with clipping active every step: the TF clip norm (per-token embedding term, a sum of
    squares that averages with 1/world^2) must equal the single-process one."""
    B, T, steps, world = 3, 5, 3, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker,
                         args=(r, world, port, B, T, steps, q, bucket_mb, wire, defer))
             for r in range(world)]
    for p in procs:
        p.start()
    flat, losses, norms = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref, ref_norms = _single(B * world, T, steps)
    assert all(n > CLIP for n in ref_norms)  # clipping was active
    np.testing.assert_allclose(norms, ref_norms, rtol=1e-4)
    np.testing.assert_allclose(flat, ref, rtol=2e-4, atol=2e-6)
    assert all(np.isfinite(losses))


@pytest.mark.parametrize("bucket_mb", [8.0, 0.0005])
def test_dp_bf16_wire_fp32_accumulation(bucket_mb):
    """--allreduce_dtype bf16: bucket chunks travel as bf16 (all_to_all + all_gather) and are
    summed in fp32 -- the result stays within bf16 rounding of the fp32 exchange."""
    B, T, steps, world = 3, 5, 3, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker,
                         args=(r, world, port, B, T, steps, q, bucket_mb, "bf16", True))
             for r in range(world)]
    for p in procs:
        p.start()
    flat, losses, norms = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref, ref_norms = _single(B * world, T, steps)
    init = CharRNN(ModelConfig(**CFG), device="cpu", seed=123).store.flat.numpy()
    np.testing.assert_allclose(norms, ref_norms, rtol=1e-2)
    d, dr = flat - init, ref - init
    assert np.linalg.norm(d - dr) / np.linalg.norm(dr) < 2e-2


def test_grad_sync_buckets_are_contiguous_and_cover_buffer():
    st = ParamStore(ModelConfig(model="lstm", vocab_size=65, rnn_size=512, num_layers=2))
    gs = GradSync(st, world_size=2, bucket_mb=4.0, enabled=False)
    b = gs.buckets
    assert b[0][0] == 0 and b[-1][1] == st.numel
    for (lo, hi), (lo2, _) in zip(b, b[1:]):
        assert hi == lo2 and hi > lo
    assert len(b) >= 3  # several buckets => overlap with backward possible
    # the head bucket closes before any layer-0 parameter
    assert b[0][1] <= st.layer_range(0)[0]


def _ns(**kw):
    d = dict(distributed=True, ps_hosts=None, worker_hosts=None, job_name=None, task_index=None)
    d.update(kw)
    return argparse.Namespace(**d)


def test_topology_from_reference_flags(monkeypatch):
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    t = topology.from_args(_ns(ps_hosts="127.0.0.1:8000", worker_hosts="127.0.0.1:9000,127.0.0.1:9001",
                               job_name="worker", task_index=1))
    assert (t.rank, t.world_size, t.role, t.master_port, t.store_host_is_ps) == (1, 2, "worker", 8000, True)
    t = topology.from_args(_ns(ps_hosts="127.0.0.1:8000", worker_hosts="a:1,b:2", job_name="ps",
                               task_index=0))
    assert t.role == "ps" and t.world_size == 2
    t = topology.from_args(_ns(worker_hosts="127.0.0.1:9100,127.0.0.1:9101", job_name="worker",
                               task_index=0))
    assert t.master_port == 9100 and not t.store_host_is_ps
    with pytest.raises(ValueError):
        topology.from_args(_ns(worker_hosts="a:1", job_name="worker", task_index=3))
    assert not topology.from_args(argparse.Namespace(distributed=False)).distributed


def test_topology_env_wins(monkeypatch):
    monkeypatch.setenv("RANK", "3")
    monkeypatch.setenv("WORLD_SIZE", "8")
    monkeypatch.setenv("LOCAL_RANK", "3")
    t = topology.from_args(_ns(worker_hosts="a:1", job_name="worker", task_index=0))
    assert (t.rank, t.world_size, t.local_rank, t.from_env) == (3, 8, 3, True)


def test_topology_local_world_from_worker_hosts():
    """Ranks that share a host share its GPUs: the local rank/world drive the device choice
    and the shared-device check (process_group.pick_device)."""
    hosts = "10.0.0.1:9000,10.0.0.1:9001,10.0.0.2:9000,10.0.0.1:9002"
    t = topology.from_args(_ns(worker_hosts=hosts, job_name="worker", task_index=3))
    assert (t.rank, t.local_rank, t.local_world_size) == (3, 2, 3)
    t = topology.from_args(_ns(worker_hosts=hosts, job_name="worker", task_index=2))
    assert (t.local_rank, t.local_world_size) == (0, 1)
