"""Sharded data-parallel optimizer step (parallel/zero.py, ZeRO stage 1) on gloo, world 2:
reduce-scatter + clip/TF-Adam on each rank's shard + all-gather must give the replicated
all-reduce path's parameters and Adam slots (clipping active); the bf16-wire exchange (fp32
accumulation) stays within bf16 rounding of it."""
import os
import socket

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

from distributed_char_rnn_amd.engine.optim import TFAdam
from distributed_char_rnn_amd.models.char_rnn import CharRNN
from distributed_char_rnn_amd.models.params import ModelConfig
from distributed_char_rnn_amd.parallel.grad_sync import GradSync
from distributed_char_rnn_amd.parallel.zero import ShardedStep

CFG = dict(model="lstm", vocab_size=11, rnn_size=8, num_layers=2)
CLIP = 0.05


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, mode, steps, q, bucket_mb=8.0):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = CharRNN(ModelConfig(**CFG), device="cpu", seed=5)
        opt = TFAdam(m.store, clip=CLIP)
        sync = GradSync(m.store, world, bucket_mb, "fp32", enabled=(mode == "replicated"))
        sync.broadcast_params(0) if mode == "replicated" else dist.broadcast(m.store.flat, 0)
        zs = None if mode == "replicated" else ShardedStep(m.store, opt, world, rank,
                                                           wire=mode.split("_")[1],
                                                           bucket_mb=bucket_mb)
        rng = np.random.default_rng(0)
        data = rng.integers(0, 11, size=(steps, 4 * world, 7)).astype(np.int32)
        st = m.zero_state(4)
        norms = []
        for s in range(steps):
            blk = data[s, rank * 4:(rank + 1) * 4]
            sync.reset()
            _, st, _ = m.train_step(blk[:, :-1], blk[:, 1:], st, sync)
            if zs is None:
                gs = sync.finish(defer_scale=True)
                norms.append(float(opt.step(0.01, grad_scale=gs)))
            else:
                norms.append(float(zs.step(0.01)))
        if zs is not None:
            zs.gather_slots()
        q.put((rank, m.store.flat.numpy().copy(), opt.m.numpy().copy(), opt.v.numpy().copy(),
               norms, opt.t))
    finally:
        dist.destroy_process_group()


def _run(mode, world=2, steps=4, bucket_mb=8.0):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, mode, steps, q, bucket_mb))
          for r in range(world)]
    for p in ps:
        p.start()
    out = [q.get(timeout=240) for _ in ps]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    return sorted(out, key=lambda o: o[0])


def test_sharded_step_equals_replicated():
    rep = _run("replicated")
    sh = _run("sharded_fp32")
    assert all(n > CLIP for n in rep[0][4]), "clipping must be active"
    for r in range(2):
        np.testing.assert_allclose(sh[r][1], rep[0][1], rtol=1e-5, atol=1e-7)   # params
        np.testing.assert_allclose(sh[r][2], rep[0][2], rtol=1e-5, atol=1e-9)   # m
        np.testing.assert_allclose(sh[r][3], rep[0][3], rtol=1e-5, atol=1e-12)  # v
        np.testing.assert_allclose(sh[r][4], rep[0][4], rtol=1e-5)              # norms
        assert sh[r][5] == rep[0][5] == 4
    np.testing.assert_array_equal(sh[0][1], sh[1][1])  # replicas stay identical


def test_many_buckets_equal_one():
    """Tiny buckets (a dozen per step, every one exchanged by the blocking collectives after
    the backward, in flat order) give the one-bucket results bitwise, replicated and sharded."""
    tiny = 1.0 / 1024  # 1 KB cap: one bucket per tensor boundary
    one_r, many_r = _run("replicated"), _run("replicated", bucket_mb=tiny)
    np.testing.assert_array_equal(many_r[0][1], one_r[0][1])
    one_s, many_s = _run("sharded_fp32"), _run("sharded_fp32", bucket_mb=tiny)
    for r in range(2):
        np.testing.assert_allclose(many_s[r][1], one_s[r][1], rtol=1e-6, atol=1e-9)
    np.testing.assert_array_equal(many_s[0][1], many_s[1][1])


def test_sharded_step_bf16_wire_close():
    rep = _run("replicated")
    sh = _run("sharded_bf16")
    dp_rep = rep[0][1] - _run_init()
    dp_sh = sh[0][1] - _run_init()
    assert np.linalg.norm(dp_sh - dp_rep) / np.linalg.norm(dp_rep) < 2e-2
    np.testing.assert_array_equal(sh[0][1], sh[1][1])


def _run_init():
    return CharRNN(ModelConfig(**CFG), device="cpu", seed=5).store.flat.numpy().copy()


def test_train_py_sharded_matches_replicated(tmp_path):
    """The trainer with --dp_mode sharded (2 gloo ranks) ends with the replicated run's
    checkpointed parameters and Adam slots (gathered on the chief before the save)."""
    import subprocess
    import sys

    from distributed_char_rnn_amd.utils import checkpoint as ckpt

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    common = ["--synthetic_text", "4000", "--num_epochs", "1", "--batch_size", "4",
              "--seq_length", "16", "--rnn_size", "16", "--num_layers", "2", "--device", "cpu",
              "--log_dir", "logs", "--save_every", "1000", "--seed", "3", "--max_steps", "6",
              "--grad_clip", "0.05"]
    env = dict(os.environ, PYTHONPATH=root, OMP_NUM_THREADS="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    finals = {}
    for mode in ("replicated", "sharded"):
        port = free_port()
        workers = f"127.0.0.1:{port},127.0.0.1:{port + 1}"
        procs = [subprocess.Popen([sys.executable, os.path.join(root, "train.py")] + common +
                                  ["--save_dir", mode, "--dp_mode", mode, "--distributed",
                                   "--worker_hosts", workers, "--job_name", "worker",
                                   "--task_index", str(i), "--dist_timeout", "120"],
                                  cwd=str(tmp_path), env=env, stdout=subprocess.PIPE,
                                  stderr=subprocess.STDOUT, text=True) for i in range(2)]
        outs = [p.communicate(timeout=300)[0] for p in procs]
        for p, o in zip(procs, outs):
            assert p.returncode == 0, o
        sd = ckpt.Saver.restore(ckpt.latest_checkpoint(str(tmp_path / mode)))
        finals[mode] = {k: np.asarray(v) for k, v in sd.items()}
    a, b = finals["replicated"], finals["sharded"]
    for k in a:
        if k.startswith("dcr/") or np.asarray(a[k]).dtype.kind not in "fc":
            continue
        np.testing.assert_allclose(b[k], a[k], rtol=1e-4, atol=1e-6, err_msg=k)
