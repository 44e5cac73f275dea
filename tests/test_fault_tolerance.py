"""Failure detection and checkpoint-based recovery.

The reference has neither: a dead worker or PS leaves the other processes blocked in gRPC
(train.py:129-130), and MonitoredTrainingSession only re-creates sessions.  Here: a rank is
killed mid-training by fault injection (``DCR_FAULT=<rank>:<step>``); the survivor must notice
(heartbeat watchdog / collective error) and exit non-zero instead of hanging, and relaunching
every rank with ``--init_from <save_dir> --resume_exact`` must finish the run from the last
checkpoint.  CPU / gloo, two worker processes on localhost (the launch.sh topology)."""
import os
import socket
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CORPUS = os.path.join(ROOT, "data", "tinyshakespeare", "input.txt")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _launch(w, extra, env_extra=None):
    port = _free_port()
    workers = f"127.0.0.1:{port},127.0.0.1:{port + 1}"
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    base = [sys.executable, os.path.join(ROOT, "train.py"), "--distributed", "--worker_hosts",
            workers, "--job_name", "worker", "--data_dir", "data/teeny", "--num_epochs", "2",
            "--batch_size", "5", "--seq_length", "20", "--device", "cpu", "--log_dir", "logs",
            "--save_every", "2", "--heartbeat", "0.5", "--dist_timeout", "120"] + extra
    procs = []
    for i in range(2):
        procs.append(subprocess.Popen(base + ["--task_index", str(i), "--tensor_file",
                                              f"shards/data-{i}.npy"], cwd=w, env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    return procs


def _latest_step(save_dir):
    with open(os.path.join(save_dir, "checkpoint")) as f:
        first = f.readline()
    return int(first.strip().split("-")[-1].rstrip('"'))


@pytest.mark.slow
def test_killed_rank_detected_and_resume_completes(tmp_path):
    d = tmp_path / "data" / "teeny"
    d.mkdir(parents=True)
    with open(CORPUS, encoding="utf-8") as f:
        d.joinpath("input.txt").write_text("".join(f.readlines()[:100]), encoding="utf-8")
    w = str(tmp_path)
    env = dict(os.environ, PYTHONPATH=ROOT)
    subprocess.run([sys.executable, os.path.join(ROOT, "data_splitter.py"), "--data_dir",
                    "data/teeny", "--num_parts", "2", "--out_dir", "shards"], cwd=w, env=env,
                   check=True, capture_output=True)

    # 1. rank 1 crashes at global step 5; rank 0 must not hang
    t0 = time.time()
    procs = _launch(w, ["--save_dir", "run"], {"DCR_FAULT": "1:5"})
    outs = [p.communicate(timeout=180)[0] for p in procs]
    rcs = [p.returncode for p in procs]
    assert rcs[1] == 17, outs[1]
    assert rcs[0] != 0, outs[0]          # the survivor failed fast instead of hanging
    assert time.time() - t0 < 150
    saved = _latest_step(os.path.join(w, "run"))
    assert saved >= 2                   # checkpoints written before the crash

    # 2. relaunch every rank from the checkpoint: the run completes
    procs = _launch(w, ["--save_dir", "run", "--init_from", "run", "--resume_exact"])
    outs = [p.communicate(timeout=300)[0] for p in procs]
    assert [p.returncode for p in procs] == [0, 0], outs
    assert "restored" in outs[0]
    nb = 1310 // 100                     # batches per epoch per shard (2621-char fixture / 2)
    assert _latest_step(os.path.join(w, "run")) == 2 * nb - 1
    # the resumed run continued after the checkpoint instead of starting over
    first = next(int(ln.split("/")[0]) for ln in outs[0].splitlines()
                 if "/" in ln and "train_loss" in ln)
    assert first > 1
