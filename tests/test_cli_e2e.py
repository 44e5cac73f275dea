"""End-to-end CLI acceptance tests -- the reference's only test suite (.travis.yml:21-34) made
automatic: train 15 epochs on the 100-line fixture -> model.ckpt-14 exists; resume with
--init_from into a second dir -> model.ckpt-14 again; sample.py prints non-empty text.  Plus the
reference's 1 ps + 2 worker localhost launch (launch.sh) on gloo, the sharder CLI and the
init_from compatibility checks."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CORPUS = os.path.join(ROOT, "data", "tinyshakespeare", "input.txt")


def run(args, cwd, timeout=300, check=True):
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env.pop("RANK", None)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable] + args, cwd=cwd, env=env, capture_output=True, text=True,
                       timeout=timeout)
    if check and r.returncode != 0:
        raise AssertionError(f"{args} failed ({r.returncode}):\n{r.stdout}\n{r.stderr}")
    return r


@pytest.fixture()
def teeny(tmp_path):
    d = tmp_path / "data" / "teeny"
    d.mkdir(parents=True)
    with open(CORPUS, encoding="utf-8") as f:
        lines = f.readlines()[:100]
    (d / "input.txt").write_text("".join(lines), encoding="utf-8")
    return tmp_path


def test_travis_flow_train_resume_sample(teeny):
    w = str(teeny)
    common = ["--data_dir", "data/teeny", "--log_dir", "logs", "--num_epochs", "15", "--device", "cpu"]
    r1 = run([os.path.join(ROOT, "train.py"), "--save_dir", "s1"] + common, w)
    assert (teeny / "s1" / "model.ckpt-14.index").stat().st_size > 0
    assert "train_loss" in r1.stdout and "model saved to" in r1.stdout
    assert (teeny / "s1" / "config.pkl").exists() and (teeny / "s1" / "chars_vocab.pkl").exists()
    run([os.path.join(ROOT, "train.py"), "--init_from", "s1", "--save_dir", "s2"] + common, w)
    assert (teeny / "s2" / "model.ckpt-14.index").stat().st_size > 0
    r3 = run([os.path.join(ROOT, "sample.py"), "--save_dir", "s2", "-n", "50", "--device", "cpu"], w)
    assert len(r3.stdout.strip()) > 0
    # the run wrote a JSONL metrics stream and a TensorBoard event file
    runs = list((teeny / "logs").iterdir())
    assert any((r / "metrics.jsonl").exists() for r in runs)
    assert any(any(p.name.startswith("events.out.tfevents") for p in r.iterdir()) for r in runs)


def test_init_from_rejects_incompatible_model(teeny):
    w = str(teeny)
    common = ["--data_dir", "data/teeny", "--log_dir", "logs", "--num_epochs", "1", "--device", "cpu"]
    run([os.path.join(ROOT, "train.py"), "--save_dir", "s1"] + common, w)
    r = run([os.path.join(ROOT, "train.py"), "--init_from", "s1", "--save_dir", "s2",
             "--rnn_size", "64"] + common, w, check=False)
    assert r.returncode != 0 and "disagree on 'rnn_size'" in (r.stderr + r.stdout)


def test_sample_types_and_prime(teeny):
    w = str(teeny)
    run([os.path.join(ROOT, "train.py"), "--data_dir", "data/teeny", "--save_dir", "s1",
         "--log_dir", "logs", "--num_epochs", "2", "--device", "cpu"], w)
    for st in ("0", "1", "2"):
        r = run([os.path.join(ROOT, "sample.py"), "--save_dir", "s1", "-n", "20", "--sample", st,
                 "--prime", "The ", "--device", "cpu", "--seed", "1"], w)
        out = r.stdout[:-1] if r.stdout.endswith("\n") else r.stdout  # print()'s newline only
        assert out.startswith("The ") and len(out) == 24, repr(out)
    r = run([os.path.join(ROOT, "sample.py"), "--save_dir", "s1", "-n", "5", "--bytes",
             "--device", "cpu"], w)
    # py3 bytes repr (sample.py:45-46): b'...', or b"..." when the text contains a single quote
    assert r.stdout.startswith(("b'", 'b"')), r.stdout


def test_splitter_cli_any_part_count(teeny):
    w = str(teeny)
    run([os.path.join(ROOT, "data_splitter.py"), "--data_dir", "data/teeny", "--num_parts", "4",
         "--out_dir", "shards"], w)
    parts = [np.load(teeny / "shards" / f"data-{i}.npy") for i in range(4)]
    text = (teeny / "data" / "teeny" / "input.txt").read_text(encoding="utf-8")
    assert sum(p.size for p in parts) == len(text)
    assert all(p.dtype == np.int32 for p in parts)


@pytest.mark.slow
def test_ps_plus_two_workers_launch(teeny):
    """launch.sh equivalent on CPU/gloo: ps hosts the rendezvous, workers train sync-DP on
    their shards, the chief checkpoints, every process exits 0 (no ps hang, A-16)."""
    import socket

    w = str(teeny)
    run([os.path.join(ROOT, "data_splitter.py"), "--data_dir", "data/teeny", "--num_parts", "2",
         "--out_dir", "shards"], w)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ps = f"127.0.0.1:{port}"
    workers = f"127.0.0.1:{port + 1},127.0.0.1:{port + 2}"
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT
    base = [sys.executable, os.path.join(ROOT, "train.py"), "--distributed", "--ps_hosts", ps,
            "--worker_hosts", workers, "--save_dir", "dist", "--data_dir", "data/teeny",
            "--num_epochs", "2", "--batch_size", "5", "--seq_length", "20", "--device", "cpu",
            "--log_dir", "logs"]
    procs = [subprocess.Popen(base + ["--job_name", "ps", "--task_index", "0"], cwd=w, env=env)]
    for i in range(2):
        procs.append(subprocess.Popen(base + ["--job_name", "worker", "--task_index", str(i),
                                              "--tensor_file", f"shards/data-{i}.npy"], cwd=w, env=env))
    rcs = [p.wait(timeout=300) for p in procs]
    assert rcs == [0, 0, 0]
    assert (teeny / "dist" / "checkpoint").exists()
