"""The reference's CLI flow (.travis.yml:21-34) on the MI355X native path: train.py on the GPU
(native HIP kernels, the reference's default model: 2-layer LSTM-128, batch 50, seq 50 -- a
shape the persistent kernels do not take, so the per-step kernels run), resume with
--init_from, sample.py on the GPU (device-side sampling loop), plus the wavefront/persistent
shape (batch 64, seq 32) through the same CLI."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CORPUS = os.path.join(ROOT, "data", "tinyshakespeare", "input.txt")


def run(args, cwd, timeout=240):
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable] + args, cwd=cwd, env=env, capture_output=True, text=True,
                       timeout=timeout)
    assert r.returncode == 0, f"{args} failed ({r.returncode}):\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    return r


@pytest.fixture()
def corpus(tmp_path):
    d = tmp_path / "data" / "small"
    d.mkdir(parents=True)
    with open(CORPUS, encoding="utf-8") as f:
        lines = f.readlines()[:2000]
    (d / "input.txt").write_text("".join(lines), encoding="utf-8")
    return tmp_path


def test_train_resume_sample_on_gpu(corpus):
    w = str(corpus)
    r = run([os.path.join(ROOT, "train.py"), "--data_dir", "data/small", "--save_dir", "s1",
             "--log_dir", "logs", "--num_epochs", "2", "--device", "cuda", "--save_every", "20"], w)
    assert "train_loss" in r.stdout and "model saved to" in r.stdout
    losses = [float(ln.split("train_loss = ")[1].split(",")[0]) for ln in r.stdout.splitlines()
              if "train_loss = " in ln]
    assert losses[-1] < losses[0]                         # it learns
    assert (corpus / "s1" / "checkpoint").exists()
    r = run([os.path.join(ROOT, "train.py"), "--data_dir", "data/small", "--save_dir", "s2",
             "--log_dir", "logs", "--num_epochs", "1", "--device", "cuda", "--init_from", "s1"], w)
    assert "restored" in r.stdout or "restored" in r.stderr
    r = run([os.path.join(ROOT, "sample.py"), "--save_dir", "s2", "-n", "200", "--prime", "The ",
             "--device", "cuda", "--seed", "3"], w)
    assert r.stdout.startswith("The ") and len(r.stdout.rstrip("\n")) >= 200


def test_train_persistent_shape_on_gpu(corpus):
    """batch 64 x seq 32, rnn_size 128: the two-layer wavefront persistent kernels."""
    w = str(corpus)
    r = run([os.path.join(ROOT, "train.py"), "--data_dir", "data/small", "--save_dir", "p1",
             "--log_dir", "logs", "--num_epochs", "3", "--batch_size", "64", "--seq_length", "32",
             "--device", "cuda", "--save_every", "1000"], w)
    losses = [float(ln.split("train_loss = ")[1].split(",")[0]) for ln in r.stdout.splitlines()
              if "train_loss = " in ln]
    assert len(losses) > 10 and losses[-1] < losses[0] - 0.3
