"""Per-step wall time of the real training loop (engine/trainer.py) on tinyshakespeare, with and
without the device-resident batch cache (trainer._device_batches), next to bench.py's time for
the same step.  Shapes: the reference defaults (2-layer LSTM-128, B = 50, T = 50) or the headline
(2-layer LSTM-512, B = 256, T = 128).  GPU box:
    python scripts/trainer_overhead.py [off|auto|on] [default|headline]"""
import json
import os
import statistics
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_char_rnn_amd.engine import trainer  # noqa: E402

graph = sys.argv[1] if len(sys.argv) > 1 else "off"
shape = sys.argv[2] if len(sys.argv) > 2 else "default"
SHAPE = {"default": [], "headline": ["--rnn_size", "512", "--batch_size", "256", "--seq_length",
                                     "128"]}[shape]


def run(cache: bool) -> float:
    orig = trainer._device_batches
    if not cache:
        trainer._device_batches = lambda *a: None
    d = tempfile.mkdtemp()
    mf = os.path.join(d, "m.jsonl")
    try:
        trainer.main(["--data_dir", "data/tinyshakespeare", "--save_dir", d + "/s", "--log_dir",
                      d + "/l", "--max_steps", "400", "--save_every", "100000", "--log_every",
                      "50", "--metrics_file", mf, "--graph", graph] + SHAPE)
    finally:
        trainer._device_batches = orig
    rows = [r for r in map(json.loads, open(mf)) if "time_per_batch" in r]
    # (a row per 50 logged steps, each the mean time per batch over its 50 steps)
    return statistics.median(r["time_per_batch"] for r in rows[2:]) * 1e3


for cache in (False, True, False, True):
    print(f"{shape} graph={graph} device_batches={cache}: median {run(cache):.3f} ms/step", flush=True)
