"""Generation throughput, 2-layer LSTM-512, vocab 65 (random init): the single-launch generator
(csrc/generate.hip) vs the replayed per-character step graph (csrc/sample.hip + hipGraph) vs
the eager per-character loop.

    PYTHONPATH=. python scripts/bench_sample.py
"""
import json
import time

import torch

from distributed_char_rnn_amd.models.char_rnn import CharRNN
from distributed_char_rnn_amd.models.params import ModelConfig

cfg = ModelConfig(model="lstm", vocab_size=65, rnn_size=512, num_layers=2)
m = CharRNN(cfg, device="cuda", seed=0)
be = m.backend
n = 500
for S in (1, 16, 64):
    for form in ("generator", "graph", "eager"):
        if form == "generator" and not be._generate_ok(S):
            continue
        kw = dict(use_graph=form != "eager", use_generator=form == "generator")
        be.sample_sequence([1, 2], 20, 1, 0, S, 0, **kw)  # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        be.sample_sequence([1, 2], n, 1, 0, S, 0, **kw)
        dt = time.perf_counter() - t0
        print(json.dumps({"streams": S, "form": form, "chars": n, "us_per_step": dt / n * 1e6,
                          "chars_per_sec": S * n / dt}), flush=True)
