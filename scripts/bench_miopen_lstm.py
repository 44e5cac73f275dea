"""Comparison baseline: stock PyTorch-ROCm ``nn.LSTM`` (MIOpen) training step on
the north-star config -- 2-layer LSTM-512, seq 128, V=65 -- with embedding, softmax-CE,
global-norm clip and Adam, bf16 autocast.  Prints one JSON line with chars/sec."""
import argparse
import json
import time

import torch
import torch.nn as nn


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--hidden", type=int, default=512)
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--vocab", type=int, default=65)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32", "fp16"])
    ap.add_argument("--model", default="lstm", choices=["lstm", "gru"])
    a = ap.parse_args()
    dev = "cuda"
    emb = nn.Embedding(a.vocab, a.hidden).to(dev)
    rnn_cls = nn.LSTM if a.model == "lstm" else nn.GRU
    lstm = rnn_cls(a.hidden, a.hidden, a.layers, batch_first=True).to(dev)
    head = nn.Linear(a.hidden, a.vocab).to(dev)
    params = list(emb.parameters()) + list(lstm.parameters()) + list(head.parameters())
    opt = torch.optim.Adam(params, lr=2e-3)
    x = torch.randint(0, a.vocab, (a.batch, a.seq), device=dev)
    y = torch.randint(0, a.vocab, (a.batch, a.seq), device=dev)
    h = torch.zeros(a.layers, a.batch, a.hidden, device=dev)
    c = torch.zeros_like(h)
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[a.dtype]

    def step(h, c):
        with torch.autocast("cuda", dtype=dt, enabled=a.dtype != "fp32"):
            if a.model == "lstm":
                out, (h2, c2) = lstm(emb(x), (h, c))
            else:
                out, h2 = lstm(emb(x), h)
                c2 = c
            logits = head(out)
            loss = nn.functional.cross_entropy(logits.float().reshape(-1, a.vocab), y.reshape(-1))
        opt.zero_grad(set_to_none=True)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(params, 5.0)
        opt.step()
        return h2.detach().float(), c2.detach().float(), loss

    for _ in range(a.warmup):
        h, c, _ = step(h, c)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        h, c, loss = step(h, c)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / a.steps
    print(json.dumps({"impl": f"torch.nn.{rnn_cls.__name__}(MIOpen)", "dtype": a.dtype, "batch": a.batch,
                      "seq": a.seq, "hidden": a.hidden, "layers": a.layers,
                      "ms_per_step": t * 1e3, "chars_per_sec": a.batch * a.seq / t,
                      "loss": float(loss)}))


if __name__ == "__main__":
    main()
