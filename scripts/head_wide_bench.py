"""Timing of the fused wide-vocabulary head (csrc/head_wide.hip) at the 8k-token config's head
shape (N = 256 x 128 tokens, V = 8192, H = 512) and its output variants, against the library
route it replaces (logits GEMM + one-read CE kernel).

    python scripts/head_wide_bench.py [--n 32768] [--v 8192] [--iters 20]
"""
import argparse

import torch

from distributed_char_rnn_amd.ops import native


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=32768)
    ap.add_argument("--v", type=int, default=8192)
    ap.add_argument("--h", type=int, default=512)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    ops = native.ops()
    N, V, H = args.n, args.v, args.h
    dev = "cuda"
    O = (torch.randn(N, H, device=dev) * 0.5).bfloat16()
    Ws = torch.randn(H, V, device=dev) * 0.05
    WsT = Ws.t().contiguous().bfloat16()
    Wsb = Ws.bfloat16()
    bias = torch.randn(V, device=dev) * 0.1
    y = torch.randint(0, V, (N,), device=dev, dtype=torch.int32)
    nb = ops.head_wide_blocks(N)
    rl = torch.empty(N, device=dev)
    dl = torch.empty(N, V, dtype=torch.bfloat16, device=dev)
    lg = torch.empty(N, V, device=dev)
    colpart = torch.empty(ops.head_wide_colpart_rows(N) * V, device=dev)
    db = torch.empty(V, device=dev)
    ws = torch.empty(ops.head_wide_workspace(N), device=dev)
    loss = torch.empty(1, device=dev)
    s = 1.0 / N
    variants = {
        "train (dlogits + d softmax_b)": lambda: ops.head_wide(O, WsT, bias, y, s, rl, dl, None,
                                                               colpart, db, ws, loss),
        "dlogits only (no d softmax_b)": lambda: ops.head_wide(O, WsT, bias, y, s, rl, dl, None,
                                                               None, None, ws, loss),
        "eval (loss only)": lambda: ops.head_wide(O, WsT, bias, y, s, None, None, None, None, None,
                                                  ws, loss),
        "train + fp32 logits": lambda: ops.head_wide(O, WsT, bias, y, s, rl, dl, lg, colpart, db,
                                                     ws, loss),
    }
    flop = 2.0 * N * V * H
    for k, fn in variants.items():
        us = timed(fn, args.iters)
        print(f"{k:34s} {us:8.1f} us   ({flop / us / 1e6:.0f} TFLOP/s per logits pass)")
    # the two head GEMMs behind it (dW_s = Oᵀ·dlog, dtop = dlog·W_sᵀ) in candidate layouts
    f32 = torch.float32
    gemms = {
        "dW_s  mm(Oᵀ, dlog) [H, V]": lambda: torch.mm(O.t(), dl, out_dtype=f32),
        "dW_sᵀ mm(dlogᵀ, O) [V, H]": lambda: torch.mm(dl.t(), O, out_dtype=f32),
        "dW_s  split-K 4 (bmm + sum)": lambda: torch.bmm(
            O.unflatten(0, (4, N // 4)).transpose(1, 2), dl.unflatten(0, (4, N // 4)),
            out_dtype=f32).sum(0),
        "dW_s  split-K 8 (bmm + sum)": lambda: torch.bmm(
            O.unflatten(0, (8, N // 8)).transpose(1, 2), dl.unflatten(0, (8, N // 8)),
            out_dtype=f32).sum(0),
        "dtop  mm(dlog, W_sᵀ) fp32": lambda: torch.mm(dl, WsT, out_dtype=f32),
        "dtop  mm(dlog, W_sᵀ) bf16": lambda: torch.mm(dl, WsT),
    }
    for k, fn in gemms.items():
        us = timed(fn, args.iters)
        print(f"{k:34s} {us:8.1f} us   ({flop / us / 1e6:.0f} TFLOP/s)")
    if ops.xent_wide_supported(V):
        xp = torch.empty(ops.xent_num_partials(N), device=dev)
        cp = torch.empty(ops.xent_wide_waves(N) * V, device=dev)

        def lib():
            lgl = torch.mm(O, Wsb, out_dtype=torch.float32)
            ops.xent_wide(lgl, bias, y, s, rl, dl, cp, db, xp, loss)
        print(f"{'library GEMM + xent_wide':34s} {timed(lib, args.iters):8.1f} us")


if __name__ == "__main__":
    main()
