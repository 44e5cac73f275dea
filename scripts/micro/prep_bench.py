#!/usr/bin/env python
"""Micro-benchmark of the batched prep kernel's task kinds at the headline shapes (2-layer
LSTM-512, B = 256, T = 128, V = 65): one launch per kind, CUDA-event timed (median of 20)."""
import torch

from distributed_char_rnn_amd.ops import native


def timeit(fn, n=20):
    ts = []
    for _ in range(n + 3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts = sorted(ts[3:])
    return ts[len(ts) // 2]


def main():
    ops = native.ops()
    dev = "cuda"
    H, GW, V, B, T = 512, 2048, 65, 256, 128
    N = B * T
    E = torch.randn(V, H, device=dev)
    W = torch.randn(H, GW, device=dev)
    bias = torch.randn(GW, device=dev)
    tab = torch.empty(V, GW, device=dev)
    x = torch.randint(0, V, (B, 16 * T), dtype=torch.int32, device=dev)[:, :T]
    oh = torch.empty(N, 72, dtype=torch.bfloat16, device=dev)
    xt = torch.empty(T, B, dtype=torch.int32, device=dev)
    slabs = [torch.randn(8, H, GW, device=dev) for _ in range(3)]
    outs = [torch.empty(H, GW, device=dev) for _ in range(3)]
    sd = torch.randn(16, 72, GW, device=dev)
    od = torch.empty(72, GW, device=dev)
    ss = torch.randn(16, H, V, device=dev)
    os_ = torch.empty(H, V, device=dev)
    kk = torch.randn(2 * H, GW, device=dev)
    wb = [torch.empty(H, GW, dtype=torch.bfloat16, device=dev) for _ in range(2)]
    wt = [torch.empty(GW, H, dtype=torch.bfloat16, device=dev) for _ in range(2)]
    cases = {
        "table": ([E], [tab], [6], [W, bias]),
        "onehot": ([x], [oh], [5], []),
        "ids_transpose": ([x, x], [xt, xt], [1, 1], []),
        "sum 3x[8,512,2048]": (slabs, outs, [3, 3, 3], []),
        "sum dEW [16,72,2048]": ([sd], [od], [3], []),
        "sum softmax_w [16,512,65] (scalar)": ([ss], [os_], [3], []),
        "weights copy+transpose (2 layers)": ([kk[H:], kk[H:], kk[:H], kk[:H]],
                                              [wb[0], wt[0], wb[1], wt[1]], [0, 1, 0, 1], []),
    }
    for name, (s, d, m, e) in cases.items():
        us = timeit(lambda: ops.prep(s, d, m, e))
        print(f"{name:40s} {us:8.1f} us")


if __name__ == "__main__":
    main()
