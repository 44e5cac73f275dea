"""Microbench of the fused TF clip-norm term (csrc/optim.hip tok_norm) at the headline shape
(N = 256*128 tokens, H = 512, K = 4H) vs the library route (GEMM to bf16 rows + sumsq)."""
import sys

import torch

from distributed_char_rnn_amd.ops import native

ops = native.ops()
N, H = (int(a) for a in sys.argv[1:3]) if len(sys.argv) > 2 else (32768, 512)
K = 4 * H
dz = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
w = (torch.randn(H, K, device="cuda") * 0.05).to(torch.bfloat16)
parts = torch.empty((N // 128) * (H // 64), device="cuda")
np_ = torch.empty(ops.opt_num_partials(N * H), device="cuda")
out = torch.empty(1, device="cuda")


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / it


t_fused = timeit(lambda: ops.tok_norm(dz, w, parts, out))
v_fused = out.item()
t_lib = timeit(lambda: ops.sumsq(torch.mm(dz, w.t()), np_, out))
flop = 2 * N * H * K
print(f"N={N} H={H} K={K}: fused {t_fused:.1f} us ({flop / t_fused / 1e6:.0f} TFLOP/s), "
      f"library {t_lib:.1f} us; values {v_fused:.6g} vs {out.item():.6g}")
