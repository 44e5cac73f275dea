"""Times gemm_nt (csrc/tokennorm.hip store form) against the library GEMM on config 5's dtop
shape (dlogits [32768, 8192] · softmax_wᵀ, softmax_w [512, 8192]), DCR_DEBUG variants given
as arguments (e.g. gnt_st=5), interleaved rounds, median.  Run on the GPU box:
    python scripts/micro/gemm_nt_bench.py gnt_st=4 gnt_st=5"""
import os
import sys

import torch

from distributed_char_rnn_amd.ops import native

ops = native.ops()
M, N, K = (int(v) for v in os.environ.get("GNT_SHAPE", "32768,512,8192").split(","))
A = (torch.randn(M, K, device="cuda") * 0.01).bfloat16()
B = (torch.randn(N, K, device="cuda") * 0.1).bfloat16()
C = torch.empty(M, N, device="cuda")
C2 = torch.empty(M, N, device="cuda")
variants = sys.argv[1:] or ["gnt_st=4"]


def run(v):
    if v == "lib":
        torch.mm(A, B.t(), out_dtype=torch.float32, out=C2)
    else:
        os.environ["DCR_DEBUG"] = v
        ops.gemm_nt(A, B, C)


times = {v: [] for v in ["lib"] + variants}
for v in times:
    run(v)
torch.cuda.synchronize()
for r in range(5):
    for v in times:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            run(v)
        e1.record()
        torch.cuda.synchronize()
        times[v].append(e0.elapsed_time(e1) * 1e3 / 5)
ref = A.float() @ B.float().t()
print(f"M={M} N={N} K={K}")
for v, t in times.items():
    t.sort()
    if v != "lib":
        run(v)
        torch.cuda.synchronize()
    out = C2 if v == "lib" else C
    err = ((out - ref).norm() / ref.norm()).item()
    print(f"{v:12s} median {t[len(t) // 2]:7.1f} us  {2 * M * N * K / t[len(t) // 2] / 1e6:6.0f} TF/s"
          f"  rel err {err:.1e}", flush=True)
