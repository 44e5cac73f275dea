"""The headline's two weight-gradient GEMM shapes (2-layer LSTM-512, 32768 tokens): layer 1's
merged [2H x 4H] = [1024 x 2048] and layer 0's [512 x 2048], hand-written wgrad kernel
(csrc/wgrad.hip, split-K slabs) vs the library split-K bmm the step uses otherwise, slabs only
(the step sums them in its prep flush); plus the relative error against an fp32 product."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from distributed_char_rnn_amd.engine.native.gemm import split_k  # noqa: E402
from distributed_char_rnn_amd.ops import native  # noqa: E402

ops = native.ops()
bf, f32 = torch.bfloat16, torch.float32
K = int(os.environ.get("WG_K", "32768"))


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for M, N in ((1024, 2048), (512, 2048), (2048, 8192), (1024, 3072)):
    A = torch.randn(K, M, device="cuda").to(bf)
    B = torch.randn(K, N, device="cuda").to(bf)
    fl = 2.0 * K * M * N
    S = split_k(K, M, N)
    a3 = A.unflatten(0, (S, K // S)).transpose(1, 2)
    b3 = B.unflatten(0, (S, K // S))
    t_lib = timeit(lambda: torch.bmm(a3, b3, out_dtype=f32))
    Sw = int(ops.wgrad_plan(1, M, N, K))
    part = torch.empty(Sw, M, N, device="cuda")
    t_wg = timeit(lambda: ops.wgrad([A], [B], [part]))
    ref = A.float().t() @ B.float()
    err = ((part.sum(0) - ref).norm() / ref.norm()).item()
    print(f"[{M} x {N}] K={K}: library S={S} {t_lib:7.1f} us ({fl / t_lib / 1e6:5.0f} TF/s)   "
          f"wgrad S={Sw} {t_wg:7.1f} us ({fl / t_wg / 1e6:5.0f} TF/s)   rel err {err:.1e}",
          flush=True)
