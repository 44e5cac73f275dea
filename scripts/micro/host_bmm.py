"""Host-side (enqueue) cost of the one-hot dEW split-K GEMM forms (no device sync inside the
timed calls): torch.bmm with out_dtype=f32 vs alternatives."""
import time

import torch

K, M, N, S = 32768, 72, 2048, 16
a = torch.zeros(K, M, device="cuda", dtype=torch.bfloat16)
b = torch.randn(K, N, device="cuda").bfloat16()
f32 = torch.float32


def t(name, fn, n=50):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{name:40s} host {1e6 * (t1 - t0) / n:8.1f} us/call   wall {1e6 * (t2 - t0) / n:8.1f} us/call",
          flush=True)


A = a.unflatten(0, (S, K // S)).transpose(1, 2)
B = b.unflatten(0, (S, K // S))
out = torch.empty(S, M, N, device="cuda", dtype=f32)
t("bmm out_dtype=f32", lambda: torch.bmm(A, B, out_dtype=f32))
t("bmm out_dtype=f32 out=", lambda: torch.bmm(A, B, out_dtype=f32, out=out))
t("bmm bf16", lambda: torch.bmm(A, B))
t("mm out_dtype=f32 (no split)", lambda: torch.mm(a.t(), b, out_dtype=f32))
t("matmul bf16", lambda: torch.matmul(A, B))
