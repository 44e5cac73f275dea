"""Time the library GEMM shapes of one training step of the bench config (2-layer LSTM-512,
B=256, T=128 -> N=32768 tokens, V=65) and split-K alternatives built from torch.bmm.

    python scripts/bench_gemms.py
"""
import torch

N, H, V = 32768, 512, 65
G = 4 * H
dev = "cuda"
bf, f32 = torch.bfloat16, torch.float32
torch.manual_seed(0)


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


X = torch.randn(N, H, device=dev).to(bf)
Z = torch.randn(N, G, device=dev).to(bf)
D = torch.randn(N, V, device=dev).to(bf)
Wx = torch.randn(H, G, device=dev).to(bf)
Ws = torch.randn(H, V, device=dev).to(bf)
out = torch.empty(H, G, device=dev)


def splitk(A, B, S):
    K, M = A.shape
    Nn = B.shape[1]
    a = A.view(S, K // S, M).transpose(1, 2)
    b = B.view(S, K // S, Nn)
    return torch.bmm(a, b, out_dtype=f32).sum(0)


rows = []
ref = torch.mm(X.t(), Z, out_dtype=f32)
rows.append(("dW  = X^T Z  [512x2048, K=32768] mm", timeit(lambda: torch.mm(X.t(), Z, out_dtype=f32, out=out)), 2 * N * H * G))
for S in (4, 8, 16, 32):
    r = splitk(X, Z, S)
    err = ((r - ref).norm() / ref.norm()).item()
    rows.append((f"dW  split-K bmm S={S} (+sum) err={err:.1e}", timeit(lambda: splitk(X, Z, S)), 2 * N * H * G))
rows.append(("dWs = O^T dlog [512x65, K=32768] mm", timeit(lambda: torch.mm(X.t(), D, out_dtype=f32)), 2 * N * H * V))
for S in (16, 64):
    rows.append((f"dWs split-K bmm S={S}", timeit(lambda: splitk(X, D, S)), 2 * N * H * V))
dx = torch.empty(N, H, device=dev)
rows.append(("dX  = Z Wx^T [32768x512, K=2048] mm", timeit(lambda: torch.mm(Z, Wx.t(), out_dtype=f32, out=dx)), 2 * N * H * G))
lg = torch.empty(N, V, device=dev)
bs = torch.zeros(V, device=dev)
rows.append(("logits = O Ws + b [32768x65, K=512]", timeit(lambda: torch.addmm(bs, X, Ws, out_dtype=f32, out=lg)), 2 * N * H * V))
dt = torch.empty(N, H, device=dev)
rows.append(("dtop = dlog Ws^T [32768x512, K=65]", timeit(lambda: torch.mm(D, Ws.t(), out_dtype=f32, out=dt)), 2 * N * H * V))
for name, us, fl in rows:
    print(f"{name:<48} {us:9.1f} us  {fl / us / 1e6:8.1f} TFLOP/s")

# NT form of the weight gradient: activations stored transposed ([H, N], K contiguous)
XT = X.t().contiguous()
ZT = Z.t().contiguous()
ref = torch.mm(X.t(), Z, out_dtype=f32)


def splitk_nt(AT, BT, S):
    M, K = AT.shape
    Nn = BT.shape[0]
    a = AT.view(M, S, K // S).transpose(0, 1)          # [S, M, K/S], lda = K
    b = BT.view(Nn, S, K // S).transpose(0, 1)         # [S, Nn, K/S]
    return torch.bmm(a, b.transpose(1, 2), out_dtype=f32).sum(0)


extra = [("dW NT  = XT ZT^T mm", timeit(lambda: torch.mm(XT, ZT.t(), out_dtype=f32, out=out)), 2 * N * H * G)]
for S in (4, 8, 16):
    r = splitk_nt(XT, ZT, S)
    err = ((r - ref).norm() / ref.norm()).item()
    extra.append((f"dW NT split-K S={S} err={err:.1e}", timeit(lambda: splitk_nt(XT, ZT, S)), 2 * N * H * G))
for name, us, fl in extra:
    print(f"{name:<52} {us:8.1f} us  {fl / us / 1e6:8.1f} TFLOP/s")

# output-precision / orientation variants of the weight gradient (the library picks stream-K
# kernels for some of them)
outT = torch.empty(G, H, device=dev)
more = [
    ("dW  mm bf16 out", timeit(lambda: torch.mm(X.t(), Z)), 2 * N * H * G),
    ("dW^T = Z^T X mm fp32 out [2048x512]", timeit(lambda: torch.mm(Z.t(), X, out_dtype=f32, out=outT)), 2 * N * H * G),
    ("dW^T mm fp32 + transpose copy", timeit(lambda: out.copy_(torch.mm(Z.t(), X, out_dtype=f32).t())), 2 * N * H * G),
    ("dW^T = Z^T X mm bf16 out", timeit(lambda: torch.mm(Z.t(), X)), 2 * N * H * G),
]
for name, us, fl in more:
    print(f"{name:<52} {us:8.1f} us  {fl / us / 1e6:8.1f} TFLOP/s")
