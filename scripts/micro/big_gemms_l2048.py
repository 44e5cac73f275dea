"""Token-reduction / projection GEMMs of the LSTM-2048 config at B = 512, T = 512 (N = 262144
tokens): input projection zx = X·W_x (fp32 out), dX = dZ·W_xᵀ (fp32 out), weight gradient
dW = Xᵀ·dZ (split-K S = 4 slabs); achieved TFLOP/s.  Run with and without TunableOp."""
import torch

f32, bf = torch.float32, torch.bfloat16
N, H = 262144 // 2, 2048  # half the tokens (memory of the micro); same per-row shapes
G = 4 * H


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / reps


X = torch.randn(N, H, device="cuda").to(bf)
Wx = (torch.randn(H, G, device="cuda") * 0.02).to(bf)
dZ = torch.randn(N, G, device="cuda").to(bf)
zx = torch.empty(N, G, device="cuda")
dX = torch.empty(N, H, device="cuda")
fl = 2.0 * N * H * G
t = timeit(lambda: torch.mm(X, Wx, out_dtype=f32, out=zx))
print(f"zx = X·W_x   [{N}x{H}]x[{H}x{G}] fp32 out: {t:.0f} us ({fl / t / 1e6:.0f} TF/s)", flush=True)
zb = torch.empty(N, G, device="cuda", dtype=bf)
t = timeit(lambda: torch.mm(X, Wx, out=zb))
print(f"zx = X·W_x   bf16 out: {t:.0f} us ({fl / t / 1e6:.0f} TF/s)", flush=True)
t = timeit(lambda: torch.mm(dZ, Wx.t(), out_dtype=f32, out=dX))
print(f"dX = dZ·W_xᵀ fp32 out: {t:.0f} us ({fl / t / 1e6:.0f} TF/s)", flush=True)
for S in (1, 4):
    a = X.unflatten(0, (S, N // S)).transpose(1, 2)
    b = dZ.unflatten(0, (S, N // S))
    t = timeit(lambda: torch.bmm(a, b, out_dtype=f32))
    print(f"dW = Xᵀ·dZ  split-K S={S} slabs: {t:.0f} us ({fl / t / 1e6:.0f} TF/s)", flush=True)
