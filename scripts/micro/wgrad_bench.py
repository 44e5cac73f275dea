"""Headline weight-gradient GEMMs (2-layer LSTM-512, N = 32768 tokens): the hand-written
wgrad kernel (one launch for dW_h1 + dW_x1, one for dW_h0, 256 x 256 tiles, split-K slabs) vs
the library split-K bmm form (S = 8), slabs only (the step sums them in its prep flush)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from distributed_char_rnn_amd.ops import native

ops = native.ops()
N, H = 32768, 512
G = 4 * H
bf, f32 = torch.bfloat16, torch.float32


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


hb = torch.randn(N, 2 * H, device="cuda").to(bf)
h0p = torch.randn(N, H, device="cuda").to(bf)
dz0 = torch.randn(N, G, device="cuda").to(bf)
dz1 = torch.randn(N, G, device="cuda").to(bf)
fl3 = 3 * 2.0 * N * H * G
S8 = 8
a0 = h0p.unflatten(0, (S8, N // S8)).transpose(1, 2)
b0 = dz0.unflatten(0, (S8, N // S8))
a1 = hb.unflatten(0, (S8, N // S8)).transpose(1, 2)
b1 = dz1.unflatten(0, (S8, N // S8))
t = timeit(lambda: (torch.bmm(a0, b0, out_dtype=f32), torch.bmm(a1[:, :H], b1, out_dtype=f32),
                    torch.bmm(a1[:, H:], b1, out_dtype=f32)))
print(f"library bmm S=8, 3 GEMMs: {t:.1f} us ({fl3 / t / 1e6:.0f} TF/s)", flush=True)
for S1, S0 in ((0, 0), (4, 8), (8, 16), (6, 12)):
    S1 = S1 or ops.wgrad_plan(2, H, G, N)
    S0 = S0 or ops.wgrad_plan(1, H, G, N)
    p1 = torch.empty(2, S1, H, G, device="cuda")
    p0 = torch.empty(1, S0, H, G, device="cuda")
    t = timeit(lambda: (ops.wgrad([hb[:, :H], hb[:, H:]], [dz1, dz1], p1),
                        ops.wgrad([h0p], [dz0], p0)))
    print(f"wgrad S={S1}/{S0}, 2 launches: {t:.1f} us ({fl3 / t / 1e6:.0f} TF/s)", flush=True)
p3 = torch.empty(3, 5, H, G, device="cuda")
t = timeit(lambda: ops.wgrad([h0p, hb[:, :H], hb[:, H:]], [dz0, dz1, dz1], p3))
print(f"wgrad S=5, 1 launch of 3: {t:.1f} us ({fl3 / t / 1e6:.0f} TF/s)", flush=True)
ref = hb[:, :H].float().t() @ dz1.float()
ops.wgrad([hb[:, :H]], [dz1], p3[:1, :1])
torch.cuda.synchronize()
print("rel err (S=1):", ((p3[0, 0] - ref).norm() / ref.norm()).item())
