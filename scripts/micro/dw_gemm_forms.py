"""Weight-gradient GEMM forms of the headline step (2-layer LSTM-512, N = 32768 tokens):
three [512 x 2048] x K=32768 products (dW_h0, dW_x1, dW_h1) as split-K batched GEMMs (the
current form) vs one [1024 x 2048] product for layer 1 (A = [h0_t | h1_{t-1}] with ld 2H),
with and without split-K; slab sums included, achieved TFLOP/s."""
import torch

N, H = 32768, 512
G = 4 * H
bf, f32 = torch.bfloat16, torch.float32
dev = "cuda"


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


def tn(A, B, S, out):
    """out = Aᵀ B (A [K, M] maybe strided rows), split-K S slabs summed."""
    K, M = A.shape
    if S == 1:
        return torch.mm(A.t(), B, out_dtype=f32, out=out)
    a = A.unflatten(0, (S, K // S)).transpose(1, 2)
    b = B.unflatten(0, (S, K // S))
    return torch.sum(torch.bmm(a, b, out_dtype=f32), 0, out=out)


hb = torch.randn(N, 2 * H, device=dev).to(bf)  # [h0_t | h1_{t-1}] rows
h0p = torch.randn(N, H, device=dev).to(bf)
dz0 = torch.randn(N, G, device=dev).to(bf)
dz1 = torch.randn(N, G, device=dev).to(bf)
o1 = torch.empty(H, G, device=dev)
o2 = torch.empty(2 * H, G, device=dev)
fl3 = 3 * 2.0 * N * H * G
for S in (4, 8, 16):
    t = timeit(lambda: (tn(h0p, dz0, S, o1), tn(hb[:, :H], dz1, S, o1), tn(hb[:, H:], dz1, S, o1)))
    print(f"3 x [512x2048] split-K S={S}: {t:.1f} us ({fl3 / t / 1e6:.0f} TF/s)", flush=True)
for S in (1, 2, 4, 8):
    t = timeit(lambda: (tn(h0p, dz0, 8, o1), tn(hb, dz1, S, o2)))
    print(f"[512x2048] S=8 + [1024x2048] S={S}: {t:.1f} us ({fl3 / t / 1e6:.0f} TF/s)", flush=True)
# unsummed slabs (the backend defers the sums into one prep launch)
for S in (4, 8):
    a1 = hb.unflatten(0, (S, N // S)).transpose(1, 2)
    b1 = dz1.unflatten(0, (S, N // S))
    a0 = h0p.unflatten(0, (S, N // S)).transpose(1, 2)
    b0 = dz0.unflatten(0, (S, N // S))
    t3 = timeit(lambda: (torch.bmm(a0, b0, out_dtype=f32), torch.bmm(a1[:, :H], b1, out_dtype=f32),
                         torch.bmm(a1[:, H:], b1, out_dtype=f32)))
    t2 = timeit(lambda: (torch.bmm(a0, b0, out_dtype=f32), torch.bmm(a1, b1, out_dtype=f32)))
    print(f"slabs only S={S}: 3 GEMMs {t3:.1f} us ({fl3 / t3 / 1e6:.0f}), 2 GEMMs {t2:.1f} us ({fl3 / t2 / 1e6:.0f})", flush=True)
