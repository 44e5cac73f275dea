"""Per-time-step recurrent GEMMs of the H = 2048 LSTM at large batch (B = 256 ... 1024):
forward NT form z = h·(W_hᵀ)ᵀ and BPTT dh = dZ·W_hᵀ, fp32 out, achieved TFLOP/s."""
import torch

f32, bf = torch.float32, torch.bfloat16
H = 2048


def timeit(fn, reps=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / reps


Wh = (torch.randn(H, 4 * H, device="cuda") * 0.02).to(bf)
WhT = Wh.t().contiguous()
for B in (256, 512, 1024):
    h = torch.randn(B, H, device="cuda").to(bf)
    dz = torch.randn(B, 4 * H, device="cuda").to(bf)
    z = torch.empty(B, 4 * H, device="cuda")
    dh = torch.empty(B, H, device="cuda")
    fl = 2.0 * B * H * 4 * H
    tf = timeit(lambda: torch.mm(h, WhT.t(), out_dtype=f32, out=z))
    tb = timeit(lambda: torch.mm(dz, Wh.t(), out_dtype=f32, out=dh))
    tb2 = timeit(lambda: torch.mm(dz, WhT, out_dtype=f32, out=dh))
    print(f"B={B}: fwd {tf:.1f} us ({fl / tf / 1e6:.0f} TF/s)  bwd TN {tb:.1f} us ({fl / tb / 1e6:.0f})"
          f"  bwd NN {tb2:.1f} us ({fl / tb2 / 1e6:.0f})", flush=True)

# BPTT step product as split-K slabs over K = 4H (the cell kernel sums nsplit slabs itself)
for B in (256, 512, 1024):
    dz = torch.randn(B, 4 * H, device="cuda").to(bf)
    fl = 2.0 * B * H * 4 * H
    for S in (2, 4, 8):
        a = dz.view(B, S, 4 * H // S).transpose(0, 1)        # [S, B, K/S]
        w1 = Wh.view(H, S, 4 * H // S).permute(1, 2, 0)       # [S, K/S, H] (Wh rows strided)
        w2 = WhT.view(S, 4 * H // S, H)                       # [S, K/S, H] contiguous
        o = torch.empty(S, B, H, device="cuda")
        t1 = timeit(lambda: torch.bmm(a, w1, out_dtype=f32, out=o))
        t2 = timeit(lambda: torch.bmm(a, w2, out_dtype=f32, out=o))
        print(f"B={B} bwd split-K S={S}: W_h strided {t1:.1f} us ({fl / t1 / 1e6:.0f}), "
              f"W_hᵀ contiguous {t2:.1f} us ({fl / t2 / 1e6:.0f})", flush=True)
