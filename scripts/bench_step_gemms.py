"""Per-time-step recurrent GEMMs of the large-H LSTM (H = 2048) on the library path:
forward z = h·W_h ([B, H] x [H, 4H]) and BPTT dh = dZ·W_hᵀ ([B, 4H] x [4H, H]), fp32 out."""
import torch

f32, bf = torch.float32, torch.bfloat16
H = 2048


def timeit(fn, reps=50):
    for _ in range(5):
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
for B in (64, 128, 256):
    h = torch.randn(B, H, device="cuda").to(bf)
    dz = torch.randn(B, 4 * H, device="cuda").to(bf)
    z = torch.empty(B, 4 * H, device="cuda")
    dh = torch.empty(B, H, device="cuda")
    tf = timeit(lambda: torch.mm(h, Wh, out_dtype=f32, out=z))
    tb = timeit(lambda: torch.mm(dz, Wh.t(), out_dtype=f32, out=dh))
    # graph-replayed chain of 64 steps (launch gaps as the T loop would see them)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(64):
            torch.mm(dz, Wh.t(), out_dtype=f32, out=dh)
    tg = timeit(lambda: g.replay(), reps=10) / 64
    print(f"B={B}: fwd z=h·W_h {tf:.1f} us, bwd dh=dZ·W_hᵀ {tb:.1f} us, bwd in a graph {tg:.1f} us/step")
