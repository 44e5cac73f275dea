"""Per-time-step recurrent GEMM of the large-H LSTM (H = 2048): operand layouts and BLAS
backends (hipBLASLt vs rocBLAS) for z = h·W_h ([B, H] x [H, 4H]) and dh = dZ·W_hᵀ, fp32 out."""
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
WhT = Wh.t().contiguous()
for lib in ("cublaslt", "cublas"):
    try:
        torch.backends.cuda.preferred_blas_library(lib)
    except Exception as e:  # noqa: BLE001
        print(lib, "unavailable", e)
        continue
    for B in (64, 128, 256):
        h = torch.randn(B, H, device="cuda").to(bf)
        dz = torch.randn(B, 4 * H, device="cuda").to(bf)
        z = torch.empty(B, 4 * H, device="cuda")
        zT = torch.empty(4 * H, B, device="cuda")
        dh = torch.empty(B, H, device="cuda")
        dhT = torch.empty(H, B, device="cuda")
        r = {}
        r["fwd h@Wh"] = timeit(lambda: torch.mm(h, Wh, out_dtype=f32, out=z))
        r["fwd h@WhT^T"] = timeit(lambda: torch.mm(h, WhT.t(), out_dtype=f32, out=z))
        r["fwd (WhT@h^T) -> zT"] = timeit(lambda: torch.mm(WhT, h.t(), out_dtype=f32, out=zT))
        r["fwd bf16 out h@Wh"] = timeit(lambda: torch.mm(h, Wh))
        r["bwd dz@Wh^T"] = timeit(lambda: torch.mm(dz, Wh.t(), out_dtype=f32, out=dh))
        r["bwd dz@WhT"] = timeit(lambda: torch.mm(dz, WhT, out_dtype=f32, out=dh))
        r["bwd (Wh@dz^T) -> dhT"] = timeit(lambda: torch.mm(Wh, dz.t(), out_dtype=f32, out=dhT))
        print(lib, f"B={B}: " + ", ".join(f"{k} {v:.1f}" for k, v in r.items()), flush=True)
