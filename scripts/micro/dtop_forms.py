"""Wide-vocabulary head backward GEMM forms (BASELINE config 5, V = 8192, H = 512, N = 32768):
dtop[N, H] = dlogits[N, V] · softmax_wᵀ, fp32 output, with the weight as the transposed view of
the [H, V] bf16 layout (current) vs the contiguous [V, H] copy the wide head already keeps.

  python scripts/micro/dtop_forms.py
"""
import torch


def bench(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    N, V, H = 32768, 8192, 512
    dlog = (torch.randn(N, V, device="cuda") * 1e-3).to(torch.bfloat16)
    Ws = torch.randn(H, V, device="cuda").to(torch.bfloat16)     # [H, V] (hd["Ws"])
    WsT = Ws.t().contiguous()                                      # [V, H] (hd["WsTw"])
    out = torch.empty(N, H, device="cuda")
    fl = 2.0 * N * V * H
    dlogT = dlog.t().contiguous()                                  # [V, N]: a vocab-major dlogits
    forms = {
        "mm(dlog, Ws.t())  [TN view]": lambda: torch.mm(dlog, Ws.t(), out_dtype=torch.float32, out=out),
        "mm(dlog, WsT)     [contig] ": lambda: torch.mm(dlog, WsT, out_dtype=torch.float32, out=out),
        "(Ws @ dlog.t()).t() [NT]   ": lambda: torch.mm(Ws, dlog.t(), out_dtype=torch.float32),
        "mm(dlogT.t(), Ws.t())      ": lambda: torch.mm(dlogT.t(), Ws.t(), out_dtype=torch.float32, out=out),
        "mm(dlogT.t(), WsT)         ": lambda: torch.mm(dlogT.t(), WsT, out_dtype=torch.float32, out=out),
        "(Ws @ dlogT).t()           ": lambda: torch.mm(Ws, dlogT, out_dtype=torch.float32),
    }
    ref = None
    for name, fn in forms.items():
        t = bench(fn)
        r = fn()
        r = out if r is None or r.data_ptr() == out.data_ptr() else r.t()
        if ref is None:
            ref = r.clone()
        err = ((r - ref).abs().max() / ref.abs().max()).item()
        print(f"{name}: {t:8.1f} us  {fl / t / 1e6:7.1f} TF/s  max rel diff {err:.2e}", flush=True)
    # d softmax_w [H, V] = Oᵀ · dlogits (K = N tokens), split-K slabs as engine/native/gemm.py
    O = (torch.randn(N, H, device="cuda") * 0.5).to(torch.bfloat16)
    for S in (1, 4, 8):
        def dws(S=S, src=dlog):
            if S == 1:
                return torch.mm(O.t(), src, out_dtype=torch.float32)
            part = torch.bmm(O.unflatten(0, (S, N // S)).transpose(1, 2),
                             src.unflatten(0, (S, N // S)), out_dtype=torch.float32)
            return part.sum(0)
        t = bench(dws)
        print(f"dWs = O^T dlog, split {S}: {t:8.1f} us  {fl / t / 1e6:7.1f} TF/s", flush=True)
    t = bench(lambda: torch.mm(dlogT, O, out_dtype=torch.float32))
    print(f"dWs^T = dlogT @ O (vocab-major dlogits): {t:8.1f} us  {fl / t / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
