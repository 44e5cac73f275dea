"""Headline softmax_w gradient d W_s = Oᵀ·dlogits (O [32768, 512] bf16, dlogits [32768, 65] bf16,
fp32 [512, 65] out) as split-K batched library GEMMs: dlogits rows of 65 bf16 (130 B, the
current buffer) vs rows padded to 80 (160 B, 16-B aligned); us per call incl. the slab sum.

  python scripts/micro/softmax_w_grad.py
"""
import torch

N, H, V = 32768, 512, 65


def bench(fn, reps=50):
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
    O = torch.randn(N, H, device="cuda").to(torch.bfloat16)
    d65 = (torch.randn(N, V, device="cuda") * 1e-3).to(torch.bfloat16)
    d80 = torch.zeros(N, 80, device="cuda", dtype=torch.bfloat16)
    d80[:, :V] = d65
    out = torch.empty(H, V, device="cuda")
    for S in (1, 4, 8, 16):
        for name, d in (("ld 65", d65), ("ld 80", d80[:, :V])):
            def fn(d=d, S=S):
                if S == 1:
                    torch.mm(O.t(), d, out_dtype=torch.float32, out=out)
                else:
                    part = torch.bmm(O.unflatten(0, (S, N // S)).transpose(1, 2),
                                     d.unflatten(0, (S, N // S)), out_dtype=torch.float32)
                    torch.sum(part, 0, out=out)
            t = bench(fn)
            print(f"S={S:2d} {name}: {t:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
