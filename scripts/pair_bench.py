"""Two-layer wavefront LSTM kernels (csrc/lstm2_persist.hip) in isolation: per-tick time of the
forward and the BPTT launch over batch sizes and batch groups per workgroup (G), plus the
s_memtime phase split of workgroup 0's group-0 phase (--stamps).

    python scripts/pair_bench.py --H 512 --T 128 --B 256 512 1024 [--G 0 1 2 4] [--stamps]

G = 0 is the plan's choice (the smallest G whose grid fits the chip).  Prints one line per
(B, G): us per tick of each kernel and the implied chars/s of the two launches alone.
"""
import argparse

import numpy as np
import torch

from distributed_char_rnn_amd.ops import native

FWD_TICK = ["tick: poll", "tick: barrier"]
FWD_GROUP = [(7, 3, "start->MFMA done (payload + MFMA)"), (3, 4, "->barrier B"),
             (4, 5, "->epilogue math"), (5, 6, "->drain done (last group)")]
BWD_GROUP = [(0, 1, "start->poll done (group 0)"), (1, 2, "->barrier A"),
             (2, 3, "->MFMA done (payload + MFMA)"), (3, 4, "->barrier B"),
             (4, 5, "->epilogue math"), (5, 6, "->drain done (last group)"),
             (6, 7, "->group end (stash, dz stores)")]


def stamps(d, n_ticks, G, bwd):
    """Mean per-tick phase durations (s_memtime ticks) of workgroup 0 over the steady ticks."""
    d = d.cpu().numpy().astype("float64").reshape(-1, G, 8)[:n_ticks]
    lo, hi = 3, n_ticks - 3
    out = []
    tick = (d[hi, 0, 0 if not bwd else 0] - d[lo, 0, 0]) / (hi - lo)
    if not bwd:
        out.append(("tick start->poll done", np.mean(d[lo:hi, 0, 1] - d[lo:hi, 0, 0])))
        out.append(("poll->barrier A", np.mean(d[lo:hi, 0, 2] - d[lo:hi, 0, 1])))
    for g in range(G):
        rows = FWD_GROUP if not bwd else BWD_GROUP
        for a, b, name in rows:
            if (b == 6 or a == 6) and g != G - 1:
                continue
            if bwd and (a, b) in ((0, 1), (1, 2)) and g > 0:
                if (a, b) == (0, 1):
                    continue
                a = 0
            v = np.mean(d[lo:hi, g, b] - d[lo:hi, g, a])
            out.append((f"g{g} {name}", v))
        if not bwd:
            nxt = d[lo:hi, g + 1, 7] if g + 1 < G else d[lo + 1:hi + 1, 0, 0]
            last = 6 if g == G - 1 else 5
            out.append((f"g{g} ->group end", np.mean(nxt - d[lo:hi, g, last])))
    return tick, out


def run(ops, H, T, B, G, want_stamps, reps=5):
    dev = "cuda"
    G = int(ops.lstm2_plan(H, B, G))
    if not G:
        return None
    nbg = int(ops.lstm2_nbg(B, G))
    Bp = nbg * 32
    r = lambda *s: (torch.randn(*s, device=dev) * 0.05).to(torch.bfloat16)  # noqa: E731
    W0T, W1T, X1T = r(4 * H, H), r(4 * H, H), r(4 * H, H)
    zx = torch.randn(T, B, 4 * H, device=dev) * 0.1
    b1 = torch.zeros(4 * H, device=dev)
    hb0, hb1 = (torch.zeros(T + 1, B, H, dtype=torch.bfloat16, device=dev) for _ in range(2))
    cb0, cb1 = (torch.zeros(T + 1, B, H, device=dev) for _ in range(2))
    g0, g1 = (torch.empty(T, B, 4 * H, dtype=torch.bfloat16, device=dev) for _ in range(2))
    hl0, hl1 = (torch.empty(B, H, device=dev) for _ in range(2))
    hr0, hr1 = (torch.empty(2 * Bp * H, dtype=torch.bfloat16, device=dev) for _ in range(2))
    cnt = torch.zeros(2, nbg * (T + 1) * 4, dtype=torch.int32, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    dfw = torch.zeros(T + 2, G, 8, dtype=torch.int64, device=dev) if want_stamps else None

    def fwd(diag=None):
        cnt.zero_()
        ops.lstm2_persist_fwd(W0T, W1T, X1T, zx, None, b1, hb0, cb0, g0, hl0, hb1, cb1, g1, hl1,
                              cnt[0], cnt[1], err, 1.0, 1 << 22, hr0, hr1, G, None, None, diag)

    Wh0, Wh1, Wx1 = r(H, 4 * H), r(H, 4 * H), r(H, 4 * H)
    dtop = torch.randn(T, B, H, device=dev) * 0.01
    dz0, dz1 = (torch.empty(T, B, 4 * H, dtype=torch.bfloat16, device=dev) for _ in range(2))
    zr0, zr1 = (torch.empty(2 * Bp * 4 * H, dtype=torch.bfloat16, device=dev) for _ in range(2))
    db0, db1 = (torch.empty(2 * nbg // G, 4 * H, device=dev) for _ in range(2))
    dbw = torch.zeros(T + 2, G, 8, dtype=torch.int64, device=dev) if want_stamps else None

    def bwd(diag=None):
        cnt.zero_()
        ops.lstm2_persist_bwd(Wh0, Wh1, Wx1, dtop, g0, cb0, g1, cb1, dz0, dz1, zr0, zr1, db0, db1,
                              cnt[0], cnt[1], err, 1 << 22, G, diag)

    out = {"B": B, "G": G, "grid": (H // 16) * (nbg // G)}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fticks = T + 2 if G == 1 else T + 1  # forward lag: 2 ticks at G = 1, else 1
    for name, fn, ticks in (("fwd", fwd, fticks), ("bwd", bwd, T + 2)):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out[name] = e0.elapsed_time(e1) * 1e3 / reps / ticks
    out["err"] = int(err.item())
    out["cps"] = B * T / ((out["fwd"] * fticks + out["bwd"] * (T + 2)) * 1e-6)
    if want_stamps:
        fwd(dfw)
        bwd(dbw)
        torch.cuda.synchronize()
        out["stamps_fwd"] = stamps(dfw, fticks, G, False)
        out["stamps_bwd"] = stamps(dbw, T + 2, G, True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--H", type=int, default=512)
    ap.add_argument("--T", type=int, default=128)
    ap.add_argument("--B", type=int, nargs="+", default=[256, 512, 1024])
    ap.add_argument("--G", type=int, nargs="+", default=[0])
    ap.add_argument("--stamps", action="store_true")
    a = ap.parse_args()
    ops = native.ops()
    for B in a.B:
        for G in a.G:
            o = run(ops, a.H, a.T, B, G, a.stamps)
            if o is None:
                print(f"H={a.H} B={B} G={G}: no co-resident grid", flush=True)
                continue
            print(f"H={a.H} T={a.T} B={B:5d} G={o['G']} grid={o['grid']:4d}  fwd {o['fwd']:6.2f} "
                  f"us/tick  bwd {o['bwd']:6.2f} us/tick  (two launches: {o['cps'] / 1e6:6.1f} M "
                  f"chars/s) err={o['err']}", flush=True)
            for k in ("stamps_fwd", "stamps_bwd"):
                if k in o:
                    tot, parts = o[k]
                    print(f"   {k}: {tot:.0f} s_memtime ticks per tick (workgroup 0)")
                    for n, v in parts:
                        print(f"     {n:<40}{v:8.0f}  {100 * v / tot:5.1f}%")


if __name__ == "__main__":
    main()
