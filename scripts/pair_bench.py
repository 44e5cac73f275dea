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


def map_block(bid, nwg_u, ncol):
    """persist_common.h map_block: block -> (unit block, column)."""
    if ncol % 8 == 0:
        xcd, j = bid % 8, bid // 8
        return j % nwg_u, xcd + 8 * (j // nwg_u)
    return bid % nwg_u, bid // nwg_u


def skew(d, H, B, T):
    """Cross-workgroup timing of the wide BPTT from [grid, T+2, 8] s_memrealtime stamps (10 ns):
    slot 1 poll done, 3 payload + MFMA done, 5 / 6 layer l+1 / l hand-off arrival."""
    d = d.cpu().numpy().astype("float64") * 0.01  # us
    grid, ncol, nwg_u = d.shape[0], (B + 15) // 16, H // 32
    cols = np.array([map_block(b, nwg_u, ncol)[1] for b in range(grid)])
    lo, hi = 4, T - 4
    rows = []
    for tau in range(lo, hi):
        for c in range(ncol):
            m = cols == c
            a1, a0 = d[m, tau, 5], d[m, tau, 6]
            last = max(a1.max(), a0.max())
            p_next = d[m, tau + 1, 1]
            p_now = d[m, tau, 1]
            rows.append((a1.max() - a1.min(), a0.max() - a0.min(), np.median(p_next - last),
                         (p_next - last).min(), p_now.max() - p_now.min(),
                         np.median(a1 - p_now), (a1 - p_now).max(), np.median(d[m, tau, 3] - p_now),
                         (d[m, tau, 3] - p_now).max(), np.median(d[m, tau + 1, 0] - d[m, tau, 0])))
    r = np.array(rows).mean(0)
    names = ["arrival skew in a column, layer l+1", "arrival skew in a column, layer l",
             "last arrival -> poll done (median consumer)", "last arrival -> poll done (first)",
             "poll-done skew in a column", "poll done -> own arrival (median)",
             "poll done -> own arrival (slowest)", "poll done -> payload+MFMA done (median)",
             "poll done -> payload+MFMA done (slowest)", "tick period"]
    per_wg = np.mean(d[:, lo:hi, 5] - d[:, lo:hi, 1], axis=1)
    xcd = np.arange(grid) % 8
    by_xcd = [per_wg[xcd == x].mean() for x in range(8)]
    return list(zip(names, r)), by_xcd


RS_PHASES = ["poll", "barrier + partial/operand loads landed", "epilogue -> dZ in LDS",
             "barrier", "products + partial stores issued", "store drain", "arrival"]


def rs_stamps(d, n_ticks):
    """Mean per-tick phase durations (s_memtime ticks) of the reduce-scatter BPTT's workgroup 0
    (RS_STAMP 0..7 of csrc/lstm2_bwd_rs.hip) over the steady ticks."""
    d = d.cpu().numpy().astype("float64").reshape(-1, 8)[:n_ticks]
    lo, hi = 3, n_ticks - 3
    tick = (d[hi, 0] - d[lo, 0]) / (hi - lo)
    return tick, [(RS_PHASES[i], np.mean(d[lo:hi, i + 1] - d[lo:hi, i])) for i in range(7)]


def rs_skew(d, H, B, T):
    """Every workgroup's reduce-scatter BPTT stamps [grid, T+2, 8] (s_memrealtime, 10 ns; RS_STAMP
    0..7): per-workgroup phase means over steady ticks (median / max over workgroups) and the
    hand-off: a column's last arrival (stamp 6) of tick tau-1 -> each member's poll done (1)."""
    d = d.cpu().numpy().astype("float64") * 0.01  # us
    nu, ncol = H // 32, (B + 15) // 16
    lo, hi = 3, T - 3
    rows = []
    live = [bid for bid in range(d.shape[0]) if d[bid, lo, 0] > 0]
    for i, name in enumerate(RS_PHASES):
        v = np.array([np.mean(d[bid, lo:hi, i + 1] - d[bid, lo:hi, i]) for bid in live])
        rows.append((f"{name} (median / max WG)", np.median(v), v.max()))
    # the column of a block under the XCD-grouped map (persist_common.h map_block_grid)
    colof = {}
    for bid in live:
        x, j = bid % 8, bid // 8
        colof[bid] = x + 8 * (j // nu)
    lat, work = [], []
    for c in set(colof.values()):
        members = [bid for bid in live if colof[bid] == c]
        for t in range(lo, hi):
            last = max(d[bid, t - 1, 6] for bid in members)
            lat += [d[bid, t, 1] - last for bid in members]
            work += [d[bid, t, 6] - d[bid, t, 1] for bid in members]
    rows.append(("last arrival -> poll done", np.median(lat), np.max(lat)))
    rows.append(("poll done -> own arrival", np.median(work), np.max(work)))
    rows.append(("tick period", np.median(np.diff(d[live[0], lo:hi, 0])), 0.0))
    return rows


def run(ops, H, T, B, G, want_stamps, reps=5, want_skew=False, drop=False, gather=False,
        xin=False, rs=False):
    dev = "cuda"
    G = int(ops.lstm2_plan(H, B, G))
    if not G:
        return None
    nbg = int(ops.lstm2_nbg(B, G))
    Bp = nbg * 32
    r = lambda *s: (torch.randn(*s, device=dev) * 0.05).to(torch.bfloat16)  # noqa: E731
    W0T, W1T, X1T = r(4 * H, H), r(4 * H, H), r(4 * H, H)
    zx = torch.randn(T, B, 4 * H, device=dev) * 0.1
    ids = None
    if gather:  # the headline's layer 0: a [V, 4H] table gathered by token id
        zx = torch.randn(65, 4 * H, device=dev) * 0.1
        ids = torch.randint(0, 65, (T, B), dtype=torch.int32, device=dev)
    # layer 1's input dropout: [T, B, H/8] keep bits (keep 0.8 per bit)
    xm = (torch.rand(T, B, H, device=dev) < 0.8).view(T, B, H // 8, 8) if drop else None
    if drop:
        w = torch.tensor([1, 2, 4, 8, 16, 32, 64, 128], dtype=torch.int32, device=dev)
        xm = (xm.int() * w).sum(-1).to(torch.uint8).contiguous()
    b1 = torch.zeros(4 * H, device=dev)
    hb0, hb1 = (torch.zeros(T + 1, B, H, dtype=torch.bfloat16, device=dev) for _ in range(2))
    cb0, cb1 = (torch.zeros(T + 1, B, H, device=dev) for _ in range(2))
    g0, g1 = (torch.empty(T, B, 4 * H, dtype=torch.bfloat16, device=dev) for _ in range(2))
    hl0, hl1 = (torch.empty(B, H, device=dev) for _ in range(2))
    hr0, hr1 = (torch.empty(2 * Bp * H, dtype=torch.bfloat16, device=dev) for _ in range(2))
    cnt = torch.zeros(2, 2 * nbg * (T + 1) * 4, dtype=torch.int32, device=dev)  # 16-row columns
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    dfw = torch.zeros(T + 2, G, 8, dtype=torch.int64, device=dev) if want_stamps else None

    # XIN: layer 0's input rows projected in-kernel (the dropout route's default)
    x0 = r(T * B, H) if xin else None
    X0T = r(4 * H, H) if xin else None
    b0 = torch.zeros(4 * H, device=dev) if xin else None

    def fwd(diag=None):
        cnt.zero_()
        ops.lstm2_persist_fwd(W0T, W1T, X1T, zx, ids, b1, hb0, cb0, g0, hl0, hb1, cb1, g1, hl1,
                              cnt[0], cnt[1], err, 1.0, 1 << 22, hr0, hr1, G, None, None, diag,
                              xm, 1.25 if drop else 1.0, b0, x0, X0T)

    Wh0, Wh1, Wx1 = r(H, 4 * H), r(H, 4 * H), r(H, 4 * H)
    dtop = torch.randn(T, B, H, device=dev) * 0.01
    dz0, dz1 = (torch.empty(T, B, 4 * H, dtype=torch.bfloat16, device=dev) for _ in range(2))
    zr0, zr1 = (torch.empty(2 * Bp * 4 * H, dtype=torch.bfloat16, device=dev) for _ in range(2))
    db0, db1 = (torch.empty(2 * nbg // G, 4 * H, device=dev) for _ in range(2))
    dbw = torch.zeros(T + 2, G, 8, dtype=torch.int64, device=dev) if want_stamps else None
    # the reduce-scatter BPTT (csrc/lstm2_bwd_rs.hip): its fp32 partial ring, T + 1 ticks
    rs = rs and not drop and bool(ops.lstm2_bwd_rs_ok(H, B))
    prs = torch.empty(int(ops.lstm2_bwd_rs_ring_floats(H, B)), device=dev) if rs else None

    def bwd(diag=None):
        cnt.zero_()
        ops.lstm2_persist_bwd(Wh0, Wh1, Wx1, dtop, g0, cb0, g1, cb1, dz0, dz1, zr0, zr1, db0, db1,
                              cnt[0], cnt[1], err, 1 << 22, G, diag, xm, 1.25 if drop else 1.0,
                              prs)

    out = {"B": B, "G": G, "grid": (H // 16) * (nbg // G)}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fticks = T + 2 if G == 1 else T + 1  # forward lag: 2 ticks at G = 1, else 1
    bticks = T + 1 if rs else T + 2
    out["rs"] = rs
    for name, fn, ticks in (("fwd", fwd, fticks), ("bwd", bwd, bticks)):
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
    out["cps"] = B * T / ((out["fwd"] * fticks + out["bwd"] * bticks) * 1e-6)
    if want_stamps:
        fwd(dfw)
        bwd(dbw)
        torch.cuda.synchronize()
        out["stamps_fwd"] = stamps(dfw, fticks, G, False)
        out["stamps_bwd"] = rs_stamps(dbw, bticks) if rs else stamps(dbw, T + 2, G, True)
    if want_skew and rs:
        grid = 8 * (H // 32) * -(-((B + 15) // 16) // 8)  # the XCD-padded grid (xcd_grid)
        dall = torch.zeros(grid, T + 2, 8, dtype=torch.int64, device=dev)
        bwd(dall)
        torch.cuda.synchronize()
        out["skew_rs"] = rs_skew(dall, H, B, T)
    if want_skew and G == 1 and ops.lstm2_bwd_wide_ok(H, B) and not rs:
        grid = (H // 32) * ((B + 15) // 16)
        dall = torch.zeros(grid, T + 2, 8, dtype=torch.int64, device=dev)
        bwd(dall)
        torch.cuda.synchronize()
        out["skew_bwd"] = skew(dall, H, B, T)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--H", type=int, default=512)
    ap.add_argument("--T", type=int, default=128)
    ap.add_argument("--B", type=int, nargs="+", default=[256, 512, 1024])
    ap.add_argument("--G", type=int, nargs="+", default=[0])
    ap.add_argument("--stamps", action="store_true")
    ap.add_argument("--drop", action="store_true", help="layer 1 input dropout (DROP kernels)")
    ap.add_argument("--gather", action="store_true", help="layer 0 rows gathered from a table")
    ap.add_argument("--xin", action="store_true", help="layer 0 input projected in-kernel")
    ap.add_argument("--skew", action="store_true", help="every workgroup's hand-off timing (wide BPTT)")
    ap.add_argument("--rs", action="store_true", help="the reduce-scatter BPTT (lstm2_bwd_rs.hip)")
    a = ap.parse_args()
    if a.rs:  # (the C++ launcher's opt-in switch for the reduce-scatter BPTT)
        import os

        os.environ["DCR_DEBUG"] = "bwd_rs=1"
    ops = native.ops()
    for B in a.B:
        for G in a.G:
            o = run(ops, a.H, a.T, B, G, a.stamps, want_skew=a.skew, drop=a.drop, gather=a.gather,
                    xin=a.xin, rs=a.rs)
            if o is None:
                print(f"H={a.H} B={B} G={G}: no co-resident grid", flush=True)
                continue
            print(f"H={a.H} T={a.T} B={B:5d} G={o['G']} grid={o['grid']:4d}  fwd {o['fwd']:6.2f} "
                  f"us/tick  bwd {o['bwd']:6.2f} us/tick  (two launches: {o['cps'] / 1e6:6.1f} M "
                  f"chars/s) err={o['err']} rs={int(o['rs'])}", flush=True)
            for k in ("stamps_fwd", "stamps_bwd"):
                if k in o:
                    tot, parts = o[k]
                    print(f"   {k}: {tot:.0f} s_memtime ticks per tick (workgroup 0)")
                    for n, v in parts:
                        print(f"     {n:<40}{v:8.0f}  {100 * v / tot:5.1f}%")
            if "skew_rs" in o:
                print("   skew_rs (every workgroup, s_memrealtime, us; median, max over workgroups):")
                for n, v, mx in o["skew_rs"]:
                    print(f"     {n:<46}{v:7.2f} {mx:7.2f}")
            if "skew_bwd" in o:
                rows, by_xcd = o["skew_bwd"]
                print("   skew_bwd (every workgroup, s_memrealtime, us, mean over steady ticks):")
                for n, v in rows:
                    print(f"     {n:<46}{v:7.2f}")
                print("     poll done -> layer l+1 arrival by XCD (b % 8): " +
                      " ".join(f"{v:.2f}" for v in by_xcd))


if __name__ == "__main__":
    main()
