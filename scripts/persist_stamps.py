"""Diagnostic: s_memtime phase shares of the persistent LSTM forward (workgroup 0)."""

import torch
from distributed_char_rnn_amd.ops import native

ops = native.ops()
import argparse

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=256)
ap.add_argument("--H", type=int, default=512)
ap.add_argument("--mode", default="exclusive", choices=["exclusive", "overlap"],
                help="BPTT variant to stamp")
ap.add_argument("--dew", action="store_true",
                help="layer-0 BPTT variant with the embedding-table gradient fused")
args = ap.parse_args()
EXCL = args.mode == "exclusive"
B, T, H = args.B, 128, args.H
dev = "cuda"
WT = (torch.randn(4 * H, H, device=dev) * 0.05).to(torch.bfloat16)
zx = torch.randn(T, B, 4 * H, device=dev) * 0.1
hbuf = torch.zeros(T + 1, B, H, dtype=torch.bfloat16, device=dev)
cbuf = torch.zeros(T + 1, B, H, device=dev)
gates = torch.empty(T, B, 4 * H, dtype=torch.bfloat16, device=dev)
hl = torch.empty(B, H, device=dev)
cnt = torch.zeros((B // 16 + 1) * (T + 1) * 4, dtype=torch.int32, device=dev)
err = torch.zeros(1, dtype=torch.int32, device=dev)
diag = torch.zeros(T, 8, dtype=torch.int64, device=dev)
# fragment-order hand-off rings as the backend uses them
hring = torch.empty(2 * B * H, dtype=torch.bfloat16, device=dev)
zring = torch.empty(2 * B * 4 * H, dtype=torch.bfloat16, device=dev)
for it in range(5):
    ops.lstm_persist_fwd(WT, zx, None, hbuf, cbuf, gates, hl, cnt, err, 1.0, 1 << 22, hring, diag)
torch.cuda.synchronize()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
ops.lstm_persist_fwd(WT, zx, None, hbuf, cbuf, gates, hl, cnt, err, 1.0, 1 << 22, hring, diag)
ev1.record()
torch.cuda.synchronize()
d = diag.cpu().numpy().astype("float64")
ms = ev0.elapsed_time(ev1)
tot = (d[-1, 0] - d[1, 0]) / (T - 2)
names = ["top->poll done", "poll->barrierA", "barrierA->mfma done", "mfma->barrierB",
         "barrierB->epilogue math", "epi->drain done", "drain->next top"]
import numpy as np
dd = np.diff(np.concatenate([d[1:-1, [0, 1, 2, 3, 4, 5, 6]], d[2:, [0]]], 1), axis=1)
print(f"kernel {ms*1e3/T:.2f} us/step (event); stamps {tot:.0f} ticks/step; err={int(err.item())}")
for n, v in zip(names, dd.mean(0)):
    print(f"  {n:<26}{v:8.0f} ticks  {100*v/tot:5.1f}%")

# ---- backward
W = (torch.randn(H, 4 * H, device=dev) * 0.05).to(torch.bfloat16)
dtop = torch.randn(T, B, H, device=dev) * 0.01
dz = torch.empty(T, B, 4 * H, dtype=torch.bfloat16, device=dev)
dbp = torch.empty(B // 16, 4 * H, device=dev)
DEW = args.dew  # layer-0 variant: embedding-table gradient fused (ids + LDS atomics)
ids = torch.randint(0, 65, (T, B), device=dev, dtype=torch.int32) if DEW else None
dewp = torch.empty(B // 16, 65, 4 * H, device=dev) if DEW else None
for it in range(3):
    ops.lstm_persist_bwd(W, dtop, dz, gates, cbuf, cnt, err, 1 << 22, zring, dbp, ids, dewp, 65,
                         diag, exclusive=EXCL)
torch.cuda.synchronize()
ev0.record()
ops.lstm_persist_bwd(W, dtop, dz, gates, cbuf, cnt, err, 1 << 22, zring, dbp, ids, dewp, 65,
                     diag, exclusive=EXCL)
ev1.record()
torch.cuda.synchronize()
d = diag.cpu().numpy().astype("float64")[::-1]  # reverse time order
ms = ev0.elapsed_time(ev1)
tot = (d[-1, 0] - d[1, 0]) / (T - 2)
dd = np.diff(np.concatenate([d[1:-1, [0, 1, 2, 3, 4, 5, 6]], d[2:, [0]]], 1), axis=1)
print(f"BWD kernel {ms*1e3/T:.2f} us/step (event); stamps {tot:.0f} ticks/step; err={int(err.item())}")
names = ["top->poll done", "poll->barrierA", "barrierA->mfma done", "mfma->barrierB",
         "barrierB->epilogue math", "epi->drain done", "drain->next top"]
for n, v in zip(names, dd.mean(0)):
    print(f"  {n:<26}{v:8.0f} ticks  {100*v/tot:5.1f}%")

# the two-layer wavefront kernels: scripts/pair_bench.py
