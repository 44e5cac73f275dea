"""Diagnostic: s_memtime phase shares of the large-H persistent forward (lstm_big.hip)."""
import numpy as np
import torch

from distributed_char_rnn_amd.ops import native

ops = native.ops()
B, T, H = 64, 256, 2048
dev = "cuda"
WT = (torch.randn(4 * H, H, device=dev) * 0.02).to(torch.bfloat16)
zx = torch.randn(T, B, 4 * H, device=dev) * 0.1
hbuf = torch.zeros(T + 1, B, H, dtype=torch.bfloat16, device=dev)
cbuf = torch.zeros(T + 1, B, H, device=dev)
gates = torch.empty(T, B, 4 * H, dtype=torch.bfloat16, device=dev)
hl = torch.empty(B, H, device=dev)
cnt = torch.zeros((B // 16 + 1) * (T + 1) * 4, dtype=torch.int32, device=dev)
err = torch.zeros(1, dtype=torch.int32, device=dev)
ring = torch.empty(2 * B * H, dtype=torch.bfloat16, device=dev)
diag = torch.zeros(T, 8, dtype=torch.int64, device=dev)
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for dg in (None, diag, None):
    cnt.zero_()
    ev0.record()
    ops.lstm_big_fwd(WT, zx, None, hbuf, cbuf, gates, hl, cnt, err, 1.0, 1 << 22, ring, False, None, dg)
    ev1.record()
    torch.cuda.synchronize()
    print(f"{'diag' if dg is not None else 'plain'}: {ev0.elapsed_time(ev1) * 1e3 / T:.2f} us/step err={int(err.item())}")
d = diag.cpu().numpy().astype("float64")
tot = (d[-1, 0] - d[2, 0]) / (T - 3)
names = ["top->poll done", "poll->barrierA", "barrierA->mfma done", "mfma->barrierB",
         "barrierB->epilogue math", "epi->drain done", "drain->next top"]
dd = np.diff(np.concatenate([d[2:-1, [0, 1, 2, 3, 4, 5, 6]], d[3:, [0]]], 1), axis=1)
print(f"stamps {tot:.0f} ticks/step")
for n, v in zip(names, dd.mean(0)):
    print(f"  {n:<26}{v:8.0f} ticks  {100 * v / tot:5.1f}%")
