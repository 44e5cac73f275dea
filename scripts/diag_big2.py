"""Diagnostic: multi-step training, large-H persistent forward vs per-step kernels."""
import os

import torch

from distributed_char_rnn_amd.engine.optim import TFAdam
from distributed_char_rnn_amd.models.char_rnn import CharRNN
from distributed_char_rnn_amd.models.params import ModelConfig

B, H, L = 64, 2048, int(os.environ.get("L", "2"))
T = int(os.environ.get("T", "64"))
res = {}
for v in ("1", "0"):
    os.environ["DCR_BIG_FWD"] = v
    cfg = ModelConfig(model="lstm", vocab_size=65, rnn_size=H, num_layers=L)
    m = CharRNN(cfg, device="cuda", seed=4)
    opt = TFAdam(m.store)
    g = torch.Generator().manual_seed(5)
    st = m.zero_state(B)
    losses = []
    for i in range(4):
        x = torch.randint(0, 65, (B, T), generator=g, dtype=torch.int32).cuda()
        y = torch.randint(0, 65, (B, T), generator=g, dtype=torch.int32).cuda()
        loss, st, _ = m.train_step(x, y, st)
        opt.step(2e-3)
        losses.append(round(loss.item(), 5))
    torch.cuda.synchronize()
    m.backend.check_errors()
    res[v] = (losses, m.store.flat.clone())
    print(v, losses, flush=True)
d = ((res["1"][1] - res["0"][1]).norm() / res["0"][1].norm()).item()
print("param rel diff", d)
