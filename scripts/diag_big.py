"""Diagnostic: large-H persistent forward vs per-step kernels vs fp32 reference at long T."""
import os

import torch

from distributed_char_rnn_amd.models.char_rnn import CharRNN
from distributed_char_rnn_amd.models.params import ModelConfig
from distributed_char_rnn_amd.models.reference import ReferenceBackend

B, H, L = 64, 2048, int(os.environ.get("L", "1"))
for T in (16, 128, 512):
    cfg = ModelConfig(model="lstm", vocab_size=65, rnn_size=H, num_layers=L)
    os.environ["DCR_BIG_FWD"] = "1"
    a = CharRNN(cfg, device="cuda", seed=4)
    os.environ["DCR_BIG_FWD"] = "0"
    b = CharRNN(cfg, device="cuda", seed=4)
    os.environ["DCR_BIG_FWD"] = "1"
    torch.manual_seed(3)
    x = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    st = [tuple(torch.zeros(B, H, device="cuda") for _ in range(2)) for _ in range(L)]
    la, sa = a.backend.eval_loss(x, x, st)
    lb, sb = b.backend.eval_loss(x, x, st)
    ref = ReferenceBackend(a.store)
    lr, sr, _ = ref.train_step(x, x, st) if T <= 128 else (torch.tensor(float("nan")), None, None)
    torch.cuda.synchronize()
    a.backend.check_errors()
    d = max(((p - q).norm() / q.norm()).item() for u, v in zip(sa, sb) for p, q in zip(u, v))
    print(f"T={T} big={la.item():.5f} perstep={lb.item():.5f} ref={lr.item():.5f} state_rel={d:.2e}",
          flush=True)
