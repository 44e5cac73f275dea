"""Diagnostic: large-H LSTM gradients of the fused per-step kernels (DCR_LIBSTEP=0) and of the
library-step path (DCR_LIBSTEP=1) against the fp32 autograd oracle, plus the loss after a few
optimizer steps of each."""
import os
import sys

import torch

from distributed_char_rnn_amd.engine.optim import TFAdam
from distributed_char_rnn_amd.models.char_rnn import CharRNN
from distributed_char_rnn_amd.models.params import ModelConfig
from distributed_char_rnn_amd.models.reference import ReferenceBackend

H = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
T = int(sys.argv[2]) if len(sys.argv) > 2 else 16
L = int(sys.argv[3]) if len(sys.argv) > 3 else 2
NOPT = int(sys.argv[4]) if len(sys.argv) > 4 else 4
B = 64


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


torch.manual_seed(0)
x = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
y = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
cfg = ModelConfig(model="lstm", vocab_size=65, rnn_size=H, num_layers=L)
grads, losses = {}, {}
MODES = ("0", "1") if os.environ.get("DIAG_NOREF") else ("0", "1", "ref")
for mode in MODES:
    os.environ["DCR_LIBSTEP"] = mode if mode != "ref" else "0"
    m = CharRNN(cfg, device="cuda", seed=3)
    be = ReferenceBackend(m.store) if mode == "ref" else m.backend
    g0 = torch.Generator(device="cuda").manual_seed(7)
    st = [tuple(torch.randn(B, H, device="cuda", generator=g0) * 0.5 for _ in range(2))
          for _ in range(L)]  # carried TBPTT state (nonzero), as in training
    loss, _, _ = be.train_step(x, y, st)
    torch.cuda.synchronize()
    grads[mode] = m.store.grad.clone()
    opt = TFAdam(m.store, clip=5.0)
    ls = [loss.item()]
    for i in range(NOPT):
        opt.step(2e-3)
        m.params_changed()
        st = [tuple(torch.zeros(B, H, device="cuda") for _ in range(2)) for _ in range(L)]
        loss, _, _ = be.train_step(x, y, st)
        ls.append(loss.item())
    losses[mode] = ls
    print(mode, "losses", ["%.4f" % v for v in ls], flush=True)
if "ref" not in grads:
    for s in m.store.specs:
        r = rel(m.store.view(s.name, grads["1"]), m.store.view(s.name, grads["0"]))
        print(f"lib vs fused {s.name:<48} rel {r:.2e}")
for mode in ("0", "1") if "ref" in grads else ():
    for s in m.store.specs:
        r = rel(m.store.view(s.name, grads[mode]), m.store.view(s.name, grads["ref"]))
        print(f"LIBSTEP={mode} {s.name:<48} rel {r:.2e}")
