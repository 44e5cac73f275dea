"""Diagnostic: bench-like training trajectories (varying batches, carried TBPTT state, TF-Adam)
of the fused per-step path, the library-step path and the fp32 autograd oracle, large H."""
import os
import sys

import torch

from distributed_char_rnn_amd.engine.optim import TFAdam
from distributed_char_rnn_amd.models.char_rnn import CharRNN
from distributed_char_rnn_amd.models.params import ModelConfig
from distributed_char_rnn_amd.models.reference import ReferenceBackend
from distributed_char_rnn_amd.utils.data import synthetic_tokens

H, T, L, STEPS = (int(a) for a in sys.argv[1:5]) if len(sys.argv) > 4 else (2048, 128, 4, 5)
B = 64
toks = torch.from_numpy(synthetic_tokens(16 * B * T + 1, 65, seed=1000)).cuda()
xs, ys = toks[:-1].view(B, 16 * T), toks[1:].view(B, 16 * T)
cfg = ModelConfig(model="lstm", vocab_size=65, rnn_size=H, num_layers=L)
for mode in ("0", "1", "ref"):
    os.environ["DCR_LIBSTEP"] = mode if mode != "ref" else "0"
    m = CharRNN(cfg, device="cuda", seed=1234)
    be = ReferenceBackend(m.store) if mode == "ref" else m.backend
    opt = TFAdam(m.store, clip=5.0)
    st = m.zero_state(B)
    ls = []
    for i in range(STEPS):
        x, y = xs[:, i * T:(i + 1) * T], ys[:, i * T:(i + 1) * T]
        loss, st, _ = be.train_step(x, y, st)
        st = [tuple(s.detach() for s in t) for t in st]
        ls.append(loss.item())
        opt.step(2e-3)
        m.params_changed()
    print(mode, ["%.4f" % v for v in ls], "norm %.3f" % opt.last_norm.item(), flush=True)
