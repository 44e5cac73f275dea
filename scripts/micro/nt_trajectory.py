"""4-layer LSTM-2048, T = 512, B = 64 (BASELINE config 4): per-step loss of a few Adam steps on
the persistent H = 2048 kernels (csrc/lstm_persist_nt.hip) vs the library-GEMM step path, and
the first step's gradient difference -- tells rounding-level divergence of a chaotic start
from a real defect.

  python scripts/micro/nt_trajectory.py [steps]
"""
import os
import sys

import torch

from distributed_char_rnn_amd.engine.optim import TFAdam
from distributed_char_rnn_amd.models.char_rnn import CharRNN
from distributed_char_rnn_amd.models.params import ModelConfig


def run(rec, xs, ys, B, H, L):
    os.environ["DCR_RECURRENCE"] = rec
    cfg = ModelConfig(model="lstm", vocab_size=65, rnn_size=H, num_layers=L)
    m = CharRNN(cfg, device="cuda:0", seed=0)
    opt = TFAdam(m.store, clip=5.0, guard=m.error_word())
    st = m.zero_state(B)
    losses, g0 = [], None
    for x, y in zip(xs, ys):
        loss, st, _ = m.train_step(x, y, st)
        torch.cuda.synchronize()
        m.backend.check_errors()
        if g0 is None:
            g0 = m.store.grad.clone()
        losses.append(loss.item())
        opt.step(2e-3)
    return losses, g0


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    B, T, H, L = 64, 512, 2048, 4
    g = torch.Generator().manual_seed(1)
    xs = [torch.randint(0, 65, (B, T), generator=g, dtype=torch.int32).cuda() for _ in range(n)]
    ys = [torch.randint(0, 65, (B, T), generator=g, dtype=torch.int32).cuda() for _ in range(n)]
    la, ga = run("auto", xs, ys, B, H, L)
    lb, gb = run("library", xs, ys, B, H, L)
    print("step  persistent  library")
    for i, (a, b) in enumerate(zip(la, lb)):
        print(f"{i:4d}  {a:10.5f}  {b:10.5f}")
    print(f"step-0 grad rel diff {((ga - gb).norm() / gb.norm()).item():.3e}")


if __name__ == "__main__":
    main()
