"""Where the step-end weight-layout refresh (one prep_kernel launch, csrc/prep.hip) spends its
time at the headline shape: the whole task table, then each task mode alone, then each task.

  python scripts/micro/prep_tasks.py [--hidden 512 --layers 2 --vocab 65]
"""
import argparse
import collections

import torch

from distributed_char_rnn_amd.models.char_rnn import CharRNN
from distributed_char_rnn_amd.models.params import ModelConfig

MODES = {0: "COPY", 1: "TRANSPOSE", 2: "ZERO", 3: "SUM", 4: "COLSUM", 5: "ONEHOT", 6: "TABLE"}


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
    ap = argparse.ArgumentParser()
    ap.add_argument("--hidden", type=int, default=512)
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--vocab", type=int, default=65)
    a = ap.parse_args()
    cfg = ModelConfig(model="lstm", vocab_size=a.vocab, rnn_size=a.hidden, num_layers=a.layers)
    be = CharRNN(cfg, device=torch.device("cuda"), seed=1)
    be = be.backend
    be._wver = None
    tasks = be._prep()
    print(f"{len(tasks)} tasks")
    print(f"all tasks, one launch: {bench(lambda: be._run_prep(tasks)):8.1f} us")
    by_mode = collections.defaultdict(list)
    for t in tasks:
        by_mode[t[2]].append(t)
    for m, ts in sorted(by_mode.items()):
        print(f"  {MODES[m]:10s} x{len(ts):2d}: {bench(lambda: be._run_prep(ts)):8.1f} us")
    for t in tasks:
        s, d = t[0], t[1]
        print(f"    {MODES[t[2]]:10s} src {tuple(s.shape)} {str(s.dtype)[6:]:8s} stride {s.stride()} "
              f"-> dst {tuple(d.shape)} {str(d.dtype)[6:]:8s} stride {d.stride()}: "
              f"{bench(lambda: be._run_prep([t])):6.1f} us")


if __name__ == "__main__":
    main()
