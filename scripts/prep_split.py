"""Time the step-start prep launch (csrc/prep.hip) of the headline model by task subset: the
weight-layout tasks by mode, the layer-0 E·W_x0 + b0 table, everything together.  GPU box."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_char_rnn_amd.models.char_rnn import CharRNN  # noqa: E402
from distributed_char_rnn_amd.models.params import ModelConfig  # noqa: E402

m = CharRNN(ModelConfig(model="lstm", vocab_size=65, rnn_size=512, num_layers=2), device="cuda")
be = m.backend
x = torch.randint(0, 65, (256, 128), device="cuda", dtype=torch.int32)
be.train_step(x, x, m.zero_state(256))
be._wver = None
tasks = be._prep()


def t(sub, n=50):
    for _ in range(3):
        be._run_prep(sub)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        be._run_prep(sub)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


print(f"all {len(tasks)} weight tasks: {t(tasks):.1f} us")
for mode in sorted({tk[2] for tk in tasks}):
    sub = [tk for tk in tasks if tk[2] == mode]
    shapes = [tuple(tk[1].shape) for tk in sub]
    print(f"mode {mode}: {len(sub)} tasks {t(sub):.1f} us  dst shapes {shapes}")
for tk in tasks:
    print(f"  mode {tk[2]} src {tuple(tk[0].shape)} {tk[0].dtype} -> dst {tuple(tk[1].shape)} "
          f"{tk[1].dtype}: {t([tk]):.1f} us")

bufs = be._buffers(256, 128, True)
ids = be._id_tasks(x, x, bufs)
for tk in ids:
    print(f"  id task mode {tk[2]} src {tuple(tk[0].shape)} -> dst {tuple(tk[1].shape)} "
          f"{tk[1].dtype}: {t([tk]):.1f} us")
print(f"id tasks: {t(ids):.1f} us;  weights + ids: {t(tasks + ids):.1f} us")
