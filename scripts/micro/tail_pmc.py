"""Counter runs of single tail tasks (csrc/tail.hip): the tables of a real headline step are
captured as in tail_bench.py; TAIL_TASK=<phase>:<index> launches that task alone REPS times
(eagerly, one dispatch each) for rocprofv3 --pmc."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from distributed_char_rnn_amd.engine.native import tail as tailmod  # noqa: E402
from distributed_char_rnn_amd.engine.optim import TFAdam  # noqa: E402
from distributed_char_rnn_amd.models.char_rnn import CharRNN  # noqa: E402
from distributed_char_rnn_amd.models.params import ModelConfig  # noqa: E402

cap = []
orig = tailmod.run


def run(ops, table, phase, ws, err, spin, **kw):
    cap.append((table, phase, ws, err, spin, kw))
    return orig(ops, table, phase, ws, err, spin, **kw)


tailmod.run = run
cfg = ModelConfig(model="lstm", vocab_size=65, rnn_size=512, num_layers=2)
m = CharRNN(cfg, device="cuda:0", seed=0)
opt = TFAdam(m.store, clip=5.0, guard=m.error_word())
m.bind_optimizer(opt)
B, T = 256, 128
x = torch.randint(0, 65, (B, T), dtype=torch.int32, device="cuda")
st = m.zero_state(B)
for _ in range(2):
    cap.clear()
    _, st, _ = m.train_step(x, x, st)
    opt.step(2e-3)
torch.cuda.synchronize()
tailmod.run = orig
ops = m.backend.ops
phase, idx = (int(v) for v in os.environ.get("TAIL_TASK", "0:8").split(":"))
reps = int(os.environ.get("REPS", "20"))
W = tailmod.TAIL_WORDS
table, ph, ws, err, spin, kw = [c for c in cap if c[1] == phase][-1]
t = list(table.words[idx * W:(idx + 1) * W])
t[4], t[5] = -1, 0  # no wait (its producer already ran)
sub = tailmod.TailTable(16)
sub.words, sub.ops, sub.tiles = t, [t[0]], [table.tiles[idx]]
kw = dict(kw, total_out=None, extra=None) if phase == 0 else dict(kw)
print(f"task {phase}:{idx} op {t[0]} {t[1]}x{t[2]} k={t[9]} tiles {table.tiles[idx]}", flush=True)
torch.cuda.synchronize()
for _ in range(reps):
    orig(ops, sub, phase, ws, err, spin, **kw)
torch.cuda.synchronize()
print("done", flush=True)
