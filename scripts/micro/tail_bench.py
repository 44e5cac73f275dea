"""Time the step's tail FINALIZE / ADAM launches (csrc/tail.hip) by task subsets: the tables of a
real headline step are captured from engine/native/tail.run and replayed alone."""
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
ops = m.backend.ops
names = {0: "SUM", 1: "COLSUM", 2: "SUMSQ", 3: "MM", 4: "ADAM"}


def timeit(fn, reps=20):
    """Per-launch time of `reps` launches replayed from one hipGraph (eager calls from Python
    leave the GPU idle between these short launches)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


W = tailmod.TAIL_WORDS
for per, dyn in ((2, False), (1, False), (2, True)):
    os.environ["DCR_DEBUG"] = f"tail_per={per}"
    print(f"== {per} workgroup(s) per CU: grid {ops.tail_grid()}, {'queue' if dyn else 'static'} tiles")
    for table, phase, ws, err, spin, kw in cap:
        kw = dict(kw, dynamic=dyn)
        tasks = [table.words[i * W:(i + 1) * W] for i in range(len(table.ops))]
        desc = [f"{names[t[0]]}[{t[1]}x{t[2]}{' k=' + str(t[9]) if t[0] == 3 else ''}{' S=' + str(t[8]) if t[0] == 0 else ''}{' wait' if t[4] >= 0 else ''}]" for t in tasks]
        print(f"phase {phase}: {len(tasks)} tasks, {sum(table.tiles)} tiles: full {timeit(lambda: orig(ops, table, phase, ws, err, spin, **kw)):.1f} us", flush=True)
        for i, t in enumerate(tasks):
            if t[4] >= 0:
                continue  # a waiting task alone would wait forever
            sub = tailmod.TailTable(16)
            sub.words = list(t)
            sub.ops = [t[0]]
            sub.tiles = [table.tiles[i]]
            kw2 = dict(kw)
            if phase == 0:
                kw2["total_out"] = None
                kw2["extra"] = None
            print(f"   {desc[i]:40s} {table.tiles[i]:5d} tiles  {timeit(lambda: orig(ops, sub, phase, ws, err, spin, **kw2)):8.1f} us", flush=True)
        # the waiting MM tasks without their wait (their producer already ran)
        for i, t in enumerate(tasks):
            if t[4] < 0:
                continue
            w = list(t)
            w[4], w[5] = -1, 0
            sub = tailmod.TailTable(16)
            sub.words, sub.ops, sub.tiles = w, [t[0]], [table.tiles[i]]
            kw2 = dict(kw, total_out=None, extra=None) if phase == 0 else dict(kw)
            print(f"   {desc[i]:40s} {table.tiles[i]:5d} tiles  {timeit(lambda: orig(ops, sub, phase, ws, err, spin, **kw2)):8.1f} us (no wait)", flush=True)
    