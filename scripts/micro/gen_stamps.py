"""Phase timing of the single-launch generator (csrc/generate.hip): the 100-MHz stamps of
characters 8..15 in the first and last workgroup, printed as per-phase deltas in us."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from distributed_char_rnn_amd.models.char_rnn import CharRNN  # noqa: E402
from distributed_char_rnn_amd.models.params import ModelConfig  # noqa: E402

S = int(os.environ.get("S", "1"))
m = CharRNN(ModelConfig(model="lstm", vocab_size=65, rnn_size=512, num_layers=2), device="cuda", seed=0)
be = m.backend
be.gen_stamps = torch.zeros(256, dtype=torch.int64, device="cuda")
for mode in (0, 1):
    be.generate([1, 2, 3], 40, mode, 7, S, 0)
    raw = be.gen_stamps.cpu().view(2, 8, 16).double()
    st = raw / 100.0  # us
    mhz = (raw[0, :, 12] - raw[0, :, 11]) / (raw[0, :, 13] - raw[0, :, 0]) * 100.0
    print("shader clock over [char start, head end] (MHz):", [round(float(x)) for x in mhz])
    names = {1: "gemv0", 2: "cell0", 3: "gath0", 4: "bar0", 5: "gemv1", 6: "cell1", 7: "gath1",
             8: "bar1", 13: "head", 14: "pick"}
    for wg in range(2):
        rows = []
        for c in range(7):
            t = st[wg, c]
            prev, out = t[0], []
            for p in (1, 2, 3, 4, 5, 6, 7, 8, 13, 14):
                out.append(f"{names[p]} {float(t[p] - prev):5.2f}")
                prev = t[p]
            out.append(f"next {float(st[wg, c + 1, 0] - t[14]):5.2f}")
            out.append(f"| char {float(st[wg, c + 1, 0] - t[0]):5.2f}")
            rows.append("  ".join(out))
        print(f"mode {mode} S {S} workgroup {'first' if wg == 0 else 'last'}:")
        print("\n".join(rows))
