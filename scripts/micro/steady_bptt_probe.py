"""Probe of the wide BPTT's steady-tick body (DCR_DEBUG=bwd_steady): per shape and hand-off form,
which gradients differ from the generic-body run (bitwise), and whether they hold NaN.

    python scripts/micro/steady_bptt_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from distributed_char_rnn_amd.models.char_rnn import CharRNN  # noqa: E402
from distributed_char_rnn_amd.models.params import ModelConfig  # noqa: E402


def run(B, T, H, extra, steps=2):
    os.environ["DCR_SPIN_LIMIT"] = str(1 << 20)
    os.environ["DCR_DEBUG"] = "persist_min_t=1" + extra
    cfg = ModelConfig(model="lstm", vocab_size=65, rnn_size=H, num_layers=2)
    m = CharRNN(cfg, device="cuda", seed=21)
    g = torch.Generator().manual_seed(B + T)
    st = m.zero_state(B)
    x = torch.randint(0, 65, (B, T), generator=g, dtype=torch.int32).cuda()
    y = torch.randint(0, 65, (B, T), generator=g, dtype=torch.int32).cuda()
    for _ in range(steps):
        loss, st, _ = m.backend.train_step(x, y, st)
    torch.cuda.synchronize()
    err = None
    try:
        m.backend.check_errors()
    except Exception as e:  # noqa: BLE001
        err = str(e)[:80]
    return m, err


def main():
    # wide_pf 0 / 2 / 4 instantiations spill VGPRs to scratch with the steady body at H = 512
    # (scripts/kernel_resources.py); 3 / 5 / 6 do not
    for B, T, H in [(256, 8, 512), (256, 12, 512), (256, 8, 256)]:
        ref, er = run(B, T, H, ",wide=0")
        for form in ("", ",wide_pf=0", ",wide_pf=2", ",wide_pf=3", ",wide_pf=4", ",wide_pf=5"):
            out = []
            for sd in (1, 0):
                a, ea = run(B, T, H, f",bwd_steady={sd}" + form)
                bad = []
                for s in a.store.specs:
                    ga, gb = a.store.gview(s.name), ref.store.gview(s.name)
                    if s.name.endswith("/bias"):
                        continue  # (summed in another order by the narrow kernel)
                    if not torch.equal(ga, gb):
                        nan = int(torch.isnan(ga).sum())
                        d = (ga - gb).abs()
                        bad.append(f"{s.name.replace('rnnlm/multi_rnn_cell/', '')}: nan={nan} "
                                   f"maxdiff={d.nan_to_num(1e30).max().item():.3g}")
                out.append(f"steady={sd} err={ea}: {'OK' if not bad else '; '.join(bad)}")
            print(f"B={B} T={T} H={H} form='{form}' | " + " | ".join(out), flush=True)


if __name__ == "__main__":
    main()
