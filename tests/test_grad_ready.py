"""The gradient-readiness contract of the native backward (engine/native/backward.py).

Data parallelism (parallel/grad_sync.py) launches an RCCL all-reduce of flat-buffer slice
[0, upto) as soon as the backend reports ``ready(upto)``; the collective is ordered after the
work queued at that moment on the calling stream.  So every slice must already be FINAL when
it is reported: a clone queued from inside the callback must equal the gradient after the step.
This holds for every scheduling path (per-step kernels, single-layer persistent BPTT with the
side stream, exclusive scheduling, two-layer wavefronts) and is checked here with a recorder in
place of GradSync (the real collective needs more than one GPU; the driver's multi-GPU bench
runs it).  Reference counterpart: the per-variable gradient push of the replicated graph,
model.py:91-98 under replica_device_setter (train.py:132-133)."""
import pytest
import torch

from distributed_char_rnn_amd.models.char_rnn import CharRNN
from distributed_char_rnn_amd.models.params import ModelConfig

pytestmark = pytest.mark.gpu


class _Recorder:
    def __init__(self, store):
        self.store = store
        self.calls, self.snaps = [], []

    def ready(self, upto):
        lim = self.store.numel if upto is None else upto
        self.calls.append(lim)
        self.snaps.append(self.store.grad[:lim].clone())  # queued on the calling stream


@pytest.mark.parametrize("model,B,T,H,L,mode", [
    ("lstm", 64, 16, 128, 2, ""),           # two-layer wavefronts (pair fwd + pair BPTT)
    ("lstm", 64, 16, 128, 3, ""),           # pair + single-layer persistent
    ("lstm", 64, 16, 128, 4, ""),           # two pairs
    ("lstm", 64, 16, 128, 3, "overlap"),    # side-stream weight GEMMs beside the BPTT
    ("gru", 64, 16, 128, 3, ""),            # GRU persistent
    ("lstm", 32, 4, 64, 2, ""),             # per-step kernels (T below the persistent cutoff)
])
def test_ready_slices_are_final(model, B, T, H, L, mode, monkeypatch):
    monkeypatch.setenv("DCR_SPIN_LIMIT", str(1 << 20))
    if mode:
        monkeypatch.setenv("DCR_MODE", mode)
    cfg = ModelConfig(model=model, vocab_size=65, rnn_size=H, num_layers=L)
    nat = CharRNN(cfg, device="cuda", seed=3)
    x = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    y = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    rec = _Recorder(nat.store)
    nat.store.grad.fill_(float("nan"))  # anything reported before it is written shows up
    nat.train_step(x, y, nat.zero_state(B), rec)
    torch.cuda.synchronize()
    nat.backend.check_errors()
    assert rec.calls, "no readiness reported"
    assert rec.calls == sorted(rec.calls), rec.calls
    assert rec.calls[-1] == nat.store.numel
    g = nat.store.grad
    for s in nat.store.specs:  # (alignment padding between tensors is never written)
        assert torch.isfinite(g[s.offset:s.offset + s.numel]).all(), s.name
    for lim, snap in zip(rec.calls, rec.snaps):
        torch.testing.assert_close(snap, g[:lim], rtol=0, atol=0, equal_nan=True)
