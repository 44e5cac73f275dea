"""engine/trainer.py _device_batches: the epoch's batches uploaded once as [nb, B, T] int32."""
import numpy as np
import pytest
import torch

from distributed_char_rnn_amd.engine import trainer


class _Loader:
    def __init__(self, nb=5, B=3, T=4):
        r = np.random.default_rng(0)
        self.x_batches = [r.integers(0, 65, (B, T)) for _ in range(nb)]
        self.y_batches = [r.integers(0, 65, (B, T)) for _ in range(nb)]


def test_device_batches_off_on_cpu():
    assert trainer._device_batches(_Loader(), 5, torch.device("cpu")) is None


def test_device_batches_size_cap(monkeypatch):
    monkeypatch.setattr(trainer, "DEVICE_BATCHES_MAX_BYTES", 16)
    assert trainer._device_batches(_Loader(), 5, torch.device("cuda")) is None


@pytest.mark.gpu
def test_device_batches_match_loader():
    ld = _Loader()
    xs, ys = trainer._device_batches(ld, 4, torch.device("cuda"))
    assert xs.shape == (4, 3, 4) and xs.dtype == torch.int32 and xs.is_cuda
    for b in range(4):
        assert np.array_equal(xs[b].cpu().numpy(), ld.x_batches[b])
        assert np.array_equal(ys[b].cpu().numpy(), ld.y_batches[b])
