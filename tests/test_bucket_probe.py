"""The backward's flush probe (engine/native/backward.py ``bucket_probe``): a readiness report
flushes the deferred gradient sums only when it completes a bucket.  The probe is found on an
on_ready object exposing ``launches_at`` or on the GradSync a bound ``ready`` belongs to; any
other callable gets no probe (flush on every report: safe)."""
import functools

from distributed_char_rnn_amd.engine.native.backward import bucket_probe
from distributed_char_rnn_amd.models.params import ModelConfig, ParamStore
from distributed_char_rnn_amd.parallel.grad_sync import GradSync


def _sync():
    store = ParamStore(ModelConfig(model="lstm", vocab_size=65, rnn_size=128, num_layers=2),
                       device="cpu")
    return store, GradSync(store, 2, bucket_mb=0.25, enabled=True)


def test_probe_from_bound_ready():
    store, sync = _sync()
    assert len(sync.buckets) >= 2
    p = bucket_probe(sync.ready)
    assert p is not None
    lo, hi = sync.buckets[0]
    assert not p(hi - 1) and p(hi) and p(None)


class _Explicit:
    def __init__(self, sync):
        self.sync = sync
        self.calls = []

    def __call__(self, off):
        self.calls.append(off)

    def launches_at(self, upto=None):
        return self.sync.launches_at(upto)


def test_probe_from_object_with_launches_at():
    store, sync = _sync()
    obj = _Explicit(sync)
    p = bucket_probe(obj)
    assert p is not None and p(sync.buckets[0][1]) and not p(0)


def test_wrapped_callables_have_no_probe():
    store, sync = _sync()
    assert bucket_probe(lambda off: sync.ready(off)) is None
    assert bucket_probe(functools.partial(sync.ready)) is None
