"""Large-H step-form selection (engine/native/libstep.py) without a GPU: which time-step form each
direction and batch takes, and what the DCR_DEBUG knobs force."""
from types import SimpleNamespace

from distributed_char_rnn_amd.engine.native.libstep import LibStepMixin
from distributed_char_rnn_amd.engine.native.plan import Knobs


class _Ops:
    @staticmethod
    def big_step_supported(B, H):
        return H % 128 == 0


def _be(H=2048, model="lstm", env=None):
    be = LibStepMixin()
    be.cfg = SimpleNamespace(model=model)
    be.H = H
    be.ops = _Ops()
    be.knobs = Knobs.from_env(env or {})
    return be


def test_default_forms():
    be = _be()
    for B in (1, 64, 128, 1024):
        assert be._lib_step("fwd", B) and be._lib_step("bwd", B)
    assert not be._big_step_ok("fwd", 64)          # library-form forward below B = 96
    assert be._big_step_ok("fwd", 96) and be._big_step_ok("fwd", 1024)
    assert not be._big_step_ok("bwd", 1024)        # library-form BPTT at every batch


def test_knobs_force_forms():
    assert not _be(env={"DCR_DEBUG": "bigstep=0"})._big_step_ok("fwd", 1024)
    forced = _be(env={"DCR_DEBUG": "bigstep=2"})
    assert forced._big_step_ok("fwd", 8) and forced._big_step_ok("bwd", 8)
    assert not _be(H=1536 + 64)._big_step_ok("fwd", 1024)   # H % 128 != 0: library form


def test_small_h_and_other_cells_keep_their_kernels():
    assert not _be(H=1024)._lib_step("fwd", 256)
    assert not _be(model="gru")._lib_step("bwd", 256)
    assert _be(H=512, env={"DCR_RECURRENCE": "library"})._lib_step("fwd", 64)
    assert not _be(env={"DCR_RECURRENCE": "step"})._lib_step("fwd", 64)
