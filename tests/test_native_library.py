"""The in-tree native library loads on the CPU host and registers every op schema (a schema
the TorchScript parser rejects would otherwise surface only on the GPU box, at first import)."""
import os

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "distributed_char_rnn_amd", "_C.so")


@pytest.mark.skipif(not os.path.exists(LIB), reason="native library not built")
def test_library_loads_and_registers_ops():
    torch.ops.load_library(LIB)
    ops = torch.ops.dcr
    for name in ("prep", "sumsq", "adam_clip", "head", "lstm2_persist_fwd",
                 "lstm2_persist_bwd", "segsum"):
        assert hasattr(ops, name), name
    assert int(ops.prep_max_tasks()) >= 16
    assert "ticket" in str(ops.sumsq.default._schema)
