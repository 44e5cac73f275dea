"""Split-K slab count of the hand-written weight-gradient launch (csrc/wgrad.hip
wgrad_splits_tiles): a modelled time -- rounds of one workgroup per CU x tokens per slab, plus
the slab sums -- per tile count.  The headline's 48 + 2 tiles stay one 250-workgroup round at
S = 5; a data-parallel bucket's 2-tile launch fills the chip (S = 32) instead of the 2
workgroups an occupancy score had chosen (639 us on the GPU).  Host-side (no device: 256 CUs)."""
import os

import pytest

LIB = os.path.join(os.path.dirname(__file__), "..", "distributed_char_rnn_amd", "_C.so")


@pytest.mark.skipif(not os.path.exists(LIB), reason="native library not built")
def test_wgrad_split_counts():
    import torch

    torch.ops.load_library(LIB)
    ops = torch.ops.dcr
    plan = {t: int(ops.wgrad_plan_tiles(t, 32768)) for t in (2, 16, 32, 48, 50, 128)}
    assert plan == {2: 32, 16: 16, 32: 8, 48: 5, 50: 5, 128: 2}, plan
    for t, s in plan.items():
        assert t * s <= 256  # one round of one workgroup per CU
    assert int(ops.wgrad_plan_tiles(48, 1024)) == 1  # slabs at least 1024 tokens deep
