"""Batched prep kernel (csrc/prep.hip) vs plain PyTorch copies / transposes / fills."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_prep_copy_transpose_zero(dcr_ops):
    torch.manual_seed(0)
    big = torch.randn(300, 2048 + 7, device="cuda")
    src_a = big[:, 5:5 + 2048]                 # row-strided view
    src_b = torch.randn(129, 65, device="cuda")
    dst_a = torch.empty(300, 2048, dtype=torch.bfloat16, device="cuda")
    dst_b = torch.zeros(80, 129, dtype=torch.bfloat16, device="cuda")
    dst_c = torch.empty(129, 65, device="cuda")
    pad = torch.full((129, 96), 7.0, dtype=torch.bfloat16, device="cuda")
    cnt = torch.ones(4, 1000, dtype=torch.int32, device="cuda")
    dst_t = torch.empty(2048, 300, dtype=torch.bfloat16, device="cuda")
    dcr_ops.prep([src_a, src_b, src_b, src_b, cnt, src_a],
                 [dst_a, dst_b[:65], dst_c, pad[:, :65], cnt, dst_t],
                 [0, 1, 0, 0, 2, 1])
    torch.cuda.synchronize()
    assert torch.equal(dst_a, src_a.to(torch.bfloat16))
    assert torch.equal(dst_b[:65], src_b.t().to(torch.bfloat16))
    assert torch.count_nonzero(dst_b[65:]) == 0
    assert torch.equal(dst_c, src_b)
    assert torch.equal(pad[:, :65], src_b.to(torch.bfloat16))
    assert torch.all(pad[:, 65:] == 7.0)      # untouched outside the view
    assert torch.count_nonzero(cnt) == 0
    assert torch.equal(dst_t, src_a.t().to(torch.bfloat16))


def test_prep_rejects_bad_shapes(dcr_ops):
    a = torch.randn(4, 8, device="cuda")
    with pytest.raises(RuntimeError):
        dcr_ops.prep([a], [torch.empty(4, 8, dtype=torch.bfloat16, device="cuda")], [1])
