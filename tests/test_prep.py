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
                 [0, 1, 0, 0, 2, 1], [])
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
        dcr_ops.prep([a], [torch.empty(4, 8, dtype=torch.bfloat16, device="cuda")], [1], [])


def test_prep_sum_colsum_onehot_table_raw(dcr_ops):
    """The tail-collapse modes: split-K slab sums (vector and scalar paths), bias column sums,
    time-major one-hot rows, the fp32 E·W + b table and raw int32 transposes -- one launch,
    against fp32 PyTorch (sums in the kernel's fixed order are checked to fp32 rounding)."""
    torch.manual_seed(1)
    dev = "cuda"
    part = torch.randn(8, 72, 2048, device=dev)               # float4 path (partial tile)
    part_s = torch.randn(16, 70, 65, device=dev)              # scalar path (65 columns)
    big = torch.zeros(2 * 72, 2048, device=dev)
    out = big[72:]                                           # a row block of a larger buffer
    out_s = torch.empty(70, 65, device=dev)
    dbp = torch.randn(16, 2048, device=dev)
    db = torch.empty(2048, device=dev)
    B, T, VP = 48, 37, 72
    idsrc = torch.randint(0, 65, (B, 3 * T), dtype=torch.int32, device=dev)
    x = idsrc[:, T:2 * T]                                    # row-strided [B, T] view
    oh = torch.full((T * B, VP), 5.0, dtype=torch.bfloat16, device=dev)
    x_tm = torch.empty(T, B, dtype=torch.int32, device=dev)
    E = torch.randn(65, 512, device=dev)
    W = torch.randn(512, 2048, device=dev)
    bias = torch.randn(2048, device=dev)
    tab = torch.empty(65, 2048, device=dev)
    dcr_ops.prep([E, part, part_s, dbp, x, x],
                 [tab, out, out_s, db, oh, x_tm],
                 [6, 3, 3, 4, 5, 1], [W, bias])
    torch.cuda.synchronize()
    torch.testing.assert_close(out, part.sum(0), rtol=1e-6, atol=1e-5)
    assert torch.count_nonzero(big[:72]) == 0
    torch.testing.assert_close(out_s, part_s.sum(0), rtol=1e-6, atol=1e-5)
    torch.testing.assert_close(db, dbp.sum(0), rtol=1e-6, atol=1e-5)
    ref_oh = torch.nn.functional.one_hot(x.t().reshape(-1).long(), VP).to(torch.bfloat16)
    assert torch.equal(oh, ref_oh)  # (72 columns: the 16-B chunk path)
    oh70 = torch.full((T * B, 70), 5.0, dtype=torch.bfloat16, device=dev)  # the scalar path
    dcr_ops.prep([x], [oh70], [5], [])
    torch.cuda.synchronize()
    assert torch.equal(oh70, ref_oh[:, :70])
    assert torch.equal(x_tm, x.t())
    ref_tab = (E.double() @ W.double() + bias.double()).float()
    torch.testing.assert_close(tab, ref_tab, rtol=1e-5, atol=1e-3)
    # bitwise reproducible: the same launch again gives the same bits
    out2 = torch.empty_like(out)
    tab2 = torch.empty_like(tab)
    dcr_ops.prep([E, part], [tab2, out2], [6, 3], [W, bias])
    torch.cuda.synchronize()
    assert torch.equal(out2, out) and torch.equal(tab2, tab)


def test_prep_copy_transpose_vec4(dcr_ops):
    """Aligned tasks take the float4 paths (16-B reads, 4-element writes); partial tiles at the
    right / bottom edges, bf16 and fp32 destinations."""
    torch.manual_seed(1)
    src = torch.randn(300, 2052, device="cuda")          # 300 rows (partial 64-row tile)
    sub = src[:, 4:4 + 1000]                             # 16-B aligned view, 1000 cols
    d_copy = torch.empty(300, 1000, dtype=torch.bfloat16, device="cuda")
    d_copy32 = torch.empty(300, 1000, device="cuda")
    d_t = torch.empty(1000, 300, dtype=torch.bfloat16, device="cuda")
    d_t32 = torch.empty(1000, 300, device="cuda")
    dcr_ops.prep([sub, sub, sub, sub], [d_copy, d_copy32, d_t, d_t32], [0, 0, 1, 1], [])
    torch.cuda.synchronize()
    assert torch.equal(d_copy, sub.to(torch.bfloat16))
    assert torch.equal(d_copy32, sub)
    assert torch.equal(d_t, sub.t().to(torch.bfloat16))
    assert torch.equal(d_t32, sub.t().contiguous())


def test_prep_gather_rows(dcr_ops):
    """GATHER: time-major bf16 embedding rows E[ids[b][t]] (the wide-vocabulary backward's
    X0 operand), from a row-strided batch-major id view, beside a TABLE task that also takes
    its operands from ``extra`` (E for GATHER, then W and bias for TABLE)."""
    torch.manual_seed(2)
    dev = "cuda"
    B, T, V, H = 40, 23, 8192, 512
    idsrc = torch.randint(0, V, (B, 2 * T), dtype=torch.int32, device=dev)
    x = idsrc[:, T:]
    E = torch.randn(V, H, device=dev)
    X0 = torch.full((T * B, H), 3.0, dtype=torch.bfloat16, device=dev)
    E2 = torch.randn(65, 256, device=dev)
    W = torch.randn(256, 1024, device=dev)
    bias = torch.randn(1024, device=dev)
    tab = torch.empty(65, 1024, device=dev)
    dcr_ops.prep([x, E2], [X0, tab], [7, 6], [E, W, bias])
    torch.cuda.synchronize()
    ref = E[x.t().reshape(-1).long()].to(torch.bfloat16)
    assert torch.equal(X0, ref)
    torch.testing.assert_close(tab, (E2.double() @ W.double() + bias.double()).float(),
                               rtol=1e-5, atol=1e-3)
