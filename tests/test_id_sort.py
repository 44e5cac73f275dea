"""V-bucketed counting sort of the wide-vocabulary segment-sum ids (csrc/embed.hip id_sort)
against torch.sort(stable=True), and the embedding gradient it feeds against the unsorted
atomic segment sum (the reference densifies the embedding IndexedSlices with an
UnsortedSegmentSum, model.py:55 / tf.gradients)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("N,V,skew", [(32768, 8192, True), (32768, 8192, False), (1000, 97, True),
                                      (5000, 16384, False), (1, 3, False), (1024, 1, False)])
def test_id_sort_is_stable_sort(N, V, skew, dcr_ops):
    g = torch.Generator(device="cuda").manual_seed(N + V)
    if skew:  # unigram-skewed like the synthetic text: a few very frequent ids
        p = torch.rand(V, device="cuda", generator=g) ** 8
        ids = torch.multinomial(p, N, replacement=True, generator=g).int()
    else:
        ids = torch.randint(0, V, (N,), device="cuda", dtype=torch.int32, generator=g)
    nws = dcr_ops.id_sort_workspace(N, V)
    assert nws > 0
    ws = torch.empty(nws, dtype=torch.int32, device="cuda")
    sid = torch.full((N,), -1, dtype=torch.int32, device="cuda")
    perm = torch.full((N,), -1, dtype=torch.int32, device="cuda")
    dcr_ops.id_sort(ids, V, ws, sid, perm)
    ref, rperm = torch.sort(ids, stable=True)
    assert torch.equal(sid, ref)
    assert torch.equal(perm, rperm.int())
    assert dcr_ops.id_sort_workspace(N, 16385) == 0  # beyond the LDS histogram: library sort


def test_sorted_segsum_matches_unsorted(dcr_ops):
    N, V, W = 4096, 8192, 512
    g = torch.Generator(device="cuda").manual_seed(2)
    p = torch.rand(V, device="cuda", generator=g) ** 8
    ids = torch.multinomial(p, N, replacement=True, generator=g).int()
    X = torch.randn(N, W, device="cuda", generator=g)
    ws = torch.empty(dcr_ops.id_sort_workspace(N, V), dtype=torch.int32, device="cuda")
    sid, perm = torch.empty_like(ids), torch.empty_like(ids)
    dcr_ops.id_sort(ids, V, ws, sid, perm)
    out = torch.empty(V, W, device="cuda")
    seg_ws = torch.empty(max(1, dcr_ops.segsum_workspace(N, W, V)), device="cuda")
    dcr_ops.segsum(X, sid, V, out, seg_ws, False, perm)
    ref = torch.zeros(V, W, device="cuda").index_add_(0, ids.long(), X)
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-4)


def test_id_sort_clears_the_segsum_output(dcr_ops):
    """The sort's first launch clears the atomic segment sum's output on the side (the
    wide-vocabulary step then runs no fill launch): the accumulating segment sum into the
    cleared buffer equals the plain one; a buffer that is not 16-B aligned is left alone."""
    N, V, W = 4096, 8192, 512
    g = torch.Generator(device="cuda").manual_seed(3)
    ids = torch.randint(0, V, (N,), device="cuda", dtype=torch.int32, generator=g)
    X = torch.randn(N, W, device="cuda", generator=g)
    ws = torch.empty(dcr_ops.id_sort_workspace(N, V), dtype=torch.int32, device="cuda")
    sid, perm = torch.empty_like(ids), torch.empty_like(ids)
    out = torch.full((V, W), 7.0, device="cuda")
    assert dcr_ops.id_sort(ids, V, ws, sid, perm, out)
    assert not bool(out.any())
    seg_ws = torch.empty(max(1, dcr_ops.segsum_workspace(N, W, V)), device="cuda")
    dcr_ops.segsum(X, sid, V, out, seg_ws, True, perm)
    ref = torch.zeros(V, W, device="cuda").index_add_(0, ids.long(), X)
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-4)
    odd = torch.full((V * W + 1,), 7.0, device="cuda")[1:]  # 4-B but not 16-B aligned
    assert not dcr_ops.id_sort(ids, V, ws, sid, perm, odd)
    assert bool((odd == 7.0).all())
