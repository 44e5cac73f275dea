"""Numerics of the fused global-norm clip + TF-Adam kernel (csrc/optim.hip) against a plain
PyTorch fp32 reference of TF 1.x `clip_by_global_norm` + `AdamOptimizer` (model.py:91-98)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(p, g, m, v, lr, b1, b2, eps, clip, t):
    norm = torch.sqrt((g.double() ** 2).sum()).float()
    s = clip / max(norm.item(), clip) if clip > 0 else 1.0
    g = g * s
    lr_t = lr * math.sqrt(1 - b2 ** t) / (1 - b1 ** t)
    m = b1 * m + (1 - b1) * g
    v = b2 * v + (1 - b2) * g * g
    p = p - lr_t * m / (torch.sqrt(v) + eps)
    return p, m, v, norm


@pytest.mark.parametrize("n", [1, 7, 4096, 1 << 20, 4265025])
@pytest.mark.parametrize("clip", [5.0, 0.01, 0.0])
def test_adam_clip_matches_reference(dcr_ops, n, clip):
    torch.manual_seed(0)
    dev = "cuda"
    p = torch.randn(n, device=dev)
    g = torch.randn(n, device=dev) * 0.1
    m = torch.randn(n, device=dev) * 0.01
    v = torch.rand(n, device=dev) * 0.01
    pbf = torch.empty(n, device=dev, dtype=torch.bfloat16)
    parts = torch.empty(dcr_ops.opt_num_partials(n), device=dev)
    norm = torch.empty(1, device=dev)
    lr, b1, b2, eps, t = 2e-3, 0.9, 0.999, 1e-8, 3
    rp, rm, rv, rn = _ref(p.clone(), g.clone(), m.clone(), v.clone(), lr, b1, b2, eps, clip, t)
    lr_t = lr * math.sqrt(1 - b2 ** t) / (1 - b1 ** t)
    dcr_ops.adam_clip(p, g, m, v, pbf, parts, norm, lr_t, b1, b2, eps, clip)
    torch.cuda.synchronize()
    assert torch.allclose(norm.cpu(), rn.cpu(), rtol=1e-5)
    torch.testing.assert_close(m, rm, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(v, rv, rtol=1e-5, atol=1e-9)
    torch.testing.assert_close(p, rp, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(pbf.float(), p.to(torch.bfloat16).float(), rtol=0, atol=0)


@pytest.mark.parametrize("n,n_norm", [(4096, 4096), (100000, 60000), (4265088, 4265024), (5000, 0)])
def test_adam_clip_partial_norm_plus_extra(dcr_ops, n, n_norm):
    """norm = sqrt(sum(g[:n_norm]^2) + extra) (TF IndexedSlices embedding term); the update
    still covers all n elements."""
    torch.manual_seed(2)
    dev = "cuda"
    p = torch.randn(n, device=dev)
    g = torch.randn(n, device=dev) * 0.1
    m = torch.zeros(n, device=dev)
    v = torch.zeros(n, device=dev)
    extra = torch.tensor([3.25], device=dev)
    parts = torch.empty(dcr_ops.opt_num_partials(n), device=dev)
    norm = torch.empty(1, device=dev)
    want = math.sqrt(float((g[:n_norm].double() ** 2).sum()) + 3.25)
    s = 1.0 / max(want, 1.0)
    lr, b1, b2, eps = 1e-3, 0.9, 0.999, 1e-8
    gs = g * s
    rm = (1 - b1) * gs
    rv = (1 - b2) * gs * gs
    rp = p - lr * rm / (rv.sqrt() + eps)
    dcr_ops.adam_clip(p, g, m, v, None, parts, norm, lr, b1, b2, eps, 1.0, 1.0, n_norm, extra)
    torch.cuda.synchronize()
    assert norm.item() == pytest.approx(want, rel=1e-5)
    torch.testing.assert_close(m, rm, rtol=1e-5, atol=1e-9)
    torch.testing.assert_close(p, rp, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n", [3, 4097, 32768 * 512])
def test_sumsq_kernel(dcr_ops, dtype, n):
    torch.manual_seed(3)
    x = (torch.randn(n, device="cuda") * 0.01).to(dtype)
    parts = torch.empty(dcr_ops.opt_num_partials(n), device="cuda")
    out = torch.empty(1, device="cuda")
    dcr_ops.sumsq(x, parts, out)
    torch.cuda.synchronize()
    assert out.item() == pytest.approx(float((x.double() ** 2).sum()), rel=1e-5)
    # one-launch form (last block sums the partials): same value, bitwise reproducible, ticket
    # left at zero, reusable launch after launch
    tick = torch.zeros(1, dtype=torch.int32, device="cuda")
    first = None
    for _ in range(3):
        out1 = torch.empty(1, device="cuda")
        dcr_ops.sumsq(x, parts, out1, tick)
        torch.cuda.synchronize()
        assert out1.item() == pytest.approx(float((x.double() ** 2).sum()), rel=1e-5)
        first = out1 if first is None else first
        assert torch.equal(out1, first)
        assert int(tick.item()) == 0
    # extra term + error word (parallel/zero.py: one launch in front of the step's all-reduce)
    extra = torch.tensor([0.25], device="cuda")
    guard = torch.tensor([9], dtype=torch.int32, device="cuda")
    out2 = torch.full((2,), -1.0, device="cuda")
    dcr_ops.sumsq(x, parts, out2, tick, extra, guard)
    torch.cuda.synchronize()
    assert out2[0].item() == pytest.approx(first.item() + 0.25, rel=1e-6)
    assert out2[1].item() == 9.0 and int(tick.item()) == 0


@pytest.mark.parametrize("world", [2, 8])
def test_adam_clip_folds_data_parallel_average(dcr_ops, world):
    """gscale = 1/world on the all-reduced SUM == the kernel on the averaged gradient."""
    torch.manual_seed(1)
    n, dev = 100003, "cuda"
    p = torch.randn(n, device=dev)
    gsum = torch.randn(n, device=dev) * world
    m = torch.zeros(n, device=dev)
    v = torch.zeros(n, device=dev)
    parts = torch.empty(dcr_ops.opt_num_partials(n), device=dev)
    na, nb = torch.empty(1, device=dev), torch.empty(1, device=dev)
    pa, ma, va = p.clone(), m.clone(), v.clone()
    dcr_ops.adam_clip(pa, gsum / world, ma, va, None, parts, na, 1e-3, 0.9, 0.999, 1e-8, 5.0)
    dcr_ops.adam_clip(p, gsum, m, v, None, parts, nb, 1e-3, 0.9, 0.999, 1e-8, 5.0, 1.0 / world)
    torch.cuda.synchronize()
    torch.testing.assert_close(nb, na, rtol=1e-5, atol=0)
    torch.testing.assert_close(p, pa, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(m, ma, rtol=1e-5, atol=1e-7)
