"""SumQueue (engine/native/gemm.py) deferral logic on the CPU with a stand-in op table: weight
GEMMs the wgrad kernel covers are grouped by token count into one launch (at most 4 problems), each
problem's split-K slabs become one SUM task of the flush, everything else runs immediately."""
import torch

from distributed_char_rnn_amd.engine.native import gemm


class FakeOps:
    """Records the calls; computes the slabs with torch so the sums can be checked."""

    def __init__(self):
        self.wgrad_calls, self.prep_calls = [], []

    def wgrad_plan(self, np_, M, N, K):
        return 0 if (M % 256 or N % 256 or K % 32) else 2

    def wgrad_plan_tiles(self, tiles, K):
        return 2

    def wgrad(self, As, Bs, parts):
        self.wgrad_calls.append(len(As))
        for part, a, b in zip(parts, As, Bs):
            S, K = part.shape[0], a.shape[0]
            for s in range(S):
                k0, k1 = K * s // S, K * (s + 1) // S
                part[s] = a[k0:k1].float().t() @ b[k0:k1].float()

    def prep_max_tasks(self):
        return 64

    def prep(self, src, dst, mode, extra):
        self.prep_calls.append(list(mode))
        for s_, d, m in zip(src, dst, mode):
            assert m == gemm.SumQueue.SUM
            d.copy_(s_.sum(0))


def _wgrad_ok_cpu(self, a, b, out):
    # the real check requires CUDA tensors; the deferral logic is what is tested here
    K, M = a.shape
    return (self.wgrad and out is not None and int(self.ops.wgrad_plan(1, M, b.shape[1], K)) > 0)


def test_sum_queue_groups_wgrad_problems(monkeypatch):
    monkeypatch.setattr(gemm.SumQueue, "wgrad_ok", _wgrad_ok_cpu)
    ops = FakeOps()
    q = gemm.SumQueue(ops, wgrad=True)
    g = torch.Generator().manual_seed(0)
    K = 128
    A = [torch.randn(K, 256, generator=g).to(torch.bfloat16) for _ in range(3)]
    Bm = [torch.randn(K, 512, generator=g).to(torch.bfloat16) for _ in range(3)]
    outs = [torch.zeros(256, 512) for _ in range(3)]
    for a, b, o in zip(A, Bm, outs):
        assert gemm.mm_tn(a, b, o, q=q) is o
    assert ops.wgrad_calls == [] and len(q.gemms) == 3   # deferred, nothing launched yet
    q.flush()
    assert ops.wgrad_calls == [3]                      # one launch for the three GEMMs
    assert ops.prep_calls == [[gemm.SumQueue.SUM] * 3]
    for a, b, o in zip(A, Bm, outs):
        ref = a.float().t() @ b.float()
        assert torch.allclose(o, ref, rtol=1e-5, atol=1e-4)
    assert q.gemms == [] and q.tasks == []


def test_sum_queue_without_wgrad_keeps_library_path():
    q = gemm.SumQueue(FakeOps(), wgrad=False)
    a = torch.randn(64, 256).to(torch.bfloat16)
    b = torch.randn(64, 256).to(torch.bfloat16)
    assert not q.wgrad_ok(a, b, torch.empty(256, 256))   # default: library split-K GEMMs
    q2 = gemm.SumQueue(FakeOps(), wgrad=True)
    assert not q2.wgrad_ok(a, b, torch.empty(256, 256))  # CPU tensors never take the kernel


def test_split_k_short_reductions():
    assert gemm.split_k(2500, 128, 512) == 4      # reference default: 2500 tokens
    assert gemm.split_k(1000, 128, 512) == 1      # too short to split
    assert gemm.split_k(32768, 512, 2048) == 8    # headline weight gradients
    assert gemm.split_k(32768, 4096, 4096) == 1   # enough output tiles already
