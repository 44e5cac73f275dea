"""Hand-written token-reduction weight-gradient GEMM (csrc/wgrad.hip) vs an fp32 PyTorch
reference of the same product: part[p][s] = A_p[chunk s]ᵀ · B_p[chunk s]."""
import pytest
import torch

from distributed_char_rnn_amd.ops import native

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shapes,K,S", [([(256, 256)], 64, 1), ([(512, 2048)] * 3, 4096, 4),
                                        ([(256, 512), (512, 256)], 3200, 3),
                                        ([(1024, 3072)], 2048, 2),
                                        ([(1024, 2048), (512, 2048)], 8192, 5)])
def test_wgrad_matches_fp32_reference(shapes, K, S):
    """One launch over problems of different shapes (the step's layer-1 and layer-0 weight
    gradients), every (problem, slab) against fp32 PyTorch."""
    ops = native.ops()
    g = torch.Generator(device="cuda").manual_seed(0)
    As, Bs, parts = [], [], []
    for p, (M, N) in enumerate(shapes):
        # A as a strided view (row stride > M, like [h0_t | h1_{t-1}] halves)
        Abuf = torch.randn(K, 2 * M, device="cuda", generator=g).to(torch.bfloat16)
        As.append(Abuf[:, :M] if p % 2 == 0 else Abuf[:, M:])
        Bs.append(torch.randn(K, N, device="cuda", generator=g).to(torch.bfloat16))
        parts.append(torch.full((S, M, N), float("nan"), device="cuda"))
    ops.wgrad(As, Bs, parts)
    torch.cuda.synchronize()
    ks = 32  # csrc/wgrad.hip kWgK
    steps = K // ks
    for p in range(len(shapes)):
        for s in range(S):
            k0, k1 = steps * s // S * ks, steps * (s + 1) // S * ks
            ref = As[p][k0:k1].float().t() @ Bs[p][k0:k1].float()
            err = ((parts[p][s] - ref).norm() / ref.norm()).item()
            assert err < 1e-5, (p, s, err)


def test_wgrad_plan():
    ops = native.ops()
    assert ops.wgrad_plan(3, 512, 2048, 32768) >= 1
    assert ops.wgrad_plan(1, 128, 512, 32768) == 0   # M not a multiple of 256
    assert ops.wgrad_plan(1, 512, 2048, 100) == 0    # K not a multiple of 32


def test_training_step_with_wgrad_matches_library(monkeypatch):
    """DCR_DEBUG=wgrad=1 routes the step's weight gradients through the wgrad kernel (deferred
    to the SumQueue flush): the gradients match the library split-K path to summation order."""
    from distributed_char_rnn_amd.models.char_rnn import CharRNN
    from distributed_char_rnn_amd.models.params import ModelConfig

    cfg = ModelConfig(model="lstm", vocab_size=65, rnn_size=512, num_layers=2)
    B, T = 256, 16
    x = torch.randint(0, 65, (B, T), device="cuda", dtype=torch.int32)
    grads = []
    for flag in ("wgrad=0", "wgrad=1"):
        monkeypatch.setenv("DCR_DEBUG", "persist_min_t=1," + flag)
        m = CharRNN(cfg, device="cuda", seed=4)
        m.backend.train_step(x, x, m.zero_state(B))
        torch.cuda.synchronize()
        grads.append(m.store.grad.clone())
    err = ((grads[1] - grads[0]).norm() / grads[0].norm()).item()
    assert err < 1e-4, err
