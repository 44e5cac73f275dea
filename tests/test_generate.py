"""Single-launch generator (csrc/generate.hip) vs the model's own step path and the oracle.

Reference semantics: Model.sample (model.py:105-140) -- zero state, prime[:-1] warms it, then
each character is drawn from softmax(h·W_s + b_s): argmax (0), inverse-CDF weighted pick (1),
weighted only after a space else argmax (2).  Checks: (a) the generator's logits of every
drawn character equal the native training forward's logits when that forward is fed the same
ids (teacher forcing), (b) every pick follows its rule on the generator's own logits, with the
uniform draw reproduced from the counter hash (common.h uniform01), (c) the final state."""
import numpy as np
import pytest
import torch

from distributed_char_rnn_amd.models.char_rnn import CharRNN
from distributed_char_rnn_amd.models.params import ModelConfig

pytestmark = pytest.mark.gpu

M64 = (1 << 64) - 1


def _mix64(z):
    z = (z + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def uniform01(seed, stream, ctr):
    r = _mix64(seed ^ _mix64((stream * 0x632BE59BD9B4E019 + ctr) & M64))
    return np.float32((r >> 40) * (1.0 / 16777216.0))


@pytest.mark.parametrize("L,H,S,mode", [(2, 128, 1, 0), (2, 512, 1, 1), (3, 256, 4, 2),
                                         (1, 1024, 2, 1)])
def test_generator_matches_step_path(L, H, S, mode):
    V, space = 65, 0
    cfg = ModelConfig(model="lstm", vocab_size=V, rnn_size=H, num_layers=L)
    m = CharRNN(cfg, device="cuda", seed=3)
    be = m.backend
    # larger weights than the init so the draws are not all near-uniform
    with torch.no_grad():
        m.store.flat.mul_(3.0)
    m.params_changed()
    prime, num, seed = [5, 9, 0, 17], 48, 1234
    ids, state, lg = be.generate(prime, num, mode, seed, S, space, want_logits=True)
    ids = torch.tensor(ids)  # [S, num]
    lg = lg.cpu()            # [num, S, V]
    # (a) teacher forcing: the training forward on prime[:-1] + the generated inputs
    seq = torch.cat([torch.tensor(prime).expand(S, -1), ids[:, :-1]], 1).to(torch.int32)
    st = m.zero_state(S)
    ref = []
    for t in range(seq.shape[1]):
        logits, st = m.step_logits(seq[:, t:t + 1].cuda(), st)
        if t >= len(prime) - 1:
            ref.append(logits.float().cpu())
    ref = torch.stack(ref)    # [num, S, V]
    # bf16 h rounding boundaries make the two recurrences drift apart slowly over the
    # characters (the same products, another summation order): tight early, looser late
    scale = ref.abs().max()
    err = (lg - ref).abs().amax(dim=(1, 2)) / scale
    assert err[:8].max() < 2e-3, err
    assert err.max() < 2e-2, err
    # (a') the first 8 characters against the fp32 autograd oracle itself (models/reference.py,
    # the reference graph of model.py:105-140), with fp32 operands and with the bf16-rounded
    # GEMM operands the kernels feed their MFMAs: the generator's error is operand rounding
    from distributed_char_rnn_amd.models.reference import ReferenceBackend, bf16_operands

    oracle = ReferenceBackend(m.store)
    for ctx, tol in ((bf16_operands, 5e-3), (None, 5e-2)):
        st_o = m.zero_state(S)
        ref_o = []
        for t in range(len(prime) - 1 + 8):
            if ctx is None:
                logits, st_o = oracle.step_logits(seq[:, t:t + 1].cuda(), st_o)
            else:
                with ctx():
                    logits, st_o = oracle.step_logits(seq[:, t:t + 1].cuda(), st_o)
            if t >= len(prime) - 1:
                ref_o.append(logits.float().cpu())
        err_o = (lg[:8] - torch.stack(ref_o)).abs().amax(dim=(1, 2)) / scale
        assert err_o.max() < tol, (ctx is not None, err_o)
    # (c) the final state after the last character's input (the generator steps every input
    # once: prime[:-1] + prime[-1] + ids[:-1])
    for (c_g, h_g), (c_r, h_r) in zip(state, st):
        assert (h_g - h_r).abs().max() < 2e-2
        assert (c_g - c_r).abs().max() < 5e-2 * max(1.0, float(c_r.abs().max()))
    # (b) the picks on the generator's own logits
    inputs = torch.cat([torch.tensor(prime[-1:]).expand(S, 1), ids[:, :-1]], 1)
    for t in range(num):
        for s in range(S):
            l64 = lg[t, s].double()
            pick = int(ids[s, t])
            weighted = mode == 1 or (mode == 2 and int(inputs[s, t]) == space)
            if not weighted:
                assert pick == int(torch.argmax(lg[t, s])), (t, s)
                continue
            p = torch.exp(l64 - l64.max())
            cdf = torch.cumsum(p, 0)
            r = float(uniform01(seed, s, t)) * float(cdf[-1])
            lo = float(cdf[pick - 1]) if pick else 0.0
            tol = 1e-4 * float(cdf[-1])
            assert lo - tol <= r <= float(cdf[pick]) + tol, (t, s, pick, r, lo, float(cdf[pick]))


def test_generator_is_sample_sequence_default():
    cfg = ModelConfig(model="lstm", vocab_size=65, rnn_size=128, num_layers=2)
    m = CharRNN(cfg, device="cuda", seed=1)
    a = m.backend.sample_sequence([3, 7, 1], 40, 1, seed=99, num_samples=2, space_id=0)
    b, _, _ = m.backend.generate([3, 7, 1], 40, 1, 99, 2, 0)
    assert a == b and len(a) == 2 and all(len(r) == 40 for r in a)
    c = m.backend.sample_sequence([3, 7, 1], 40, 1, seed=100, num_samples=2, space_id=0)
    assert c != a
