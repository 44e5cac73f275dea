"""Text sampling from a trained model (reference: ``Model.sample``, model.py:105-140;
sample.py:27-46).

Semantics kept: zero state; feed ``prime[:-1]`` to warm the state; then ``num`` steps from
``prime[-1]``; ``sampling_type`` 0 = argmax, 1 = weighted pick (inverse CDF via cumsum +
searchsorted of ``rand * sum``), 2 = weighted pick only when the *previous* char is a space,
else argmax.  Sampling is batched (``num_samples`` independent streams) and, on the GPU, the
whole autoregressive loop runs device-side (one fused kernel per generated char, no host sync
until the end) via the native backend's ``sample_sequence``.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ..models.char_rnn import CharRNN


def weighted_pick(weights: np.ndarray, rng: np.random.Generator) -> int:
    t = np.cumsum(weights)
    s = np.sum(weights)
    return int(np.searchsorted(t, rng.random() * s))


def sample(model: CharRNN, chars: Sequence[str], vocab: Dict[str, int], num: int = 200,
           prime: str = "The ", sampling_type: int = 1, seed: Optional[int] = None,
           num_samples: int = 1) -> List[str]:
    if not prime:
        prime = chars[0]
    for ch in prime:
        if ch not in vocab:
            raise KeyError(f"prime character {ch!r} not in vocabulary")
    native = getattr(model.backend, "sample_sequence", None)
    if native is not None and model.device.type == "cuda":
        ids = native([vocab[c] for c in prime], num, sampling_type,
                     seed if seed is not None else int(np.random.SeedSequence().entropy % (1 << 62)),
                     num_samples, vocab.get(" ", -1))
        return [prime + "".join(chars[int(i)] for i in row) for row in ids]

    rng = np.random.default_rng(seed)
    S = num_samples
    state = model.zero_state(S)
    with torch.no_grad():
        for ch in prime[:-1]:
            x = np.full((S, 1), vocab[ch], dtype=np.int32)
            _, state = model.step_logits(x, state)
        outs = [prime for _ in range(S)]
        cur = [prime[-1]] * S
        for _ in range(num):
            x = np.array([[vocab[c]] for c in cur], dtype=np.int32)
            logits, state = model.step_logits(x, state)
            probs = torch.softmax(logits.float(), dim=-1).cpu().numpy()
            nxt = []
            for s in range(S):
                p = probs[s]
                if sampling_type == 0:
                    k = int(np.argmax(p))
                elif sampling_type == 2:
                    k = weighted_pick(p, rng) if cur[s] == " " else int(np.argmax(p))
                else:
                    k = weighted_pick(p, rng)
                k = min(k, len(chars) - 1)
                nxt.append(chars[k])
            cur = nxt
            outs = [o + c for o, c in zip(outs, cur)]
    return outs
