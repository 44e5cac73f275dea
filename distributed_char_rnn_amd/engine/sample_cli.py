"""``sample.py`` implementation (reference: sample.py:13-49).

Loads ``config.pkl`` + ``chars_vocab.pkl`` (restricted unpickler), rebuilds the model for
inference, restores the latest checkpoint named in ``<save_dir>/checkpoint`` and prints the
sampled text.  Differences: the text is printed as text (the reference printed the py3
``b'...'`` bytes repr, A-15; ``--bytes`` restores that), and a missing checkpoint is an error
instead of silently printing nothing (sample.py:43).
"""
from __future__ import annotations

import os
import sys

import torch

from ..models.char_rnn import CharRNN
from ..models.params import ModelConfig
from ..utils import checkpoint as ckpt
from ..utils import safe_pickle
from ..utils.config import sample_parser
from .sampler import sample


def load_for_inference(save_dir: str, device="auto"):
    saved = safe_pickle.load(os.path.join(save_dir, "config.pkl"))
    chars, vocab = safe_pickle.load(os.path.join(save_dir, "chars_vocab.pkl"))
    if device == "auto":
        device = "cuda" if torch.cuda.is_available() else "cpu"
    cfg = ModelConfig(model=saved.model, vocab_size=saved.vocab_size, rnn_size=saved.rnn_size,
                      num_layers=saved.num_layers)
    model = CharRNN(cfg, device=device, seed=0)
    prefix = ckpt.latest_checkpoint(save_dir)
    if prefix is None:
        raise FileNotFoundError(f"no checkpoint found in {save_dir}")
    sd = ckpt.Saver.restore(prefix)
    model.store.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()
                                 if k in model.store.by_name})
    model.params_changed()
    return model, tuple(chars), dict(vocab), saved


def main(argv=None) -> int:
    args = sample_parser().parse_args(argv)
    model, chars, vocab, _ = load_for_inference(args.save_dir, args.device)
    prime = args.prime or chars[0]  # sample.py:36-37
    outs = sample(model, chars, vocab, args.n, prime, args.sample, seed=args.seed,
                  num_samples=args.num_samples)
    for o in outs:
        print(o.encode("utf-8") if args.bytes else o)
    return 0


if __name__ == "__main__":
    sys.exit(main())
