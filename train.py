#!/usr/bin/env python
"""Train a character-level RNN LM (reference entry point: train.py).  Same flags as the
reference plus MI355X-era additions; see ``python train.py --help``."""
import sys

from distributed_char_rnn_amd.engine.trainer import main

if __name__ == "__main__":
    sys.exit(main())
