#!/usr/bin/env python
"""Sample text from a trained model (reference entry point: sample.py)."""
import sys

from distributed_char_rnn_amd.engine.sample_cli import main

if __name__ == "__main__":
    sys.exit(main())
