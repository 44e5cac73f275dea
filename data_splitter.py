#!/usr/bin/env python
"""Offline corpus sharding (reference entry point: data_splitter.py)."""
import sys

from distributed_char_rnn_amd.utils.splitter import main

if __name__ == "__main__":
    sys.exit(main())
