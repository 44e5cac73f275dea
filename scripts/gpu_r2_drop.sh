#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r2f
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/r2f
timeout -k 10 300 python -u -m pytest tests/test_dropout.py tests/test_pair_batch.py -x -v --timeout 120 --timeout-method thread > $O/pytest_drop.log 2>&1 || { tail -60 $O/pytest_drop.log; exit 1; }
tail -3 $O/pytest_drop.log
