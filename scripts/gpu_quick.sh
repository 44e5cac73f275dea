#!/bin/bash
# Quick GPU iteration on 1x MI355X: selected GPU tests (args = pytest -k expression) + bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
K="${1:-persist}"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "$K" > gpurun_out/pytest_quick.log 2>&1 || { tail -40 gpurun_out/pytest_quick.log; exit 1; }
tail -3 gpurun_out/pytest_quick.log
timeout -k 10 180 python bench.py --steps 40 --warmup 5 || exit 1
