#!/bin/bash
# Whole GPU test suite + smoke + headline bench (both clip-norm modes).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_full.log 2>&1 || { tail -40 gpurun_out/pytest_full.log; exit 1; }
tail -2 gpurun_out/pytest_full.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 180 python bench.py --steps 60 --warmup 5 | tee gpurun_out/bench_tf.json || exit 1
timeout -k 10 180 python bench.py --steps 60 --warmup 5 --clip_norm dense | tee gpurun_out/bench_dense.json || exit 1
