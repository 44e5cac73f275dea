#!/bin/bash
# TF clip-norm semantics on the GPU: optimizer/sumsq kernels, native-vs-oracle slot, readiness,
# then the headline bench in both clip-norm modes (cost of the per-token term).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "optim or native_model or grad_ready or e2e" > gpurun_out/pytest_norm.log 2>&1 \
  || { tail -40 gpurun_out/pytest_norm.log; exit 1; }
tail -3 gpurun_out/pytest_norm.log
timeout -k 10 180 python bench.py --steps 60 --warmup 5 || exit 1
timeout -k 10 180 python bench.py --steps 60 --warmup 5 --clip_norm dense || exit 1
timeout -k 10 180 python bench.py --steps 60 --warmup 5 || exit 1
