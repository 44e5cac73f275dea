#!/bin/bash
# Whole GPU test suite + smoke + headline bench.
set -o pipefail
mkdir -p gpurun_out/r2c
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/r2c
timeout -k 10 200 python -u -m pytest tests/test_gpu_dp.py -x -v --timeout 120 --timeout-method thread > $O/pytest_dp.log 2>&1 || { tail -60 $O/pytest_dp.log; exit 1; }
tail -4 $O/pytest_dp.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_full.log 2>&1 || { tail -60 $O/pytest_full.log; exit 1; }
tail -3 $O/pytest_full.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 180 python bench.py --steps 40 --warmup 5 > $O/bench.json || exit 1
cat $O/bench.json
