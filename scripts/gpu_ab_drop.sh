#!/bin/bash
# Same-box A/B of two native builds with dropout 0.8/0.8 and without (headline); dropout tests.
set -o pipefail
export TMPDIR=/tmp PYTHONPATH=$PWD
mkdir -p gpurun_out/ab_drop
timeout -k 10 600 python -u -m pytest tests/test_dropout.py tests/test_head.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_drop/pytest.log 2>&1 || { tail -40 gpurun_out/ab_drop/pytest.log; exit 1; }
tail -1 gpurun_out/ab_drop/pytest.log
echo "== dropout"; bash scripts/ab_bench.sh build/ab/A.so build/ab/B.so 3 --input_keep_prob 0.8 --output_keep_prob 0.8 || exit 1
echo "== headline"; bash scripts/ab_bench.sh build/ab/A.so build/ab/B.so 2 || exit 1
