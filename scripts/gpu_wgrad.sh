#!/bin/bash
set -o pipefail
O=$PWD/gpurun_out/${1:-wgrad}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 120 python -u -m pytest tests/test_wgrad.py -x -v --timeout 60 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python scripts/micro/wgrad_bench.py > $O/bench.txt 2>&1 || { tail $O/bench.txt; exit 1; }
cat $O/bench.txt
