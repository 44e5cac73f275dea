#!/bin/bash
# Pair-forward group prefetch: pair / dropout tests, then same-box A/B at B = 512 / 1024 / 256.
set -o pipefail
O=$PWD/gpurun_out/${1:-pair_pref}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests/test_pair_batch.py tests/test_persist.py tests/test_dropout.py tests/test_long_t.py tests/test_padded.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for b in 512; do echo "== B=$b"; bash scripts/ab_bench.sh build/ab/A.so build/ab/B.so 2 --batch $b || exit 1; done
echo "== B=256"; bash scripts/ab_bench.sh build/ab/A.so build/ab/B.so 3 || exit 1
