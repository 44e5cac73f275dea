#!/bin/bash
# Round 2: batch-group pair kernels -- tests, kernel sweep, end-to-end bench at B = 256/512/1024.
set -o pipefail
mkdir -p gpurun_out/r2b
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/r2b
timeout -k 10 300 python -u -m pytest tests/test_pair_batch.py -x -v --timeout 120 --timeout-method thread > $O/pytest_pair.log 2>&1 || { tail -40 $O/pytest_pair.log; exit 1; }
tail -3 $O/pytest_pair.log
timeout -k 10 200 python -u scripts/pair_bench.py --B 256 512 1024 > $O/pair_bench.txt 2>&1 || { tail -30 $O/pair_bench.txt; exit 1; }
cat $O/pair_bench.txt
for B in 256 512 1024; do
  timeout -k 10 120 python bench.py --steps 30 --warmup 5 --batch $B > $O/bench_b$B.json 2> $O/bench_b$B.err || { tail -20 $O/bench_b$B.err; exit 1; }
  cat $O/bench_b$B.json
done
timeout -k 10 400 python -u -m pytest tests/test_persist.py -x -q --timeout 120 --timeout-method thread > $O/pytest_persist.log 2>&1 || { tail -40 $O/pytest_persist.log; exit 1; }
tail -3 $O/pytest_persist.log
