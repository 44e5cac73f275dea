#!/bin/bash
# Whole GPU suite + smoke + headline bench + dropout bench + batch sweep.
set -o pipefail
mkdir -p gpurun_out/r2g
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/r2g
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_full.log 2>&1 || { tail -60 $O/pytest_full.log; exit 1; }
tail -2 $O/pytest_full.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
for B in 256 1024; do
  timeout -k 10 180 python bench.py --steps 30 --warmup 5 --batch $B > $O/bench_b$B.json || exit 1
  timeout -k 10 180 python bench.py --steps 30 --warmup 5 --batch $B --input_keep_prob 0.8 --output_keep_prob 0.8 > $O/bench_drop_b$B.json || exit 1
done
for f in $O/bench*.json; do echo $f; python -c "import json,sys; d=json.load(open('$f')); print(d['value']/1e6, d['ms_per_step'])"; done
