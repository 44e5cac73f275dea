#!/bin/bash
# Whole GPU suite + smoke + headline bench (B=256, 1024) + dropout bench + headline profile.
#   bash scripts/gpu_full.sh <outdir-name>
set -o pipefail
O=gpurun_out/${1:-full}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_full.log 2>&1 || { tail -60 $O/pytest_full.log; exit 1; }
tail -2 $O/pytest_full.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
for B in 256 1024; do
  timeout -k 10 180 python bench.py --steps 30 --warmup 5 --batch $B > $O/bench_b$B.json || exit 1
done
timeout -k 10 180 python bench.py --steps 30 --warmup 5 --batch 256 --input_keep_prob 0.8 --output_keep_prob 0.8 > $O/bench_drop_b256.json || exit 1
for f in $O/bench*.json; do echo $f; python -c "import json,sys; d=json.load(open('$f')); print(d['value']/1e6, d['ms_per_step'])"; done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_b256 -o run -- python3 bench.py --steps 20 --warmup 3 --batch 256 > $O/prof_b256.log 2>&1 || { tail -20 $O/prof_b256.log; exit 1; }
