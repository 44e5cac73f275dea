#!/bin/bash
# quick A/B: tests of the pair kernels + B=256 bench with and without dropout + dropout profile
set -o pipefail
O=gpurun_out/${1:-r2q}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 500 python -u -m pytest tests/test_dropout.py tests/test_pair_batch.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 180 python bench.py --steps 30 --warmup 5 --batch 256 > $O/bench_b256.json || exit 1
timeout -k 10 180 python bench.py --steps 30 --warmup 5 --batch 256 --input_keep_prob 0.8 --output_keep_prob 0.8 > $O/bench_drop_b256.json || exit 1
for f in $O/bench*.json; do echo $f; python -c "import json,sys; d=json.load(open('$f')); print(d['value']/1e6, d['ms_per_step'])"; done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_drop -o run -- python3 bench.py --steps 20 --warmup 3 --batch 256 --input_keep_prob 0.8 --output_keep_prob 0.8 > $O/prof_drop.log 2>&1 || { tail -20 $O/prof_drop.log; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_b256 -o run -- python3 bench.py --steps 20 --warmup 3 --batch 256 > $O/prof_b256.log 2>&1 || { tail -20 $O/prof_b256.log; exit 1; }
