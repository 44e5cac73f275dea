#!/bin/bash
# dropout masks staged in LDS (pair kernels), vectorized segment sum; dEW route A/B
set -o pipefail
O=gpurun_out/r2k
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 500 python -u -m pytest tests/test_native_model.py tests/test_dropout.py tests/test_long_t.py -x -q -rA --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for B in 256; do
  timeout -k 10 180 python bench.py --steps 30 --warmup 5 --batch $B > $O/bench_b$B.json || exit 1
  DCR_DEW=segsum timeout -k 10 180 python bench.py --steps 30 --warmup 5 --batch $B > $O/bench_seg_b$B.json || exit 1
  timeout -k 10 180 python bench.py --steps 30 --warmup 5 --batch $B --input_keep_prob 0.8 --output_keep_prob 0.8 > $O/bench_drop_b$B.json || exit 1
done
for f in $O/bench*.json; do echo $f; python -c "import json,sys; d=json.load(open('$f')); print(d['value']/1e6, d['ms_per_step'])"; done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_drop -o run -- python3 bench.py --steps 20 --warmup 3 --batch 256 --input_keep_prob 0.8 --output_keep_prob 0.8 > $O/prof_drop.log 2>&1 || { tail -20 $O/prof_drop.log; exit 1; }
DCR_DEW=segsum timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_seg -o run -- python3 bench.py --steps 20 --warmup 3 --batch 256 > $O/prof_seg.log 2>&1 || { tail -20 $O/prof_seg.log; exit 1; }
