#!/bin/bash
# Fast GPU iteration: selected GPU tests (pytest -k expression, $2) + headline bench + kernel
# trace of the headline step.   bash scripts/gpu_iter.sh <outdir-name> [-k expr]
set -o pipefail
O=gpurun_out/${1:-iter}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
K="${2:-prep or sumsq or smoke or native_model or long_t}"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 180 python bench.py --steps 30 --warmup 5 --batch 256 > $O/bench_b256.json || exit 1
python -c "import json; d=json.load(open('$O/bench_b256.json')); print('B256', d['value']/1e6, d['ms_per_step'])"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_b256 -o run -- python3 bench.py --steps 10 --warmup 3 --batch 256 > $O/prof_b256.log 2>&1 || { tail -20 $O/prof_b256.log; exit 1; }
python scripts/step_trace.py $O/prof_b256/run_results.db
