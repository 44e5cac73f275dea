#!/bin/bash
# Kernel trace of the reference-default shape (2-layer LSTM-128, B = 50, T = 50).
set -o pipefail
O=$PWD/gpurun_out/${1:-prof_small}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --batch 50 --seq 50 --hidden 128 --steps 30 --warmup 5 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python scripts/step_trace.py $O/prof/run_results.db > $O/step_trace.txt
cat $O/step_trace.txt
tail -1 $O/prof.log
