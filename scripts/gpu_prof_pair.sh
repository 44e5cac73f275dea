#!/bin/bash
# Kernel profiles: 3-layer GRU-1024 at B = 256 (NT = 2) and the headline with dropout 0.8/0.8.
set -o pipefail
O=$PWD/gpurun_out/${1:-prof_pair}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/gru256 -o run -- python3 bench.py --model gru --hidden 1024 --layers 3 --seq 256 --batch 256 --steps 3 --warmup 1 > $O/gru256.log 2>&1 || { tail -20 $O/gru256.log; exit 1; }
python scripts/step_trace.py $O/gru256/run_results.db > $O/gru256_trace.txt
tail -1 $O/gru256_trace.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/drop -o run -- python3 bench.py --steps 10 --warmup 3 --input_keep_prob 0.8 --output_keep_prob 0.8 > $O/drop.log 2>&1 || { tail -20 $O/drop.log; exit 1; }
python scripts/step_trace.py $O/drop/run_results.db > $O/drop_trace.txt
cat $O/drop_trace.txt
