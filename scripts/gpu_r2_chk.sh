#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r2h
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/r2h
timeout -k 10 200 python -u scripts/pair_bench.py --B 256 1024 > $O/pair.txt 2>&1 || { tail -30 $O/pair.txt; exit 1; }
cat $O/pair.txt
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_b256 -o run -- python3 bench.py --steps 20 --warmup 3 --batch 256 > $O/prof_b256.log 2>&1 || { tail -20 $O/prof_b256.log; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_drop -o run -- python3 bench.py --steps 20 --warmup 3 --batch 256 --input_keep_prob 0.8 --output_keep_prob 0.8 > $O/prof_drop.log 2>&1 || { tail -20 $O/prof_drop.log; exit 1; }
