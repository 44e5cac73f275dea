#!/bin/bash
# Reference-default training throughput (host overhead) + kernel tables of the headline bench at
# B = 256 and B = 1024.
set -o pipefail
mkdir -p gpurun_out/r2d
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/r2d
timeout -k 10 240 python train.py --data_dir data/tinyshakespeare --save_dir /tmp/refdef --log_dir /tmp/refdef_logs --num_epochs 1 --save_every 100000 --log_every 50 --summary_every 0 > $O/train_refdefault.log 2>&1 || { tail -20 $O/train_refdefault.log; exit 1; }
tail -5 $O/train_refdefault.log
for B in 256 1024; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_b$B -o run -- python3 bench.py --steps 20 --warmup 3 --batch $B > $O/prof_b$B.log 2>&1 || { tail -20 $O/prof_b$B.log; exit 1; }
done
