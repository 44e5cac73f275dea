#!/bin/bash
# Large-batch rows of the LSTM-2048 config and a kernel profile of the GRU-1024 config; each
# GPU step under its own time limit, a heartbeat file keeps long graph captures visibly alive.
set -o pipefail
O=$PWD/gpurun_out/${1:-large_batch}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
( while true; do date +%T >> $O/heartbeat.txt; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_gru -o run -- python3 bench.py --model gru --hidden 1024 --layers 3 --seq 256 --batch 128 --steps 3 --warmup 1 > $O/prof_gru.log 2>&1 || { tail -20 $O/prof_gru.log; exit 1; }
python scripts/prof_summary.py $O/prof_gru/run_results.db --per-step 4 > $O/gru_summary.txt
head -25 $O/gru_summary.txt
for b in 128 256 512; do
  echo "== lstm2048x4 seq512 B$b"
  timeout -k 10 400 python -u bench.py --hidden 2048 --layers 4 --seq 512 --batch $b --steps 2 --warmup 1 > $O/l2048_b$b.json 2> $O/l2048_b$b.err || { tail -20 $O/l2048_b$b.err; exit 1; }
  cat $O/l2048_b$b.json
done
