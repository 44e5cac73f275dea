#!/bin/bash
# LSTM-2048 large-batch investigation: step-GEMM forms (default and TunableOp) and a kernel
# profile of the B = 512 training step.
set -o pipefail
O=$PWD/gpurun_out/${1:-l2048_prof}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
( while true; do date +%T >> $O/heartbeat.txt; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 120 python scripts/micro/step_gemm_large_b.py > $O/step_gemm.txt 2>&1 || { tail $O/step_gemm.txt; exit 1; }
cat $O/step_gemm.txt
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$O/tunable.csv \
  timeout -k 10 300 python scripts/micro/step_gemm_large_b.py > $O/step_gemm_tunable.txt 2>&1 || { tail $O/step_gemm_tunable.txt; exit 1; }
cat $O/step_gemm_tunable.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b512 -o run -- python3 bench.py --hidden 2048 --layers 4 --seq 512 --batch 512 --steps 2 --warmup 1 > $O/prof_b512.log 2>&1 || { tail -20 $O/prof_b512.log; exit 1; }
python scripts/prof_summary.py $O/prof_b512/run_results.db --per-step 3 > $O/b512_summary.txt
head -30 $O/b512_summary.txt
