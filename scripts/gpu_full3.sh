#!/bin/bash
# Whole GPU suite + smoke + headline bench + kernel trace + every BASELINE.json config (each
# config prints as it finishes, a heartbeat file keeps long captures visibly alive).
set -o pipefail
O=$PWD/gpurun_out/${1:-full3}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
( while true; do date +%T >> $O/heartbeat.txt; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_full.log 2>&1 || { tail -60 $O/pytest_full.log; exit 1; }
tail -2 $O/pytest_full.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_b256 -o run -- python3 bench.py --steps 20 --warmup 3 --batch 256 > $O/prof_b256.log 2>&1 || { tail -20 $O/prof_b256.log; exit 1; }
python scripts/step_trace.py $O/prof_b256/run_results.db > $O/step_trace_b256.txt
tail -1 $O/step_trace_b256.txt
bash scripts/bench_all_configs.sh 2>&1 | tee $O/all_configs.txt
