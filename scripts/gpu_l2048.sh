#!/bin/bash
# LSTM-2048 config checks (large-H library-step path), each step under its own time limit;
# a heartbeat file keeps the run visibly alive through long graph captures.
set -o pipefail
O=gpurun_out/l2048; mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
( while true; do date +%T >> $O/heartbeat.txt; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
for args in "$@"; do
  echo "== $args"
  s=$(date +%s)
  timeout -k 10 400 python -u bench.py --hidden 2048 --layers 4 $args > $O/run.json 2> $O/run.err || { tail -20 $O/run.err; exit 1; }
  python -c "import json; d=json.load(open('$O/run.json')); print('ms/step %.1f  chars/s %.3fM loss %.3f' % (d['ms_per_step'], d['value']/1e6, d['final_loss']))"
  echo "   wall $(( $(date +%s) - s )) s"
done
