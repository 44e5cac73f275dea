#!/bin/bash
# GRU batch tiles per workgroup: tests, then config-3 rows at B = 128 / 256; LSTM-2048 loss
# check of the library-step path against the fused per-step kernels at B = 128.
set -o pipefail
O=$PWD/gpurun_out/${1:-gru_nt}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
( while true; do date +%T >> $O/heartbeat.txt; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python -u -m pytest tests/test_gru_persist.py tests/test_native_model.py -k "gru or library_step" -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for b in 128 256; do
  timeout -k 10 300 python -u bench.py --model gru --hidden 1024 --layers 3 --seq 256 --batch $b --steps 10 --warmup 3 > $O/gru_b$b.json 2> $O/gru_b$b.err || { tail -20 $O/gru_b$b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/gru_b$b.json')); print('GRU B=$b ms/step %.2f  chars/s %.3fM loss %.3f' % (d['ms_per_step'], d['value']/1e6, d['final_loss']))"
done
for rec in auto step; do
  DCR_RECURRENCE=$rec timeout -k 10 400 python -u bench.py --hidden 2048 --layers 4 --seq 512 --batch 128 --steps 2 --warmup 1 > $O/l2048_$rec.json 2> $O/l2048_$rec.err || { tail -20 $O/l2048_$rec.err; exit 1; }
  python -c "import json; d=json.load(open('$O/l2048_$rec.json')); print('LSTM-2048 B=128 recurrence=$rec ms/step %.1f loss %.4f' % (d['ms_per_step'], d['final_loss']))"
done
