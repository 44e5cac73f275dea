#!/bin/bash
# Library-step path test + LSTM-2048 config rows at large batch (each step under its own limit).
set -o pipefail
O=$PWD/gpurun_out/${1:-l2048_rows}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
( while true; do date +%T >> $O/heartbeat.txt; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u -m pytest tests/test_native_model.py -k library_step -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python scripts/micro/step_gemm_large_b.py > $O/step_forms.txt 2>&1 || { tail $O/step_forms.txt; exit 1; }
grep split $O/step_forms.txt
for b in ${BATCHES:-512 1024}; do
  timeout -k 10 500 python -u bench.py --hidden 2048 --layers 4 --seq 512 --batch $b --steps 2 --warmup 1 > $O/b$b.json 2> $O/b$b.err || { tail -20 $O/b$b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b$b.json')); print('B=$b ms/step %.1f  chars/s %.3fM loss %.3f' % (d['ms_per_step'], d['value']/1e6, d['final_loss']))"
done
