#!/bin/bash
# In-kernel input bias (dense zx routes): affected GPU tests, then dropout headline + GRU rows.
set -o pipefail
O=$PWD/gpurun_out/${1:-bias_fold}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests/test_dropout.py tests/test_gru_persist.py tests/test_pair_batch.py tests/test_persist.py tests/test_long_t.py tests/test_native_model.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() { timeout -k 10 300 python -u bench.py "$@" 2> $O/err.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms/step %.3f chars/s %.3fM loss %.4f' % (d['ms_per_step'], d['value']/1e6, d['final_loss']))" || { tail $O/err.txt; exit 1; }; }
echo -n "headline dropout 0.8/0.8: "; run --steps 30 --warmup 5 --input_keep_prob 0.8 --output_keep_prob 0.8
echo -n "headline: "; run --steps 30 --warmup 5
echo -n "GRU B=256: "; run --model gru --hidden 1024 --layers 3 --seq 256 --batch 256 --steps 10 --warmup 3
echo -n "GRU B=128: "; run --model gru --hidden 1024 --layers 3 --seq 256 --batch 128 --steps 10 --warmup 3
