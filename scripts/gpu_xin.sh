#!/bin/bash
# In-kernel input projection of the G = 1 two-layer forward: full GPU suite, then same-box A/B
# (DCR_DEBUG=xin=1: in-kernel projection; default: library zx GEMM) with dropout, and a 4-layer LSTM-512 (layers 2-3 dense).
set -o pipefail
O=$PWD/gpurun_out/${1:-xin}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() { timeout -k 10 300 python -u bench.py "$@" 2> $O/err.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms/step %.3f chars/s %.3fM loss %.4f' % (d['ms_per_step'], d['value']/1e6, d['final_loss']))" || { tail $O/err.txt; exit 1; }; }
for i in 1 2; do
  echo -n "dropout 0.8 xin:  "; DCR_DEBUG=xin=1 run --steps 30 --warmup 5 --input_keep_prob 0.8 --output_keep_prob 0.8
  echo -n "dropout 0.8 lib:  "; run --steps 30 --warmup 5 --input_keep_prob 0.8 --output_keep_prob 0.8
done
echo -n "headline:         "; run --steps 30 --warmup 5
echo -n "4-layer xin:      "; DCR_DEBUG=xin=1 run --layers 4 --steps 20 --warmup 5
echo -n "4-layer lib:      "; run --layers 4 --steps 20 --warmup 5
