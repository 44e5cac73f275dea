#!/bin/bash
# --graph: correctness vs eager, then eager/graph benches at the reference default config
# (2-layer LSTM-128, B=50, T=50) and the headline config
set -o pipefail
O=gpurun_out/${1:-graph}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest tests/test_graph_step.py tests/test_persist.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for g in "" "--graph"; do
  timeout -k 10 180 python bench.py --steps 200 --warmup 10 --batch 50 --seq 50 --hidden 128 $g > $O/bench_refdef$g.json || exit 1
  timeout -k 10 180 python bench.py --steps 30 --warmup 5 --batch 256 $g > $O/bench_b256$g.json || exit 1
done
for f in $O/bench*.json; do echo $f; python -c "import json,sys; d=json.load(open('$f')); print(d['value']/1e6, d['ms_per_step'])"; done
timeout -k 10 300 python train.py --synthetic_text 2000000 --batch_size 50 --seq_length 50 --rnn_size 128 --num_epochs 1 --max_steps 400 --save_every 100000 --log_every 100 --graph on --save_dir $O/ckpt_g --log_dir $O/logs_g > $O/train_graph.txt 2>&1 || { tail -30 $O/train_graph.txt; exit 1; }
timeout -k 10 300 python train.py --synthetic_text 2000000 --batch_size 50 --seq_length 50 --rnn_size 128 --num_epochs 1 --max_steps 400 --save_every 100000 --log_every 100 --graph off --save_dir $O/ckpt_e --log_dir $O/logs_e > $O/train_eager.txt 2>&1 || { tail -30 $O/train_eager.txt; exit 1; }
grep -E "^[0-9]+/" $O/train_graph.txt | tail -2; grep -E "^[0-9]+/" $O/train_eager.txt | tail -2
