#!/bin/bash
set -o pipefail
O=gpurun_out/pad
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest tests/test_padded.py tests/test_graph_step.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python train.py --data_dir data/tinyshakespeare --batch_size 50 --seq_length 50 --rnn_size 100 --num_epochs 1 --max_steps 300 --save_every 100000 --log_every 100 --save_dir $O/ckpt --log_dir $O/logs > $O/train_h100.txt 2>&1 || { tail -30 $O/train_h100.txt; exit 1; }
grep -E "^[0-9]+/" $O/train_h100.txt | tail -3
timeout -k 10 120 python sample.py --save_dir $O/ckpt -n 200 > $O/sample_h100.txt 2>&1 || { tail -20 $O/sample_h100.txt; exit 1; }
head -c 300 $O/sample_h100.txt
