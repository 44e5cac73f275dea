#!/bin/bash
# torch.nn.LSTM / nn.GRU (MIOpen) comparison runs for the BASELINE.json configs (1x MI355X).
set -o pipefail
export PYTHONPATH=$PWD
run() { timeout -k 10 300 python scripts/bench_miopen_lstm.py "$@" 2>&1 | grep '"impl"'; }
run --model gru --hidden 1024 --layers 3 --seq 256 --batch 128 --steps 5 --warmup 2 || exit 1
run --hidden 2048 --layers 4 --seq 512 --batch 64 --steps 3 --warmup 1 || exit 1
run --hidden 512 --layers 2 --seq 128 --batch 256 --vocab 8192 --steps 10 --warmup 3 || exit 1
run --hidden 128 --layers 1 --seq 32 --batch 64 --steps 20 --warmup 5 || exit 1
