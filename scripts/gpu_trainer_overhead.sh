#!/bin/bash
set -o pipefail
export TMPDIR=/tmp PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 120 python -u -m pytest tests/test_trainer_batches.py -q --timeout 60 --timeout-method thread || exit 1
timeout -k 10 300 python -u scripts/trainer_overhead.py off 2>&1 | grep -v "^step\|^ *$" | tee gpurun_out/trainer_overhead.txt || exit 1
timeout -k 10 300 python -u scripts/trainer_overhead.py auto 2>&1 | grep "median" | tee -a gpurun_out/trainer_overhead.txt || exit 1
timeout -k 10 120 python bench.py --batch 50 --seq 50 --hidden 128 --steps 100 --warmup 10 | tee -a gpurun_out/trainer_overhead.txt
