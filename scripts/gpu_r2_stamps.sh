#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r2e
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 200 python -u scripts/pair_bench.py --B 256 --G 1 2 4 --stamps > gpurun_out/r2e/stamps_b256.txt 2>&1 || { tail -30 gpurun_out/r2e/stamps_b256.txt; exit 1; }
timeout -k 10 200 python -u scripts/pair_bench.py --B 1024 --stamps > gpurun_out/r2e/stamps_b1024.txt 2>&1 || { tail -30 gpurun_out/r2e/stamps_b1024.txt; exit 1; }
cat gpurun_out/r2e/stamps_b256.txt gpurun_out/r2e/stamps_b1024.txt
