#!/bin/bash
# PyTorch TunableOp (hipBLASLt/rocBLAS solution search) on the bench's library GEMMs.
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
echo "== default"
timeout -k 10 120 python scripts/bench_gemms.py 2>&1 | grep -v amdgpu.ids
echo "== tunableop (tuning)"
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results.csv \
  timeout -k 10 300 python scripts/bench_gemms.py 2>&1 | grep -v amdgpu.ids
echo "== tunableop (tuned file)"
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results.csv \
  timeout -k 10 120 python scripts/bench_gemms.py 2>&1 | grep -v amdgpu.ids
