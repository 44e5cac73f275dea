#!/bin/bash
# Library GEMM form micro-benchmarks (headline weight gradients, LSTM-2048 step products).
set -o pipefail
O=$PWD/gpurun_out/${1:-gemm_forms}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 180 python scripts/micro/dw_gemm_forms.py > $O/dw_forms.txt 2>&1 || { tail $O/dw_forms.txt; exit 1; }
cat $O/dw_forms.txt
timeout -k 10 180 python scripts/micro/step_gemm_large_b.py > $O/step_forms.txt 2>&1 || { tail $O/step_forms.txt; exit 1; }
cat $O/step_forms.txt
