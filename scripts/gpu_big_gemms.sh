#!/bin/bash
set -o pipefail
O=$PWD/gpurun_out/${1:-big_gemms}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 200 python scripts/micro/big_gemms_l2048.py > $O/default.txt 2>&1 || { tail $O/default.txt; exit 1; }
cat $O/default.txt
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$O/tunable.csv \
  timeout -k 10 400 python scripts/micro/big_gemms_l2048.py > $O/tuned.txt 2>&1 || { tail $O/tuned.txt; exit 1; }
cat $O/tuned.txt
