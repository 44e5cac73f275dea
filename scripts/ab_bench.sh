#!/bin/bash
# Same-box A/B of two builds of the native library (box-to-box spread is 1-3 %, larger than
# many single changes): alternates `bench.py` runs of A and B.
#   bash scripts/ab_bench.sh build/ab/A.so build/ab/B.so [rounds] [bench args...]
set -o pipefail
A=$1; B=$2; N=${3:-3}; shift 3
export PYTHONPATH=$PWD
for i in $(seq $N); do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    ms=$(DCR_NATIVE_LIB=$PWD/$lib timeout -k 10 120 python bench.py --steps 40 --warmup 5 "$@" \
         | python -c "import json,sys; print('%.4f' % json.loads(sys.stdin.read())['ms_per_step'])") || exit 1
    echo "$v $ms"
  done
done
