#!/bin/bash
# Same-box A/B of two native builds on the small configs (reference default, tiny) and headline.
set -o pipefail
export TMPDIR=/tmp PYTHONPATH=$PWD
echo "== ref default"; bash scripts/ab_bench.sh build/ab/A.so build/ab/B.so 3 --batch 50 --seq 50 --hidden 128 || exit 1
echo "== tiny"; bash scripts/ab_bench.sh build/ab/A.so build/ab/B.so 2 --batch 64 --seq 32 --hidden 128 --layers 1 || exit 1
echo "== headline"; bash scripts/ab_bench.sh build/ab/A.so build/ab/B.so 2 || exit 1
