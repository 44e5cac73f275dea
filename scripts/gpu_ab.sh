#!/bin/bash
# same-box A/B: build/ab/old.so vs build/ab/new.so (scripts/ab_variant.py), after the pair tests
set -o pipefail
O=gpurun_out/${1:-ab}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest tests/test_pair_batch.py tests/test_dropout.py tests/test_persist.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash scripts/ab_bench.sh build/ab/old.so build/ab/new.so 4 --batch 256 > $O/b256.txt 2>&1 || { cat $O/b256.txt; exit 1; }
bash scripts/ab_bench.sh build/ab/old.so build/ab/new.so 2 --batch 1024 > $O/b1024.txt 2>&1 || { cat $O/b1024.txt; exit 1; }
grep -v amdgpu.ids $O/b256.txt $O/b1024.txt
