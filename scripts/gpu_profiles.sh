#!/bin/bash
# Evidence for profiles/: full GPU suite, headline bench at B=256/512/1024 and with dropout,
# rocprofv3 kernel stats of each, pair-kernel phase stamps.
#   bash scripts/gpu_profiles.sh <outdir-name>
set -o pipefail
O=gpurun_out/${1:-prof}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_full.log 2>&1 || { tail -60 $O/pytest_full.log; exit 1; }
tail -1 $O/pytest_full.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
for B in 256 512 1024; do
  timeout -k 10 180 python bench.py --steps 30 --warmup 5 --batch $B > $O/bench_b$B.json || exit 1
done
timeout -k 10 180 python bench.py --steps 30 --warmup 5 --batch 256 --input_keep_prob 0.8 --output_keep_prob 0.8 > $O/bench_drop_b256.json || exit 1
timeout -k 10 180 python bench.py --steps 30 --warmup 5 --batch 256 --input_keep_prob 0.5 --output_keep_prob 0.5 > $O/bench_drop50_b256.json || exit 1
for f in $O/bench*.json; do echo $f; python -c "import json,sys; d=json.load(open('$f')); print(d['value']/1e6, d['ms_per_step'])"; done
timeout -k 10 200 python -u scripts/pair_bench.py --B 256 512 1024 --stamps > $O/pair_stamps.txt 2>&1 || { tail -30 $O/pair_stamps.txt; exit 1; }
for B in 256 1024; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_b$B -o run -- python3 bench.py --steps 20 --warmup 3 --batch $B > $O/prof_b$B.log 2>&1 || { tail -20 $O/prof_b$B.log; exit 1; }
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_drop -o run -- python3 bench.py --steps 20 --warmup 3 --batch 256 --input_keep_prob 0.8 --output_keep_prob 0.8 > $O/prof_drop.log 2>&1 || { tail -20 $O/prof_drop.log; exit 1; }
