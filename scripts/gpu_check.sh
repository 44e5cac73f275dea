#!/bin/bash
# Round GPU check on 1x MI355X (run on the GPU box from the repo root): GPU tests, smoke, bench,
# rocprofv3 kernel stats of the headline bench.  Every GPU step has its own time limit; the
# script stops at the first failing step.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
step smoke
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench
timeout -k 10 180 python bench.py --steps 40 --warmup 5 | tee gpurun_out/bench.json || exit 1
timeout -k 10 180 python bench.py --steps 40 --warmup 5 || exit 1
if [ "$1" = "prof" ]; then
  step rocprof
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- \
    python3 bench.py --steps 20 --warmup 3 > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
  find gpurun_out/prof -name '*kernel_stats.csv' | head -3
fi
step done
