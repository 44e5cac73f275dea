#!/bin/bash
# Same-box A/B of this tree (B) against an older checkout built in ./abold (A, a git worktree,
# not committed): alternating bench.py runs, bench args passed through.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
for i in 1 2 3; do
  for v in A B; do
    d=$R; [ $v = A ] && d=$R/abold
    out=$(cd $d && PYTHONPATH=$d timeout -k 10 120 python bench.py --steps 40 --warmup 5 "$@") || exit 1
    echo "$v $(echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.4f ms loss %.6f' % (d['ms_per_step'], d['final_loss']))")"
  done
done
