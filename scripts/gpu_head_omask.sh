#!/bin/bash
# Output-dropout mask applied by the head kernel: dropout tests, then same-box A/B.
set -o pipefail
O=$PWD/gpurun_out/${1:-head_omask}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests/test_dropout.py tests/test_head.py tests/test_graph_step.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() { timeout -k 10 300 python -u bench.py "$@" 2> $O/err.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms/step %.3f chars/s %.3fM loss %.4f' % (d['ms_per_step'], d['value']/1e6, d['final_loss']))" || { tail $O/err.txt; exit 1; }; }
for i in 1 2 3; do
  echo -n "head mask: "; run --steps 30 --warmup 5 --input_keep_prob 0.8 --output_keep_prob 0.8
  echo -n "pass mask: "; DCR_DEBUG=head_omask=0 run --steps 30 --warmup 5 --input_keep_prob 0.8 --output_keep_prob 0.8
done
