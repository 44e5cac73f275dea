#!/bin/bash
# One line per BASELINE.json config on 1x MI355X (run on the GPU box from the repo root).
set -o pipefail
run() {
  local name="$1"; shift
  timeout -k 10 400 python bench.py "$@" 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', 'ms/step=%.3f' % d['ms_per_step'], 'chars/s=%.3fM' % (d['value']/1e6), 'loss=%.3f' % d['final_loss'])"
}
run "lstm512x2 seq128 B256 (headline)" --steps 40 --warmup 5 || exit 1
run "lstm512x2 seq128 B256 (repeat)  " --steps 40 --warmup 5 || exit 1
run "gru1024x3 seq256 B128           " --model gru --hidden 1024 --layers 3 --seq 256 --batch 128 --steps 10 --warmup 3 || exit 1
run "gru1024x3 seq256 B256 (NT=2)    " --model gru --hidden 1024 --layers 3 --seq 256 --batch 256 --steps 10 --warmup 3 || exit 1
run "lstm2048x4 seq512 B64           " --hidden 2048 --layers 4 --seq 512 --batch 64 --steps 3 --warmup 1 || exit 1
run "lstm2048x4 seq512 B128 (NT=4)   " --hidden 2048 --layers 4 --seq 512 --batch 128 --steps 3 --warmup 1 || exit 1
run "lstm2048x4 seq512 B1024 (large)  " --hidden 2048 --layers 4 --seq 512 --batch 1024 --steps 2 --warmup 1 || exit 1
run "lstm512x2 seq128 B256 vocab8192 " --vocab 8192 --steps 10 --warmup 3 || exit 1
run "lstm128x1 seq32 B50 (tiny)      " --hidden 128 --layers 1 --seq 32 --batch 64 --steps 20 --warmup 5 || exit 1
run "lstm128x2 seq50 B50 (ref default)" --hidden 128 --layers 2 --seq 50 --batch 50 --steps 30 --warmup 5 || exit 1
run "lstm512x2 seq128 B256 dropout0.8 " --input_keep_prob 0.8 --output_keep_prob 0.8 --steps 30 --warmup 5 || exit 1
