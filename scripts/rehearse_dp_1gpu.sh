#!/bin/bash
# Multi-rank data-parallel rehearsal on ONE GPU (the GPU box has one card): 2 ranks of bench.py
# and train.py share cuda:0 over gloo with the per-step kernels (DCR_RECURRENCE=step: two processes'
# persistent grids cannot be co-resident).  Checks the GPU-side DP plumbing (bucketed all-reduce
# of CUDA gradient buffers, barriers, max-over-ranks timing, rank-0 output); RCCL itself needs
# the driver's 8-GPU node.
set -o pipefail
export PYTHONPATH=$PWD DCR_RECURRENCE=step
mkdir -p gpurun_out
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 4 --warmup 1 \
  --dist_backend gloo --batch 64 --seq 32 > gpurun_out/dp_rehearsal.log 2>&1 || { tail -30 gpurun_out/dp_rehearsal.log; exit 1; }
grep '"metric"' gpurun_out/dp_rehearsal.log
# the JSON line must report the 2-rank job with a finite loss
python - <<'PY' || exit 1
import json, math
line = [l for l in open("gpurun_out/dp_rehearsal.log") if l.startswith('{"metric"')][-1]
r = json.loads(line)
assert r["n_gpus"] == 2, r["n_gpus"]
assert math.isfinite(r["final_loss"]) and r["value"] > 0, r
print("dp rehearsal ok: n_gpus", r["n_gpus"], "final_loss", r["final_loss"])
PY
