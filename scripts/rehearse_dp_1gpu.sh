#!/bin/bash
# Multi-rank data-parallel rehearsal on ONE GPU (the GPU box has one card): 2 ranks of bench.py
# share cuda:0 over gloo, launched exactly as the driver launches the N-GPU bench (torchrun,
# 127.0.0.1).  Two passes: the headline shape on the persistent wavefront kernels
# (DCR_GPU_SHARE: a file lock serialises the two processes' persistent launches, which cannot be
# co-resident), then the per-step kernels (DCR_RECURRENCE=step).  Checks the GPU-side DP
# plumbing (bucketed all-reduce of CUDA gradient buffers, the exclusive bucket schedule,
# barriers, max-over-ranks timing, rank-0 output); RCCL itself needs the driver's 8-GPU node.
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
rm -f /tmp/dcr_rehearsal.lock
check() {  # the JSON line must report the 2-rank job with a finite loss
python - "$1" <<'PY' || exit 1
import json, math, sys
line = [l for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1]
r = json.loads(line)
assert r["n_gpus"] == 2, r["n_gpus"]
assert math.isfinite(r["final_loss"]) and r["value"] > 0, r
print("dp rehearsal ok:", sys.argv[1], "n_gpus", r["n_gpus"], "ms/step", round(r["ms_per_step"], 3),
      "final_loss", r["final_loss"])
PY
}
DCR_GPU_SHARE=/tmp/dcr_rehearsal.lock timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 4 \
  --warmup 1 --dist_backend gloo > gpurun_out/dp_rehearsal_persistent.log 2>&1 \
  || { tail -30 gpurun_out/dp_rehearsal_persistent.log; exit 1; }
check gpurun_out/dp_rehearsal_persistent.log || exit 1
DCR_RECURRENCE=step timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 4 --warmup 1 \
  --dist_backend gloo --batch 64 --seq 32 > gpurun_out/dp_rehearsal.log 2>&1 \
  || { tail -30 gpurun_out/dp_rehearsal.log; exit 1; }
check gpurun_out/dp_rehearsal.log || exit 1
