#!/usr/bin/env bash
# Local multi-process launch (reference: launch.sh, one ps + two workers on localhost).
# The ps process hosts the rendezvous store and exits when the workers finish; each worker
# drives one GPU (cuda:task_index) and gradients are all-reduced with RCCL over xGMI.
# For N GPUs of one node prefer:  python -m torch.distributed.run --standalone \
#     --nproc-per-node N train.py [flags]
set -euo pipefail
NW=${NUM_WORKERS:-2}
SAVE_DIR=${SAVE_DIR:-distrib-train}
PS=127.0.0.1:${PS_PORT:-8000}
WORKERS=$(python - <<PY
print(",".join(f"127.0.0.1:{9000+i}" for i in range(${NW})))
PY
)
python data_splitter.py --data_dir data/tinyshakespeare --num_parts "${NW}" --out_dir sharded_data
python train.py --distributed --ps_hosts "$PS" --worker_hosts "$WORKERS" --job_name ps \
    --task_index 0 --save_dir "$SAVE_DIR" "$@" &
PIDS=($!)
for ((i = 0; i < NW; i++)); do
  python train.py --distributed --ps_hosts "$PS" --worker_hosts "$WORKERS" --job_name worker \
      --task_index "$i" --save_dir "$SAVE_DIR" --tensor_file "sharded_data/data-$i.npy" "$@" &
  PIDS+=($!)
done
rc=0
for p in "${PIDS[@]}"; do wait "$p" || rc=$?; done
exit $rc
