#!/bin/bash
# rocprofv3 PMC passes over a short headline bench run (one counter group per run, each under
# its own time limit; the slot limits of MI355X_MICROARCH.md "rocprofv3 PMC slots").
# PMC_SCRIPT=<script.py> profiles another python script instead of bench.py.
set -o pipefail
export TMPDIR=/tmp PYTHONPATH=$PWD
D=${1:-gpurun_out/pmc}; shift
BA=${*:---steps 5 --warmup 2}
mkdir -p $D
i=0
for pass in \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" \
  "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT" \
  "TCC_HIT TCC_MISS TCC_REQ" \
  "FETCH_SIZE" \
  "WRITE_SIZE"; do
  i=$((i+1))
  echo "== pass $i: $pass"
  timeout -s KILL 90 rocprofv3 --pmc $pass -d $D/p$i -o run --output-format csv -- \
    python3 ${PMC_SCRIPT:-bench.py} $BA > $D/p$i.log 2>&1 || { tail -5 $D/p$i.log; exit 1; }
done
echo done
