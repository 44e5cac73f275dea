#!/bin/bash
# Round evidence: every BASELINE.json config (bench_all_configs.sh) + PMC passes of the headline
set -o pipefail
export TMPDIR=/tmp PYTHONPATH=$PWD
mkdir -p gpurun_out/evidence
bash scripts/bench_all_configs.sh > gpurun_out/evidence/configs.txt 2>&1 || { cat gpurun_out/evidence/configs.txt; exit 1; }
cat gpurun_out/evidence/configs.txt
bash scripts/pmc_passes.sh > gpurun_out/evidence/pmc.txt 2>&1 || { tail -20 gpurun_out/evidence/pmc.txt; exit 1; }
tail -2 gpurun_out/evidence/pmc.txt
