# counter passes over single tail tasks (scripts/micro/tail_pmc.py); one pass per rocprofv3 run
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/tailpmc; mkdir -p $out
for task in 0:8 1:9 1:7 0:2; do
  tag=${task/:/_}
  TAIL_TASK=$task timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU --kernel-trace -d /tmp/pmc_a_$tag -o p -- python scripts/micro/tail_pmc.py > $out/a_$tag.log 2>&1 || exit 1
  python scripts/micro/pmc_summary.py /tmp/pmc_a_$tag tail_kernel > $out/a_$tag.txt
  TAIL_TASK=$task timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAIT_ANY GRBM_GUI_ACTIVE --kernel-trace -d /tmp/pmc_b_$tag -o p -- python scripts/micro/tail_pmc.py > $out/b_$tag.log 2>&1 || exit 1
  python scripts/micro/pmc_summary.py /tmp/pmc_b_$tag tail_kernel > $out/b_$tag.txt
done
