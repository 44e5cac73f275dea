#!/bin/bash
# The one GPU-box runner (replaces the round-1/2 one-off gpu_*.sh wrappers).
#
#   bash scripts/gpu.sh <out-name> <step> [<step> ...]
#
# Each step runs under its own time limit, writes under gpurun_out/<out-name>/, and the script
# stops at the first failing step (no GPU work after a fault / abort / timeout).  Steps:
#
#   tests[=<pytest -k expr>]   pytest -m gpu (optionally a -k subset)
#   smoke                      __graft_entry__.smoke()
#   bench[=<bench.py args>]    bench.py (default: headline, 20 steps); args use ',' for ' '
#   trace[=<bench.py args>]    rocprofv3 --kernel-trace --stats of bench.py + one-step trace
#   configs                    every BASELINE.json config (scripts/bench_all_configs.sh)
#   pmc[=<bench.py args>]      the PMC counter passes (scripts/pmc_passes.sh)
#   py=<script,args>           any python script of the repo (e.g. py=scripts/pair_bench.py,--stamps)
#   ab=<A.so>,<B.so>[,rounds,<bench args>]  same-box A/B of two builds (scripts/ab_bench.sh)
#   abenv=<VAR=value>[;<bench args>]  same-box A/B of bench.py without / with an environment
#                              setting (e.g. abenv=DCR_DEBUG=wide=0), 3 alternating rounds
#   abargs=<args A>|<args B>[|...]  same-box comparison of bench.py argument sets (',' for ' ';
#                              an empty set is the default run), 3 alternating rounds
#
# Example: gpurun --timeout 900 -- bash scripts/gpu.sh r3_base tests bench trace
set -o pipefail
NAME=${1:?out name}; shift
O=$PWD/gpurun_out/$NAME
mkdir -p "$O"
export TMPDIR=/tmp PYTHONPATH=$PWD
( while true; do date +%T >> "$O/heartbeat.txt"; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
sp() { echo "${1//,/ }"; }   # ',' -> ' ' in step arguments

for step in "$@"; do
  key=${step%%=*}; arg=""; [[ "$step" == *=* ]] && arg=${step#*=}
  echo "== $step ($(date +%T))"
  case "$key" in
    tests)
      K=(); [ -n "$arg" ] && K=(-k "$(sp "$arg")")
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 \
        --timeout-method thread "${K[@]}" > "$O/pytest.log" 2>&1 || { tail -60 "$O/pytest.log"; exit 1; }
      tail -3 "$O/pytest.log" ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    bench)
      A=${arg:---steps,20,--warmup,3}
      timeout -k 10 300 python bench.py $(sp "$A") | tee -a "$O/bench.jsonl" || exit 1 ;;
    trace)
      A=${arg:---steps,20,--warmup,3}
      tag=$(echo "$A" | tr -c 'a-zA-Z0-9' '_' | cut -c1-40)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$tag" -o run -- \
        python3 bench.py $(sp "$A") > "$O/prof_$tag.log" 2>&1 || { tail -20 "$O/prof_$tag.log"; exit 1; }
      python scripts/step_trace.py "$O/prof_$tag/run_results.db" ${TRACE_MARKER:-lstm2_fwd} > "$O/step_trace_$tag.txt" || exit 1
      tail -1 "$O/step_trace_$tag.txt"; tail -1 "$O/prof_$tag.log" ;;
    configs)
      bash scripts/bench_all_configs.sh 2>&1 | tee "$O/all_configs.txt" || exit 1 ;;
    pmc)
      bash scripts/pmc_passes.sh "$O/pmc" $(sp "$arg") > "$O/pmc.log" 2>&1 || { tail -20 "$O/pmc.log"; exit 1; }
      python scripts/pmc_summary.py "$O/pmc" > "$O/pmc_summary.md" || exit 1
      cat "$O/pmc_summary.md" ;;
    py)
      read -r -a P <<< "$(sp "$arg")"
      echo "== ${P[*]}" >> "$O/py_$(basename "${P[0]}" .py).log"
      timeout -k 10 600 python -u "${P[@]}" >> "$O/py_$(basename "${P[0]}" .py).log" 2>&1 || {
        tail -40 "$O/py_$(basename "${P[0]}" .py).log"; exit 1; }
      tail -40 "$O/py_$(basename "${P[0]}" .py).log" ;;
    ab)
      bash scripts/ab_bench.sh $(sp "$arg") > "$O/ab.log" 2>&1 || { tail -20 "$O/ab.log"; exit 1; }
      cat "$O/ab.log" ;;
    abenv)
      EV=${arg%%;*}; BA="--steps,40,--warmup,5"; [[ "$arg" == *";"* ]] && BA=${arg#*;}
      for i in 1 2 3; do
        for v in base env; do
          if [ $v = base ]; then
            ms=$(timeout -k 10 120 python bench.py $(sp "$BA") | python -c "import json,sys; print('%.4f' % json.loads(sys.stdin.read())['ms_per_step'])") || exit 1
          else
            ms=$(env "$EV" timeout -k 10 120 python bench.py $(sp "$BA") | python -c "import json,sys; print('%.4f' % json.loads(sys.stdin.read())['ms_per_step'])") || exit 1
          fi
          echo "$v $ms" | tee -a "$O/abenv.log"
        done
      done ;;
    abargs)
      IFS='|' read -r -a VS <<< "$arg"
      for i in 1 2 3; do
        for v in "${VS[@]}"; do
          ms=$(timeout -k 10 120 python bench.py --steps 40 --warmup 5 $(sp "$v") | tail -1 | python -c "import json,sys; print('%.4f' % json.loads(sys.stdin.read())['ms_per_step'])") || exit 1
          echo "[$v] $ms" | tee -a "$O/abargs.log"
        done
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
