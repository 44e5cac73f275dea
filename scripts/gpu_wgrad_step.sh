#!/bin/bash
# wgrad kernel in the training step: numerics tests, then same-box A/B against the library
# split-K GEMMs (DCR_DEBUG=wgrad=0) on the headline, GRU-1024 B=256 and the 8k-vocab configs.
set -o pipefail
O=$PWD/gpurun_out/${1:-wgrad_step}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests/test_wgrad.py tests/test_native_model.py tests/test_persist.py tests/test_long_t.py tests/test_gru_persist.py tests/test_pair_batch.py tests/test_dropout.py tests/test_clip_norm.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() { timeout -k 10 300 python -u bench.py "$@" 2> $O/err.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms/step %.3f chars/s %.3fM loss %.4f' % (d['ms_per_step'], d['value']/1e6, d['final_loss']))" || { tail $O/err.txt; exit 1; }; }
for i in 1 2 3; do
  echo -n "headline wgrad: "; run --steps 40 --warmup 5
  echo -n "headline lib:   "; DCR_DEBUG=wgrad=0 run --steps 40 --warmup 5
done
echo -n "GRU B=256 wgrad: "; run --model gru --hidden 1024 --layers 3 --seq 256 --batch 256 --steps 10 --warmup 3
echo -n "GRU B=256 lib:   "; DCR_DEBUG=wgrad=0 run --model gru --hidden 1024 --layers 3 --seq 256 --batch 256 --steps 10 --warmup 3
echo -n "8k vocab wgrad: "; run --vocab 8192 --steps 10 --warmup 3
echo -n "8k vocab lib:   "; DCR_DEBUG=wgrad=0 run --vocab 8192 --steps 10 --warmup 3
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python scripts/step_trace.py $O/prof/run_results.db > $O/step_trace.txt
cat $O/step_trace.txt
