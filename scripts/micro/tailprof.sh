cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
DCR_ORACLE_LOG=gpurun_out/nas_oracle2.jsonl timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_native_model.py -k nas > gpurun_out/nas_tests.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tailprof -o tp -- python scripts/micro/tail_bench.py > gpurun_out/tailprof.log 2>&1
