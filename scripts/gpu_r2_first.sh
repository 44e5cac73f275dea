set -o pipefail
mkdir -p gpurun_out/r2a
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 180 python bench.py --steps 40 --warmup 5 > gpurun_out/r2a/bench.json 2> gpurun_out/r2a/bench.err || exit 1
cat gpurun_out/r2a/bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r2a/prof -o run -- python3 bench.py --steps 20 --warmup 3 > gpurun_out/r2a/prof.log 2>&1 || exit 1
find gpurun_out/r2a/prof -name '*stats*' | head
