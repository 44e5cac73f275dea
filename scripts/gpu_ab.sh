set -o pipefail
mkdir -p gpurun_out/ab1
bash scripts/ab_bench.sh build/ab/old.so build/ab/new.so 4 --batch 256 > gpurun_out/ab1/b256.txt 2>&1 || exit 1
cat gpurun_out/ab1/b256.txt
bash scripts/ab_bench.sh build/ab/old.so build/ab/new.so 3 --batch 256 --input_keep_prob 0.8 --output_keep_prob 0.8 > gpurun_out/ab1/drop.txt 2>&1 || exit 1
cat gpurun_out/ab1/drop.txt
