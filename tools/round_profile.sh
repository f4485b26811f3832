#!/bin/bash
# Round-end measurement on the GPU box (run through gpurun from the repo root):
#   1. rocprofv3 PMC passes over bench.py -> corrected HBM bytes per launch
#      (gpurun_out/pmc_resize_normalize.json, also copied to profiles/ so the
#      bench line below carries it as roofline.traffic)
#   2. bench.py (the driver's command) -> gpurun_out/bench.json
#   3. rocprofv3 --kernel-trace --stats over the same bench.py command
#   4. tools/kbench.py over every operator (HIP events) and its rocprofv3
#      --kernel-trace --stats summary
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { echo "=== $1 $(date +%T)"; }
step pmc
timeout -k 10 400 rocprofv3 -i "$R/tools/pmc_bench.txt" -d "$R/gpurun_out/pmc_bench" -o pmc --output-format csv \
    -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pmc_bench.log 2>&1 || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc_bench resize_ --out gpurun_out/pmc_resize_normalize.json > gpurun_out/pmc_summary.txt || exit 1
cp gpurun_out/pmc_resize_normalize.json profiles/pmc_resize_normalize.json
step bench
timeout -k 10 300 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
cat gpurun_out/bench.json
step stats
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_bench" -o bench --output-format csv \
    -- python3 "$R/bench.py" > gpurun_out/prof_bench.log 2>&1 || exit $?
tail -1 gpurun_out/prof_bench.log
find gpurun_out/prof_bench -name "*kernel_stats.csv" -exec head -5 {} \;
step kbench
timeout -k 10 300 python3 tools/kbench.py --op all --iters 30 > gpurun_out/kbench.jsonl 2> gpurun_out/kbench.err || exit $?
step kbench_stats
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_kbench" -o kbench --output-format csv \
    -- python3 "$R/tools/kbench.py" --op all --iters 30 > gpurun_out/prof_kbench.log 2>&1 || exit $?
find gpurun_out/prof_kbench -name "*kernel_stats.csv" -exec cat {} \;
