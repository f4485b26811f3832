#!/bin/bash
# Round-end measurement on the GPU box (run through gpurun from the repo root):
#   tools/round_profile.sh <tag>      e.g. r02
#   1. rocprofv3 PMC passes (tools/pmc_bench.txt) over bench.py for every
#      workload (its dominant kernel) -> corrected HBM bytes per launch
#      (profiles/pmc_<workload>.json, read by bench.py as roofline.traffic)
#   2. bench.py (the driver's command) -> gpurun_out/<tag>_bench.json
#   3. rocprofv3 --kernel-trace --stats over the same bench.py command
#   4. bench.py --workload for the other BASELINE configs
#   5. tools/kbench.py over every operator (HIP events) and its rocprofv3
#      --kernel-trace --stats summary
# Every GPU step has its own time limit; the script stops at the first failure.
# Only gpurun_out/ travels back from the GPU box: afterwards copy
# gpurun_out/pmc_<workload>.json to profiles/ (bench.py's roofline.traffic)
# and the <tag>_* files you keep.
set -o pipefail
T=${1:-rXX}
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { echo "=== $1 $(date +%T)"; }
for W in resize_normalize:resize_direct warp:warp_ cvt_normalize:color_kernel cubic_stats:cubic_direct yuv_resize:yuv_resize; do
  wl=${W%%:*}; key=${W##*:}
  step "pmc $wl"
  timeout -k 10 400 rocprofv3 -i "$R/tools/pmc_bench.txt" -d "$R/gpurun_out/pmc_$wl" -o pmc --output-format csv \
      -- python3 "$R/bench.py" --workload "$wl" --steps 5 --warmup 2 --no-cpu-baseline > "gpurun_out/pmc_$wl.log" 2>&1 || exit $?
  python3 tools/pmc_summary.py "gpurun_out/pmc_$wl" "$key" --out "gpurun_out/pmc_$wl.json" > "gpurun_out/pmc_${wl}_summary.txt" || exit 1
  cp "gpurun_out/pmc_$wl.json" "profiles/pmc_$wl.json"
done
step bench
timeout -k 10 300 python3 bench.py > "gpurun_out/${T}_bench.json" 2> "gpurun_out/${T}_bench.err" || exit $?
cat "gpurun_out/${T}_bench.json"
step stats
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_bench" -o bench --output-format csv \
    -- python3 "$R/bench.py" > gpurun_out/prof_bench.log 2>&1 || exit $?
find gpurun_out/prof_bench -name "*kernel_stats.csv" -exec cp {} "gpurun_out/${T}_bench_kernel_stats.csv" \;
head -4 "gpurun_out/${T}_bench_kernel_stats.csv"
for wl in warp cvt_normalize cubic_stats yuv_resize; do
  step "bench $wl"
  timeout -k 10 300 python3 bench.py --workload "$wl" > "gpurun_out/${T}_bench_$wl.json" 2> "gpurun_out/${T}_bench_$wl.err" || exit $?
  cat "gpurun_out/${T}_bench_$wl.json"
done
step kbench
timeout -k 10 300 python3 tools/kbench.py --op all --iters 30 > "gpurun_out/${T}_kbench.jsonl" 2> gpurun_out/kbench.err || exit $?
step kbench_stats
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_kbench" -o kbench --output-format csv \
    -- python3 "$R/tools/kbench.py" --op all --iters 30 > gpurun_out/prof_kbench.log 2>&1 || exit $?
find gpurun_out/prof_kbench -name "*kernel_stats.csv" -exec cp {} "gpurun_out/${T}_kbench_kernel_stats.csv" \;
step done
