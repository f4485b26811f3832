#!/bin/bash
# Round-5 closing run on the GPU box (through gpurun, from the repo root).
# Every GPU step has its own time limit; the script stops at the first failure.
#   1. the -m gpu suite and smoke()
#   2. rocprofv3 PMC passes (tools/pmc_bench.txt) over bench.py for every
#      workload's dominant kernel -> gpurun_out/pmc_<workload>.json (copied to
#      profiles/ afterwards: bench.py's roofline.traffic)
#   3. bench.py as the driver runs it (--warmup 5 --steps 20), twice, and its
#      rocprofv3 --kernel-trace --stats summary
#   4. bench.py --workload for the other BASELINE configs
#   5. tools/kbench.py --op all (HIP events) and its rocprofv3 stats
#   6. PMC passes over kbench for the kernels no bench workload covers
#      (two-tap resize, INTER_AREA unit kernel, Lanczos)
# Only gpurun_out/ travels back: copy what is kept to profiles/ afterwards.
set -o pipefail
T=${1:-r05}
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { echo "=== $1 $(date +%T)"; }
step tests
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/${T}_gpu_tests.log 2>&1 || { tail -30 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.log
step smoke
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" || exit 1
for W in resize_normalize:resize_cols warp:warp_exp cvt_normalize:color_kernel cubic_stats:cubic_cols yuv_resize:yuv_cols; do
  wl=${W%%:*}; key=${W##*:}
  step "pmc $wl"
  timeout -k 10 400 rocprofv3 -i "$R/tools/pmc_bench.txt" -d "$R/gpurun_out/pmc_$wl" -o pmc --output-format csv \
      -- python3 "$R/bench.py" --workload "$wl" --steps 5 --warmup 2 --no-cpu-baseline > "gpurun_out/pmc_$wl.log" 2>&1 || exit $?
  python3 tools/pmc_summary.py "gpurun_out/pmc_$wl" "$key" --out "gpurun_out/pmc_$wl.json" > "gpurun_out/pmc_${wl}_summary.txt" || exit 1
  cp "gpurun_out/pmc_$wl.json" "profiles/pmc_$wl.json"
done
step bench
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --warmup 5 --steps 20 > "gpurun_out/${T}_bench_$i.json" 2> "gpurun_out/${T}_bench_$i.err" || exit $?
  cat "gpurun_out/${T}_bench_$i.json"
done
step stats
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_bench" -o bench --output-format csv \
    -- python3 "$R/bench.py" --warmup 5 --steps 20 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 || exit $?
find gpurun_out/prof_bench -name "*kernel_stats.csv" -exec cp {} "gpurun_out/${T}_bench_kernel_stats.csv" \;
head -4 "gpurun_out/${T}_bench_kernel_stats.csv"
for wl in warp cvt_normalize cubic_stats yuv_resize; do
  step "bench $wl"
  timeout -k 10 300 python3 bench.py --workload "$wl" --warmup 5 --steps 20 > "gpurun_out/${T}_bench_$wl.json" 2> "gpurun_out/${T}_bench_$wl.err" || exit $?
  cat "gpurun_out/${T}_bench_$wl.json"
done
step "stats cubic_stats"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_cubic" -o cubic --output-format csv \
    -- python3 "$R/bench.py" --workload cubic_stats --warmup 5 --steps 20 --no-cpu-baseline > gpurun_out/prof_cubic.log 2>&1 || exit $?
find gpurun_out/prof_cubic -name "*kernel_stats.csv" -exec cp {} "gpurun_out/${T}_cubic_stats_kernel_stats.csv" \;
step kbench
timeout -k 10 400 python3 tools/kbench.py --op all --iters 30 > "gpurun_out/${T}_kbench.jsonl" 2> gpurun_out/kbench.err || exit $?
step kbench_stats
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_kbench" -o kbench --output-format csv \
    -- python3 "$R/tools/kbench.py" --op all --iters 30 > gpurun_out/prof_kbench.log 2>&1 || exit $?
find gpurun_out/prof_kbench -name "*kernel_stats.csv" -exec cp {} "gpurun_out/${T}_kbench_kernel_stats.csv" \;
for W in "resize:1280x720:resize_strip" "resize_other:area_1080p_960:area_u8_unit" "lanczos:lanczos_1080p_640x360_u8:lanczos"; do
  op=${W%%:*}; rest=${W#*:}; only=${rest%%:*}; key=${rest#*:}
  step "pmc $key"
  timeout -s KILL 300 rocprofv3 -i "$R/tools/pmc_bench.txt" -d "$R/gpurun_out/pmc_k_$key" -o pmc --output-format csv \
      -- python3 "$R/tools/kbench.py" --op "$op" --only "$only" --iters 5 > "gpurun_out/pmc_k_$key.log" 2>&1 || exit $?
  python3 tools/pmc_summary.py "gpurun_out/pmc_k_$key" "$key" --out "gpurun_out/pmc_k_$key.json" \
      > "gpurun_out/pmc_k_${key}_summary.txt" || exit 1
done
step done
