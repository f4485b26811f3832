#!/bin/bash
# Round-3 closing run on the GPU box (through gpurun, from the repo root):
#   tools/final_r03.sh     the -m gpu suite, smoke(), and PMC passes
#                          (tools/pmc_bench.txt) over kbench for the kernels
#                          changed this round that no bench workload covers
#                          (two-tap strip, area unit / column-sum kernels)
# tools/round_profile.sh <tag> does the bench lines, rocprof stats and kbench.
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out
step() { echo "=== $1 $(date +%T)"; }
step tests
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/final_gpu_tests.log 2>&1 || { tail -30 gpurun_out/final_gpu_tests.log; exit 1; }
tail -2 gpurun_out/final_gpu_tests.log
step smoke
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" || exit 1
for W in "resize:1280x720:resize_strip" "resize_other:area_1080p_960:area_u8_unit" "resize_other:area_1080p_640:area_u8_colsum"; do
  op=${W%%:*}; rest=${W#*:}; only=${rest%%:*}; key=${rest#*:}
  step "pmc $key"
  timeout -s KILL 300 rocprofv3 -i "$R/tools/pmc_bench.txt" -d "$R/gpurun_out/pmc_k_$key" -o pmc --output-format csv \
      -- python3 "$R/tools/kbench.py" --op "$op" --only "$only" --iters 5 > "gpurun_out/pmc_k_$key.log" 2>&1 || exit $?
  python3 tools/pmc_summary.py "gpurun_out/pmc_k_$key" "$key" --out "gpurun_out/pmc_k_$key.json" \
      > "gpurun_out/pmc_k_${key}_summary.txt" || exit 1
done
step "cubic store policy A/B"
if [ -d arm-neon-opencv_amd/lib_cwb ]; then
  for i in 1 2; do for l in lib lib_cwb; do
    timeout -k 10 200 python3 tools/kbench_lib.py arm-neon-opencv_amd/$l --op cubic --iters 30 | sed "s/^/$l /" || exit 1
  done; done
fi
step done
