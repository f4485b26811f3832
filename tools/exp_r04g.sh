#!/bin/bash
# Round-4 run 7: cfg5 with the in-launch reduction (cubic column kernel's
# last-arrival hand-off): sums tests first, then the full GPU suite, the cfg5
# bench (driver flags) and its rocprof stats.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { echo "=== $1 $(date +%T)"; }
R=$GRAFT_REPO_ROOT
step sums_tests
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "channel_sums or mean_stddev or cubic" \
    > gpurun_out/g_tests_sums.log 2>&1 || { tail -30 gpurun_out/g_tests_sums.log; exit 1; }
tail -2 gpurun_out/g_tests_sums.log
step tests
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/g_tests.log 2>&1 || { tail -30 gpurun_out/g_tests.log; exit 1; }
tail -2 gpurun_out/g_tests.log
step cubic
for rep in 1 2; do
  timeout -k 10 120 python3 bench.py --workload cubic_stats --warmup 5 --steps 20 --no-cpu-baseline | tee -a gpurun_out/g_bench_cubic.json || exit 1
done
timeout -k 10 300 python3 tools/kbench.py --op cubic --iters 30 --sweep 'CUBIC_DIRECT=1,2' 2>&1 | grep -v amdgpu.ids | tee gpurun_out/g_kbench_cubic.jsonl
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/g_prof_cubic -o cubic --output-format csv -- python3 $R/bench.py --workload cubic_stats --warmup 5 --steps 20 > $R/gpurun_out/g_prof_cubic.log 2>&1 || exit 1
cd $R
find gpurun_out/g_prof_cubic -name "*kernel_stats.csv" -exec cat {} \; | grep -v distribution_elementwise
step headline
for rep in 1 2; do
  timeout -k 10 120 python3 bench.py --warmup 5 --steps 20 --no-cpu-baseline | tee -a gpurun_out/g_bench_headline.json || exit 1
done
step warp
timeout -k 10 120 python3 tools/kbench.py --op warp --only rot15_u8 --iters 30 2>&1 | grep -v amdgpu.ids
step done
