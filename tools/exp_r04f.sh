#!/bin/bash
# Round-4 run 6: full GPU suite at the compact-span warp fix + cubic column
# kernel; warp A/B (compact spans vs the round-3 box slots, lib_ow); cubic
# column-kernel variants (rows per wave, store policy); cfg5 rocprof stats.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { echo "=== $1 $(date +%T)"; }
K=arm-neon-opencv_amd
R=$GRAFT_REPO_ROOT
step tests
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/f_tests.log 2>&1 || { tail -30 gpurun_out/f_tests.log; exit 1; }
tail -2 gpurun_out/f_tests.log
step warp_ab
for rep in 1 2 3; do
  for l in lib lib_ow; do
    timeout -k 10 120 python3 tools/kbench_lib.py $K/$l --op warp --only rot15_u8 --iters 30 | sed "s/^/$l /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/f_variants.txt
step cubic_ab
for rep in 1 2; do
  for l in lib lib_cr2 lib_cr8 lib_cs0; do
    timeout -k 10 120 python3 tools/kbench_lib.py $K/$l --op cubic --iters 30 | sed "s/^/$l /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/f_variants.txt
step cubic_prof
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/f_prof_cubic -o cubic --output-format csv -- python3 $R/bench.py --workload cubic_stats --warmup 5 --steps 20 > $R/gpurun_out/f_prof_cubic.log 2>&1 || exit 1
cd $R
find gpurun_out/f_prof_cubic -name "*kernel_stats.csv" -exec cat {} \;
step done
