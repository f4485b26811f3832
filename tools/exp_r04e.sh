#!/bin/bash
# Round-4 run 5: Lanczos u8 with dot2 taps; column-kernel variants (16 rows,
# nt / sc0 gathers) against the default; warp ring slots / tile height sweep.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { echo "=== $1 $(date +%T)"; }
K=arm-neon-opencv_amd
step tests
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "lanczos or resize_normalize or resize_linear or warp or channel_sums or cubic" \
    > gpurun_out/e_tests.log 2>&1 || { tail -30 gpurun_out/e_tests.log; exit 1; }
tail -2 gpurun_out/e_tests.log
for l in c16 cl2 cl1; do
  VACV_LIB_DIR=$K/lib_$l timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "resize_linear or resize_normalize or resize_full" \
      > gpurun_out/e_tests_$l.log 2>&1 || { tail -30 gpurun_out/e_tests_$l.log; exit 1; }
  tail -1 gpurun_out/e_tests_$l.log
done
step kbench
timeout -k 10 300 python3 tools/kbench.py --op lanczos --iters 20 | tee gpurun_out/e_kbench.jsonl || exit 1
for rep in 1 2 3; do
  for l in lib lib_c16 lib_cl2 lib_cl1; do
    timeout -k 10 120 python3 tools/kbench_lib.py $K/$l --op resize_normalize --iters 30 | sed "s/^/$l /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/e_variants.txt
timeout -k 10 300 python3 tools/kbench.py --op resize --only 1280 --iters 30 --sweep 'RESIZE_DIRECT=1,2' 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/e_variants.txt
timeout -k 10 300 python3 tools/kbench.py --op warp --only rot15_u8 --iters 30 --sweep 'WARP_SLOTS=2,3,4;WARP_TILE_H=16,32' 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/e_variants.txt
step cubic
timeout -k 10 300 python3 tools/kbench.py --op cubic --iters 30 --sweep 'CUBIC_DIRECT=1,2' 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/e_variants.txt
timeout -k 10 120 python3 bench.py --workload cubic_stats --warmup 5 --steps 20 | tee gpurun_out/e_bench_cubic.json || exit 1
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/e_prof_cubic -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload cubic_stats --warmup 5 --steps 20 > /dev/null 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
find gpurun_out/e_prof_cubic -name "*kernel_stats.csv" -exec cat {} \;
step done
