#!/bin/bash
# Round-4 experiment run 2: the Lanczos fix, kernel variants (tools/variants.sh
# builds): headline diagnosis / cache policies / rows kernel, warp ring
# diagnosis / policies, strip store policy and strip width.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { echo "=== $1 $(date +%T)"; }
step lanczos_test
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "lanczos or resize_direct or resize_normalize or resize_linear" \
    > gpurun_out/b_tests.log 2>&1 || { tail -30 gpurun_out/b_tests.log; exit 1; }
tail -2 gpurun_out/b_tests.log
step kbench_new
timeout -k 10 300 python3 tools/kbench.py --op lanczos --iters 20 | tee gpurun_out/b_kbench_new.jsonl || exit 1
step variants
K=arm-neon-opencv_amd
for rep in 1 2; do
  for l in lib lib_nf lib_d1 lib_d3 lib_d4 lib_s0 lib_s16 lib_rows; do
    timeout -k 10 120 python3 tools/kbench_lib.py $K/$l --op resize_normalize --iters 30 | sed "s/^/$l /" || exit 1
  done
  for l in lib lib_wd1 lib_wd2 lib_wd4 lib_ws0 lib_wl0; do
    timeout -k 10 120 python3 tools/kbench_lib.py $K/$l --op warp --only rot15 --iters 30 | sed "s/^/$l /" || exit 1
  done
  for l in lib lib_ts0; do
    timeout -k 10 120 python3 tools/kbench_lib.py $K/$l --op resize --only 1280 --iters 30 --sweep 'RESIZE_STRIP=1,2' | sed "s/^/$l /" || exit 1
  done
done 2>&1 | tee gpurun_out/b_variants.txt
step rows_test
VACV_DIRECT_ROWS_LIB=1 timeout -k 10 200 python3 tools/kbench_lib.py $K/lib_rows --op resize --only 640x360 --iters 10 | sed "s/^/lib_rows /"
step done
