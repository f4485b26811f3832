#!/bin/bash
# Round-5 run ag: warp_exp_kernel 128 x 16 tiles (VACV_RESIZE_TILE_W=128,
# whole-line u8 output rows) -- warp tests on it, kbench and WRITE_SIZE both ways.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out
VACV_RESIZE_TILE_W=128 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -m gpu -k "warp" > gpurun_out/ag_tests.log 2>&1 || { tail -60 gpurun_out/ag_tests.log; exit 1; }
tail -2 gpurun_out/ag_tests.log
for rep in 1 2; do
  timeout -k 10 150 python3 tools/kbench.py --op warp --iters 30 --sweep 'RESIZE_TILE_W=64,128' || exit 1
done 2>&1 | grep -v amdgpu.ids | grep "rot15\|rot45\|rot0"
for tw in 64 128; do
  VACV_RESIZE_TILE_W=$tw timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE -d "$R/gpurun_out/pmc_ag$tw" -o p --output-format csv \
    -- python3 "$R/tools/kbench.py" --op warp --iters 5 --only rot15_u8 > gpurun_out/pmc_ag.log 2>&1 || exit 1
  python3 tools/pmc_summary.py gpurun_out/pmc_ag$tw warp_exp | grep -E "kernel<|fetch_bytes|write_bytes" | sed "s/^/tw$tw /"
done
