#!/bin/bash
# Round-5 run p: Lanczos XCD-contiguous block order (DIRECT_XCD sweep) and
# rows in flight (D = 2 / 3 / 4 libraries); Lanczos tests; FETCH of both orders.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
    -m gpu -k "lanczos" > gpurun_out/p_tests.log 2>&1 || { tail -60 gpurun_out/p_tests.log; exit 1; }
tail -2 gpurun_out/p_tests.log
for rep in 1 2; do
  timeout -k 10 150 python3 tools/kbench.py --op lanczos --iters 30 --sweep 'DIRECT_XCD=0,1' | sed "s/^/d3 /" || exit 1
  for d in 2 4; do
    VACV_LIB_DIR=arm-neon-opencv_amd/lib_lzd$d timeout -k 10 150 python3 tools/kbench.py --op lanczos --iters 30 | sed "s/^/d$d /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids
for x in 0 1; do
  VACV_DIRECT_XCD=$x timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmc_p$x" -o p --output-format csv \
    -- python3 "$R/tools/kbench.py" --op lanczos --iters 5 --only lanczos_1080p > gpurun_out/pmc_p.log 2>&1 || exit 1
  python3 tools/pmc_summary.py gpurun_out/pmc_p$x lanczos | grep -E "fetch_bytes" | sed "s/^/xcd$x /"
done
