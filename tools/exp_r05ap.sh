#!/bin/bash
# Round-5 run ap: match_template -- integral column pass with 16 rows of loads
# in flight; match tests, kbench, rocprof per-kernel times of the match ops.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -m gpu -k "match" > gpurun_out/ap_tests.log 2>&1 || { tail -60 gpurun_out/ap_tests.log; exit 1; }
tail -2 gpurun_out/ap_tests.log
timeout -k 10 150 python3 tools/kbench.py --op match --iters 20 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_ap" -o ap --output-format csv \
    -- python3 "$R/tools/kbench.py" --op match --iters 10 > gpurun_out/prof_ap.log 2>&1 || exit 1
find gpurun_out/prof_ap -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-160 | head -12
