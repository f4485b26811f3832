#!/bin/bash
# Round-5 run w: warp_exp_kernel image rows at their columns' unit parity
# (LDS banks independent of the source row): warp tests, kbench, bank conflicts.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -m gpu -k "warp" > gpurun_out/w_tests.log 2>&1 || { tail -60 gpurun_out/w_tests.log; exit 1; }
tail -2 gpurun_out/w_tests.log
for rep in 1 2; do
  timeout -k 10 150 python3 tools/kbench.py --op warp --iters 30 | sed "s/^/lib /" || exit 1
done 2>&1 | grep -v amdgpu.ids
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES -d "$R/gpurun_out/pmc_w" -o p --output-format csv \
    -- python3 "$R/tools/kbench.py" --op warp --iters 5 --only rot15_u8 > gpurun_out/pmc_w.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_w warp_exp
