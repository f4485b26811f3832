#!/bin/bash
# Round-5 run e: warp_exp_kernel with the quarter-unit re-lay: warp tests,
# kbench exp vs ring, and the LDS counters of exp.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -m gpu -k "warp" > gpurun_out/e_tests.log 2>&1 || { tail -60 gpurun_out/e_tests.log; exit 1; }
tail -2 gpurun_out/e_tests.log
for rep in 1 2; do
  timeout -k 10 120 python3 tools/kbench.py --op warp --iters 30 | sed "s/^/exp /" || exit 1
  VACV_WARP_KERNEL=6 timeout -k 10 120 python3 tools/kbench.py --op warp --iters 30 | sed "s/^/ring /" || exit 1
done 2>&1 | grep -v amdgpu.ids | grep -v nearest
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES \
  -d "$R/gpurun_out/pmc_e" -o p --output-format csv -- python3 "$R/tools/kbench.py" --op warp --only rot15_u8 --iters 5 > gpurun_out/pmc_e.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_e warp_exp
