#!/bin/bash
# Round-4 run 17: Lanczos walk with a store per step (counted waits) vs the
# previous head (lib_hd), same box; all Lanczos parity tests.
set -o pipefail
export TMPDIR=/tmp
K=arm-neon-opencv_amd
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_parity.py tests/test_oracle.py -x -q --timeout 200 --timeout-method thread -k "lanczos" > gpurun_out/s_tests.log 2>&1 || { tail -20 gpurun_out/s_tests.log; exit 1; }
tail -1 gpurun_out/s_tests.log
for rep in 1 2 3; do
  for l in lib lib_hd; do
    timeout -k 10 120 python3 tools/kbench_lib.py $K/$l --op lanczos --iters 30 | sed "s/^/$l /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids
