#!/bin/bash
# Round-4 run 13: strip kernel with hoisted fetch addresses: tests, A/B of the
# store policy (lib_ss0: write-back) and 128-column strips, same box.
set -o pipefail
export TMPDIR=/tmp
K=arm-neon-opencv_amd
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu -k "resize or strip" \
    > gpurun_out/m_tests.log 2>&1 || { tail -30 gpurun_out/m_tests.log; exit 1; }
tail -1 gpurun_out/m_tests.log
for rep in 1 2 3; do
  for l in lib lib_ss0; do
    timeout -k 10 120 python3 tools/kbench_lib.py $K/$l --op resize --only 1280 --iters 30 | sed "s/^/$l /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids
timeout -k 10 120 python3 tools/kbench.py --op resize --only 1280 --iters 30 --sweep 'RESIZE_STRIP=1,2' 2>&1 | grep -v amdgpu.ids
