#!/bin/bash
# Round-5 run aj: the headline with non-temporal gathers (product now) --
# resize tests; output-store policy variants (VACV_DIRECT_SAUX: 2 nt (product),
# 3 sc0|nt, 18 sc1|nt, 0 default); kbench + the 20-step bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -m gpu -k "resize_normalize or linear" > gpurun_out/aj_tests.log 2>&1 || { tail -60 gpurun_out/aj_tests.log; exit 1; }
tail -2 gpurun_out/aj_tests.log
for rep in 1 2; do
  for v in lib lib_sa3 lib_sa18 lib_sa0; do
    VACV_LIB_DIR=arm-neon-opencv_amd/$v timeout -k 10 150 python3 tools/kbench.py --op resize_normalize --iters 40 | sed "s/^/$v /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids
for v in lib lib_sa3 lib lib_sa3; do
  VACV_LIB_DIR=arm-neon-opencv_amd/$v timeout -k 10 200 python3 bench.py --warmup 5 --steps 20 --no-cpu-baseline > gpurun_out/aj_b.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/aj_b.json')); print('$v bench', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
