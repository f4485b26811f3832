#!/bin/bash
# Round-5 run al: yuv gathers non-temporal (lib_yl2) vs default (lib) now that
# yuv_cols_kernel's blocks are line-exact; kbench + the 20-step yuv bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for v in lib lib_yl2; do
    VACV_LIB_DIR=arm-neon-opencv_amd/$v timeout -k 10 150 python3 tools/kbench.py --op yuv_resize --iters 40 | sed "s/^/$v /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids
for v in lib lib_yl2 lib lib_yl2; do
  VACV_LIB_DIR=arm-neon-opencv_amd/$v timeout -k 10 200 python3 bench.py --workload yuv_resize --warmup 5 --steps 20 --no-cpu-baseline > gpurun_out/al_b.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/al_b.json')); print('$v bench', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
