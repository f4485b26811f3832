#!/bin/bash
# Round-5 run ai: headline tap-gather cache policy (VACV_DIRECT_LAUX: 0 default
# (product), 1 sc0, 2 nt, 3 sc0|nt) now that no source line is shared between
# column blocks; kbench + the 20-step bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for v in lib lib_la2 lib_la1 lib_la3; do
    VACV_LIB_DIR=arm-neon-opencv_amd/$v timeout -k 10 150 python3 tools/kbench.py --op resize_normalize --iters 40 | sed "s/^/$v /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids
for v in lib lib_la2 lib lib_la2; do
  VACV_LIB_DIR=arm-neon-opencv_amd/$v timeout -k 10 200 python3 bench.py --warmup 5 --steps 20 --no-cpu-baseline > gpurun_out/ai_b.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ai_b.json')); print('$v bench', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
