#!/bin/bash
# Round-5 run x: fp32 colour / dtype output stores, non-temporal (lib) vs the
# default policy (lib_cwb); cfg3 bench both ways.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for v in lib lib_cwb; do
    VACV_LIB_DIR=arm-neon-opencv_amd/$v timeout -k 10 150 python3 tools/kbench.py --op cvt --iters 20 | sed "s/^/$v /" || exit 1
    VACV_LIB_DIR=arm-neon-opencv_amd/$v timeout -k 10 150 python3 tools/kbench.py --op dtype --iters 20 | sed "s/^/$v /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids
for v in lib lib_cwb; do
  VACV_LIB_DIR=arm-neon-opencv_amd/$v timeout -k 10 200 python3 bench.py --workload cvt_normalize --warmup 5 --steps 20 --no-cpu-baseline > gpurun_out/x_bench_$v.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/x_bench_$v.json')); print('$v bench', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
