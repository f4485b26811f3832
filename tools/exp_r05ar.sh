#!/bin/bash
# Round-5 run ar: cfg5 cubic_cols_kernel tap loads default policy (lib_cl0) and
# output stores sc1|nt (lib_cs18) vs the product (nt / nt): kbench + cfg5 bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for v in lib lib_cl0 lib_cs18; do
    VACV_LIB_DIR=arm-neon-opencv_amd/$v timeout -k 10 150 python3 tools/kbench.py --op cubic --iters 40 | sed "s/^/$v /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids
for v in lib lib_cl0 lib_cs18 lib lib_cl0 lib_cs18; do
  VACV_LIB_DIR=arm-neon-opencv_amd/$v timeout -k 10 200 python3 bench.py --workload cubic_stats --warmup 5 --steps 20 --no-cpu-baseline > gpurun_out/ar_b.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ar_b.json')); print('$v bench', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
