#!/bin/bash
# Round-5 run ak: the headline, output stores sc1|nt (lib_sa18) and gathers
# sc1|nt (lib_cl18) against the product (nt gathers, nt stores): kbench and
# the 20-step bench, interleaved.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for v in lib lib_sa18 lib_cl18; do
    VACV_LIB_DIR=arm-neon-opencv_amd/$v timeout -k 10 150 python3 tools/kbench.py --op resize_normalize --iters 40 | sed "s/^/$v /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids
for v in lib lib_sa18 lib_cl18 lib lib_sa18 lib_cl18; do
  VACV_LIB_DIR=arm-neon-opencv_amd/$v timeout -k 10 200 python3 bench.py --warmup 5 --steps 20 --no-cpu-baseline > gpurun_out/ak_b.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ak_b.json')); print('$v bench', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
