#!/bin/bash
# Round-5 run n: warp_exp_kernel output store cache policy: nt (default) vs
# write-back (lib_sa0) vs sc0 (lib_sa1), u8 / nearest / normalised.
set -o pipefail
export TMPDIR=/tmp
K=arm-neon-opencv_amd
for rep in 1 2; do
  for l in lib lib_sa0 lib_sa1; do
    timeout -k 10 120 python3 tools/kbench_lib.py $K/$l --op warp --only rot15 --iters 30 | sed "s/^/$l /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids
