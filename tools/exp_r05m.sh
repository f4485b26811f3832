#!/bin/bash
# Round-5 run m: warp_exp_kernel phase clocks (VACV_RING_DBG=16 build) for
# bilinear, nearest and normalised output at 720p rot 15 x128.
set -o pipefail
export TMPDIR=/tmp
K=arm-neon-opencv_amd
mkdir -p gpurun_out
for kind in linear nearest normalize; do
  timeout -k 10 120 python3 tools/warp_prof.py $K/lib_dbg16 15 $kind > gpurun_out/prof_m_$kind.txt 2>&1 || exit 1
  echo "== $kind"; grep expprof gpurun_out/prof_m_$kind.txt | tail -6
done
