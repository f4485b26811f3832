#!/bin/bash
# Round-5 run d: PMC of warp_exp_kernel vs warp_ring_kernel (720p rot15 u8,
# 128 frames, kbench), one rocprofv3 pass per counter line.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out
i=0
while read -r line; do
  i=$((i+1)); ctrs=${line#pmc: }
  for k in exp ring; do
    if [ $k = ring ]; then export VACV_WARP_KERNEL=6; else unset VACV_WARP_KERNEL; fi
    timeout -s KILL 120 rocprofv3 --pmc $ctrs -d "$R/gpurun_out/pmc_d_$k" -o p$i --output-format csv \
      -- python3 "$R/tools/kbench.py" --op warp --only rot15_u8 --iters 5 > gpurun_out/pmc_d_${k}_$i.log 2>&1 || { tail -5 gpurun_out/pmc_d_${k}_$i.log; exit 1; }
  done
done < tools/pmc_warp3.txt
unset VACV_WARP_KERNEL
python3 tools/pmc_summary.py gpurun_out/pmc_d_exp warp_exp > gpurun_out/pmc_d_exp.json
python3 tools/pmc_summary.py gpurun_out/pmc_d_ring warp_ring > gpurun_out/pmc_d_ring.json
cat gpurun_out/pmc_d_exp.json gpurun_out/pmc_d_ring.json
