#!/bin/bash
# Round-5 run ah: FETCH / WRITE of warp_exp_kernel with 64 x 32 and 128 x 16 tiles.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out
for tw in 64 128; do
  for c in FETCH_SIZE WRITE_SIZE; do
    VACV_RESIZE_TILE_W=$tw timeout -s KILL 120 rocprofv3 --pmc $c -d "$R/gpurun_out/pmc_ah$tw" -o p_$c --output-format csv \
      -- python3 "$R/tools/kbench.py" --op warp --iters 5 --only rot15_u8 > gpurun_out/pmc_ah.log 2>&1 || exit 1
  done
  python3 tools/pmc_summary.py gpurun_out/pmc_ah$tw warp_exp | grep -E "kernel<|fetch_bytes_corrected|write_bytes" | sed "s/^/tw$tw /"
done
