#!/bin/bash
# Round-4 run 8: PMC passes over kbench for the Lanczos u8 kernel and the warp
# ring kernel (where do their cycles go).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$(pwd)
step() { echo "=== $1 $(date +%T)"; }
for W in "lanczos:lanczos_1080p_640x360_u8:lanczos" "warp:warp_720p_rot15_u8:warp_ring"; do
  op=${W%%:*}; rest=${W#*:}; only=${rest%%:*}; key=${rest#*:}
  step "pmc $key"
  timeout -s KILL 300 rocprofv3 -i "$R/tools/pmc_bench.txt" -d "$R/gpurun_out/pmc_h_$key" -o pmc --output-format csv \
      -- python3 "$R/tools/kbench.py" --op "$op" --only "$only" --iters 5 > "gpurun_out/pmc_h_$key.log" 2>&1 || exit $?
  python3 tools/pmc_summary.py "gpurun_out/pmc_h_$key" "$key" --out "gpurun_out/pmc_h_$key.json" || exit 1
done
step done
