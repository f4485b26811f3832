#!/bin/bash
# Round-4 run 9: Lanczos with the uniform interior horizontal pass: parity,
# kbench, PMC.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$(pwd)
step() { echo "=== $1 $(date +%T)"; }
step tests
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "lanczos" \
    > gpurun_out/i_tests.log 2>&1 || { tail -30 gpurun_out/i_tests.log; exit 1; }
tail -1 gpurun_out/i_tests.log
step kbench
timeout -k 10 300 python3 tools/kbench.py --op lanczos --iters 30 2>&1 | grep -v amdgpu.ids | tee gpurun_out/i_kbench.jsonl
for W in "lanczos:lanczos_1080p_640x360_u8:lanczos"; do
  op=${W%%:*}; rest=${W#*:}; only=${rest%%:*}; key=${rest#*:}
  step "pmc $key"
  timeout -s KILL 300 rocprofv3 -i "$R/tools/pmc_bench.txt" -d "$R/gpurun_out/pmc_i_$key" -o pmc --output-format csv \
      -- python3 "$R/tools/kbench.py" --op "$op" --only "$only" --iters 5 > "gpurun_out/pmc_i_$key.log" 2>&1 || exit $?
  python3 tools/pmc_summary.py "gpurun_out/pmc_i_$key" "$key" --out "gpurun_out/pmc_i_$key.json" | grep -E "SALU|VALU|WAVE_CYC|GRBM|kernel"
done
step done
