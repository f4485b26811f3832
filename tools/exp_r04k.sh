#!/bin/bash
# Round-4 run 11: Lanczos per-OUT vertical order check; PMC of the two-tap
# strip kernel (1080p -> 1280x720 u8).
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "lanczos" \
    > gpurun_out/k_tests.log 2>&1 || { tail -30 gpurun_out/k_tests.log; exit 1; }
tail -1 gpurun_out/k_tests.log
timeout -k 10 120 python3 tools/kbench.py --op lanczos --iters 30 2>&1 | grep -v amdgpu.ids
timeout -k 10 120 python3 tools/kbench.py --op resize --only 1280 --iters 30 2>&1 | grep -v amdgpu.ids
timeout -s KILL 300 rocprofv3 -i "$R/tools/pmc_bench.txt" -d "$R/gpurun_out/pmc_k_strip" -o pmc --output-format csv \
    -- python3 "$R/tools/kbench.py" --op resize --only 1280 --iters 5 > gpurun_out/pmc_k_strip.log 2>&1 || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc_k_strip resize_strip --out gpurun_out/pmc_k_strip.json > /dev/null || exit 1
python3 - <<'PY'
import json
d=json.load(open('gpurun_out/pmc_k_strip.json')); c=d['counters']; wc=c['SQ_WAVE_CYCLES']
print(d['kernel'], {k: c[k] for k in ['SQ_INSTS_VALU','SQ_INSTS_SALU','SQ_INSTS_LDS','SQ_WAVES','SQ_LDS_BANK_CONFLICT']})
print({k: round(c[k]/wc,3) for k in ['SQ_WAIT_ANY','SQ_WAIT_INST_ANY','SQ_ACTIVE_INST_ANY','SQ_ACTIVE_INST_VALU','SQ_ACTIVE_INST_LDS']}, 'waves/CU', round(wc*4/(c['GRBM_GUI_ACTIVE']/8)/256,1), 'hbm', d['hbm_bytes_per_launch'])
PY
