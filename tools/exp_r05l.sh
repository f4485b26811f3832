#!/bin/bash
# Round-5 run l: headline resize_cols_kernel with 128-column blocks (CW = 2):
# resize tests, kbench resize_normalize CW=2 (default) vs 64-column blocks,
# the driver-flag bench twice, and the FETCH / WRITE counters.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -m gpu -k "resize_normalize or resize_linear or resize_full or random_geometry" > gpurun_out/l_tests.log 2>&1 || { tail -60 gpurun_out/l_tests.log; exit 1; }
tail -2 gpurun_out/l_tests.log
for rep in 1 2; do
  timeout -k 10 120 python3 tools/kbench.py --op resize_normalize --iters 30 | sed "s/^/cw2 /" || exit 1
  VACV_RESIZE_TILE_W=64 timeout -k 10 120 python3 tools/kbench.py --op resize_normalize --iters 30 | sed "s/^/cw1 /" || exit 1
done 2>&1 | grep -v amdgpu.ids
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --warmup 5 --steps 20 --no-cpu-baseline > gpurun_out/l_bench_$i.json 2>/dev/null || exit 1
  VACV_RESIZE_TILE_W=64 timeout -k 10 200 python3 bench.py --warmup 5 --steps 20 --no-cpu-baseline > gpurun_out/l_bench64_$i.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/l_bench_$i.json')); e=json.load(open('gpurun_out/l_bench64_$i.json')); print('bench cw2', d['roofline']['kernel_ms'], d['roofline']['frac'], 'cw1', e['roofline']['kernel_ms'], e['roofline']['frac'])"
done
for k in cw2 cw1; do
  if [ $k = cw1 ]; then export VACV_RESIZE_TILE_W=64; else unset VACV_RESIZE_TILE_W; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c -d "$R/gpurun_out/pmc_l_$k" -o p_$c --output-format csv \
      -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pmc_l_$k.log 2>&1 || exit 1
  done
  python3 tools/pmc_summary.py gpurun_out/pmc_l_$k resize_cols | grep -E "fetch_bytes|write_bytes|resize_cols"
done
