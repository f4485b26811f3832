#!/bin/bash
# Round-5 run k: yuv_cols_kernel: the yuv / colour tests, then kbench
# yuv_resize default (column kernel) vs VACV_RESIZE_DIRECT=2 (row-major), and
# bench.py --workload yuv_resize with the driver's flags.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -m gpu -k "cvt_color_resize" > gpurun_out/k_tests.log 2>&1 || { tail -60 gpurun_out/k_tests.log; exit 1; }
tail -2 gpurun_out/k_tests.log
for rep in 1 2; do
  timeout -k 10 120 python3 tools/kbench.py --op yuv_resize --iters 30 | sed "s/^/cols /" || exit 1
  VACV_RESIZE_DIRECT=2 timeout -k 10 120 python3 tools/kbench.py --op yuv_resize --iters 30 | sed "s/^/rows /" || exit 1
done 2>&1 | grep -v amdgpu.ids
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --workload yuv_resize --warmup 5 --steps 20 --no-cpu-baseline > gpurun_out/k_bench_yuv_$i.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/k_bench_yuv_$i.json')); print('bench', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
