#!/bin/bash
# Round-5 run o: yuv_cols_kernel with a whole row group per workgroup: yuv
# tests, kbench yuv_resize, bench.py --workload yuv_resize, FETCH/WRITE.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -m gpu -k "cvt_color_resize" > gpurun_out/o_tests.log 2>&1 || { tail -60 gpurun_out/o_tests.log; exit 1; }
tail -2 gpurun_out/o_tests.log
for rep in 1 2; do
  timeout -k 10 120 python3 tools/kbench.py --op yuv_resize --iters 30 | sed "s/^/cols /" || exit 1
done 2>&1 | grep -v amdgpu.ids
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --workload yuv_resize --warmup 5 --steps 20 --no-cpu-baseline > gpurun_out/o_bench_yuv_$i.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/o_bench_yuv_$i.json')); print('bench', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d "$R/gpurun_out/pmc_o" -o p_$c --output-format csv \
    -- python3 "$R/bench.py" --workload yuv_resize --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pmc_o.log 2>&1 || exit 1
done
python3 tools/pmc_summary.py gpurun_out/pmc_o yuv_cols | grep -E "fetch_bytes|write_bytes|yuv_cols"
