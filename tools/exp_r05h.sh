#!/bin/bash
# Round-5 run h: the whole -m gpu suite at the warp_exp_kernel head, then
# bench.py --workload warp (driver flags) with exp vs ring, twice, and the
# DPP-store variant (lib_x0) in kbench.
set -o pipefail
export TMPDIR=/tmp
K=arm-neon-opencv_amd
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/h_gpu_tests.log 2>&1 || { tail -40 gpurun_out/h_gpu_tests.log; exit 1; }
tail -2 gpurun_out/h_gpu_tests.log
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --workload warp --warmup 5 --steps 20 --no-cpu-baseline > gpurun_out/h_bench_warp_exp_$i.json 2>/dev/null || exit 1
  VACV_WARP_KERNEL=6 timeout -k 10 200 python3 bench.py --workload warp --warmup 5 --steps 20 --no-cpu-baseline > gpurun_out/h_bench_warp_ring_$i.json 2>/dev/null || exit 1
done
for f in gpurun_out/h_bench_warp_*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"; done
for rep in 1 2; do
  timeout -k 10 120 python3 tools/kbench.py --op warp --only rot15_u8 --iters 30 | sed "s/^/exp /" || exit 1
  timeout -k 10 120 python3 tools/kbench_lib.py $K/lib_x0 --op warp --only rot15_u8 --iters 30 | sed "s/^/exp_x0 /" || exit 1
done 2>&1 | grep -v amdgpu.ids | grep -v nearest
