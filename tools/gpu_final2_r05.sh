#!/bin/bash
# Round-5 last check at the final head (after the packed area stores): the
# -m gpu suite, smoke(), the headline bench line, kbench --op all.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/r05g_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r05g_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r05g_gpu_tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 200 python3 bench.py --warmup 5 --steps 20 > gpurun_out/r05g_bench_1.json 2>/dev/null || exit 1
cat gpurun_out/r05g_bench_1.json
timeout -k 10 400 python3 tools/kbench.py --op all --iters 30 > gpurun_out/r05g_kbench.jsonl 2> gpurun_out/kbench.err || exit 1
