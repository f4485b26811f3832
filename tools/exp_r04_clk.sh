set -o pipefail
mkdir -p gpurun_out
( for i in $(seq 1 40); do echo "t=$(date +%s.%N)"; rocm-smi --showclocks --showpower --showtemp 2>/dev/null | grep -E "sclk|Power|Temperature|fclk|mclk" ; sleep 0.2; done ) > gpurun_out/clk.log 2>&1 &
P=$!
sleep 2
timeout -k 10 120 python3 bench.py --workload warp --warmup 5 --steps 20000 --no-cpu-baseline > gpurun_out/clk_bench_warp.json 2>gpurun_out/clk_bench_warp.err
rc=$?
sleep 1
timeout -k 10 120 python3 bench.py --warmup 5 --steps 15000 --no-cpu-baseline > gpurun_out/clk_bench_head.json 2>gpurun_out/clk_bench_head.err
wait $P
cat gpurun_out/clk_bench_warp.json gpurun_out/clk_bench_head.json
exit $rc
