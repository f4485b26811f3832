set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$(pwd)
A=arm-neon-opencv_amd
timeout -k 10 200 python3 tools/kbench.py --op resize --only 1280x720 --iters 30 --sweep 'RESIZE_STRIP=1,2' > gpurun_out/d1_strip.jsonl 2>&1 || exit $?
for d in 1 2 3; do timeout -k 10 200 python3 tools/kbench_lib.py $A/lib_sdbg$d --op resize --only 1280x720 --iters 30 | sed "s/^/sdbg$d /" >> gpurun_out/d1_strip.jsonl || exit $?; done
timeout -k 10 200 python3 tools/kbench.py --op resize_other --only area --iters 30 > gpurun_out/d1_area.jsonl 2>&1 || exit $?
for d in 1 2 3; do timeout -k 10 200 python3 tools/kbench_lib.py $A/lib_adbg$d --op resize_other --only area --iters 30 | sed "s/^/adbg$d /" >> gpurun_out/d1_area.jsonl || exit $?; done
timeout -k 10 300 rocprofv3 -i "$R/tools/pmc_strip2.txt" -d "$R/gpurun_out/pmc_d1area" -o pmc --output-format csv -- python3 "$R/tools/kbench.py" --op resize_other --only area_1080p_960 --iters 5 > gpurun_out/pmc_d1area.log 2>&1 || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc_d1area area_u8_colsum > gpurun_out/pmc_d1area.txt || exit 1
timeout -k 10 300 rocprofv3 -i "$R/tools/pmc_strip2.txt" -d "$R/gpurun_out/pmc_d1strip" -o pmc --output-format csv -- python3 "$R/tools/kbench.py" --op resize --only 1280x720 --iters 5 > gpurun_out/pmc_d1strip.log 2>&1 || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc_d1strip resize_strip > gpurun_out/pmc_d1strip.txt || exit 1
cat gpurun_out/d1_strip.jsonl gpurun_out/d1_area.jsonl
