#!/bin/bash
# Round-5 run s: lanczos_u8_kernel variants -- D=8, 8K / 32K tasks, XCD order
# on / off; PMC of the default build.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out
for rep in 1 2; do
  timeout -k 10 150 python3 tools/kbench.py --op lanczos --iters 30 --sweep 'DIRECT_XCD=0,1' | sed "s/^/lib /" || exit 1
  for v in lzr8 lzt8 lzt32; do
    VACV_LIB_DIR=arm-neon-opencv_amd/lib_$v timeout -k 10 150 python3 tools/kbench.py --op lanczos --iters 30 | sed "s/^/$v /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids
P=gpurun_out/pmc_s
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" "FETCH_SIZE" "WRITE_SIZE"; do
  n=$(echo $grp | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$R/$P/$n" -o p --output-format csv \
    -- python3 "$R/tools/kbench.py" --op lanczos --iters 5 --only lanczos_1080p > gpurun_out/pmc_s.log 2>&1 || exit 1
done
python3 tools/pmc_summary.py $P lanczos_u8 > gpurun_out/s_pmc.json || exit 1
cat gpurun_out/s_pmc.json
