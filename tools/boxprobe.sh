#!/bin/bash
# One box's clocks and the two reference kernels, for the warp_affine_normalize
# box-to-box spread: rocm-smi's clock table once, then
# tools/r06.sh clocks steps (sclk / power sampled beside kbench).
#   tools/boxprobe.sh TAG
set -o pipefail
T=$1
mkdir -p gpurun_out
timeout -k 5 30 rocm-smi --showclocks --showpower --showmaxpower > "gpurun_out/${T}_smi.txt" 2>&1
grep -E "clock level|Power" "gpurun_out/${T}_smi.txt" | head -20
bash tools/r06.sh "$T" clocks:warp:warp_normalize_720p_rot15:3000 clocks:resize_normalize:resize_normalize_1080p_640x360:6000 \
    clocks:warp:warp_720p_rot15_u8:6000
