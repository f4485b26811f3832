#!/bin/bash
# VGPR / spill / SGPR / static-LDS counts of the gfx950 kernels in a built
# object (its .hip_fatbin):
#   tools/kregs.sh arm-neon-opencv_amd/build/k_warp_frames.o [kernel-regex]
set -e
O=$1; K=${2:-.}
T=$(mktemp -d)
objcopy --dump-section .hip_fatbin="$T/fb.bin" "$O" "$T/tmp.o"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input="$T/fb.bin" \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output="$T/dev.co"
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$T/dev.co" | \
    awk -v k="$K" '/\.name:/ {n=$2} /\.vgpr_count:/ {v=$2} /\.vgpr_spill_count:/ {sp=$2} /\.sgpr_count:/ {sg=$2}
         /\.group_segment_fixed_size:/ {l=$2}
         /\.wavefront_size:/ { if (n ~ k) printf "%-80s vgpr %s spill %s sgpr %s lds %s\n", substr(n,1,80), v, sp, sg, l }'
rm -rf "$T"
