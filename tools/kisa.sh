#!/bin/bash
# Disassembly of the gfx950 kernels in a built object (its .hip_fatbin),
# optionally only the kernels whose symbol matches a regex:
#   tools/kisa.sh arm-neon-opencv_amd/build/k_resize_direct.o [symbol-regex] > out.s
set -e
O=$1; K=${2:-.}
T=$(mktemp -d)
objcopy --dump-section .hip_fatbin="$T/fb.bin" "$O" "$T/tmp.o"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input="$T/fb.bin" \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output="$T/dev.co"
/opt/rocm/lib/llvm/bin/llvm-objdump -d --no-show-raw-insn --symbolize-operands "$T/dev.co" | \
    awk -v k="$K" '/^[0-9a-f]+ <_Z[^>]*>:$/ { on = ($0 ~ k) } on'
rm -rf "$T"
