#!/bin/bash
# Variant builds of libvacv_hip.so for A/B runs on the GPU (tools/kbench_lib.py):
# each reuses the main build's objects and recompiles only the named sources
# with extra flags.
#   tools/variants.sh <name> "<sources without .hip>" "<EXTRA flags>"
# e.g. tools/variants.sh s0 "k_resize_strip" "-DVACV_STRIP_AUX=2"
#   -> arm-neon-opencv_amd/lib_d1/libvacv_hip.so
set -e
N=$1; SRCS=$2; X=$3
P=$(cd "$(dirname "$0")/../arm-neon-opencv_amd" && pwd)
rm -rf "$P/build_$N" "$P/lib_$N"
mkdir -p "$P/build_$N" "$P/lib_$N"
cp "$P"/build/*.o "$P/build_$N/"
for s in $SRCS; do rm -f "$P/build_$N/$s.o"; done
make -s -C "$P" OBJ="$P/build_$N" LIB="$P/lib_$N" EXTRA="$X" "$P/lib_$N/libvacv_hip.so"
echo "built lib_$N ($X)"
