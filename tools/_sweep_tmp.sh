set -e
for L in lib lib_nt lib_st; do
  VACV_HIP_LIB=$PWD/arm-neon-opencv_amd/$L/libvacv_hip.so timeout -k 10 200 python tools/kbench.py --op resize_normalize --iters 20 --sweep "VACV_RESIZE_WGS=2048,1000000000;VACV_RESIZE_TILE_H=0,1,2,4" | sed "s/^/$L /"
done
