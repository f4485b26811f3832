set -e
export TMPDIR=/tmp
R=$(pwd)
for ROWS in 1; do
  VACV_RESIZE_ROWS=$ROWS timeout -k 10 200 rocprofv3 -i $R/tools/pmc_resize.txt -d $R/gpurun_out/pmc_rowsB$ROWS -o p --output-format csv -- python3 $R/tools/kbench.py --op resize_normalize --iters 5 > gpurun_out/pmc_rowsB$ROWS.log 2>&1
  python3 tools/pmc_summary.py gpurun_out/pmc_rowsB$ROWS resize > gpurun_out/pmc_rowsB$ROWS.txt
done
