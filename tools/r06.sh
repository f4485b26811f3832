#!/bin/bash
# Round-6 GPU runs, one parameterised script (replaces round 5's per-experiment
# tools/exp_r05*.sh launchers).  Run through gpurun from the repo root:
#   tools/r06.sh TAG STEP [STEP ...]
# Steps (each under its own time limit; the script stops at the first failure):
#   tests            the -m gpu suite (+ smoke)
#   kbench:OP[:ONLY] tools/kbench.py --op OP [--only ONLY] --iters 30
#   sweep:OP:ONLY:SW tools/kbench.py sweep of tuning knobs SW ('K=a,b;K2=c')
#   bench:WL         bench.py --workload WL --warmup 5 --steps 20 (driver flags)
#   stats:WL         rocprofv3 --kernel-trace --stats over that bench command
#   kstats:OP:ONLY   rocprofv3 --kernel-trace --stats over kbench
#   pmc:WL:KEY       PMC passes (tools/pmc_bench.txt) over bench.py WL, kernel KEY
#   kpmc:OP:ONLY:KEY PMC passes over kbench
#   lib:DIR          run the following steps on lib variant DIR (VACV_LIB_DIR)
#   clocks:OP:ONLY[:ITERS]  kbench twice with rocm-smi sclk / power sampled beside it
# Output: gpurun_out/${TAG}_*.  Only gpurun_out/ travels back.
set -o pipefail
T=$1; shift
R=$(pwd)
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
say() { echo "=== $T $1 $(date +%T)"; }
for S in "$@"; do
  IFS=: read -r kind a b c <<< "$S"
  say "$S"
  case $kind in
    tests)
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread ${a:+-k "$a"} \
          > "gpurun_out/${T}_gpu_tests.log" 2>&1 || { tail -40 "gpurun_out/${T}_gpu_tests.log"; exit 1; }
      tail -2 "gpurun_out/${T}_gpu_tests.log"
      timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    kbench)
      timeout -k 10 400 python3 tools/kbench.py --op "$a" ${b:+--only "$b"} --iters 30 \
          >> "gpurun_out/${T}_kbench.jsonl" 2>> "gpurun_out/${T}_kbench.err" || { tail -20 "gpurun_out/${T}_kbench.err"; exit 1; }
      tail -n 30 "gpurun_out/${T}_kbench.jsonl" | cut -c1-220 ;;
    sweep)
      timeout -k 10 400 python3 tools/kbench.py --op "$a" --only "$b" --iters 30 --sweep "$c" \
          >> "gpurun_out/${T}_sweep.jsonl" 2>> "gpurun_out/${T}_sweep.err" || { tail -20 "gpurun_out/${T}_sweep.err"; exit 1; }
      tail -n 12 "gpurun_out/${T}_sweep.jsonl" | cut -c1-260 ;;
    bench)
      timeout -k 10 300 python3 bench.py --workload "$a" --warmup 5 --steps 20 ${b:+$b} \
          > "gpurun_out/${T}_bench_$a.json" 2> "gpurun_out/${T}_bench_$a.err" || { tail -20 "gpurun_out/${T}_bench_$a.err"; exit 1; }
      cut -c1-1200 "gpurun_out/${T}_bench_$a.json" ;;
    stats)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${T}_prof_$a" -o s --output-format csv \
          -- python3 "$R/bench.py" --workload "$a" --warmup 5 --steps 20 --no-cpu-baseline \
          > "gpurun_out/${T}_prof_$a.log" 2>&1 || exit $?
      find "gpurun_out/${T}_prof_$a" -name "*kernel_stats.csv" -exec cp {} "gpurun_out/${T}_bench_${a}_kernel_stats.csv" \;
      head -4 "gpurun_out/${T}_bench_${a}_kernel_stats.csv" | cut -c1-250 ;;
    kstats)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${T}_kprof_$b" -o s --output-format csv \
          -- python3 "$R/tools/kbench.py" --op "$a" --only "$b" --iters 30 > "gpurun_out/${T}_kprof_$b.log" 2>&1 || exit $?
      find "gpurun_out/${T}_kprof_$b" -name "*kernel_stats.csv" -exec cp {} "gpurun_out/${T}_kbench_${b}_kernel_stats.csv" \;
      head -4 "gpurun_out/${T}_kbench_${b}_kernel_stats.csv" | cut -c1-250 ;;
    pmc)
      timeout -s KILL 400 rocprofv3 -i "$R/tools/pmc_bench.txt" -d "$R/gpurun_out/${T}_pmc_$a" -o pmc --output-format csv \
          -- python3 "$R/bench.py" --workload "$a" --steps 5 --warmup 2 --no-cpu-baseline > "gpurun_out/${T}_pmc_$a.log" 2>&1 || exit $?
      python3 tools/pmc_summary.py "gpurun_out/${T}_pmc_$a" "$b" --out "gpurun_out/${T}_pmc_$a.json" \
          > "gpurun_out/${T}_pmc_${a}_summary.txt" || exit 1
      cp "gpurun_out/${T}_pmc_$a.json" "profiles/pmc_$a.json"  # later bench steps of this call read it
      cat "gpurun_out/${T}_pmc_${a}_summary.txt" | cut -c1-200 ;;
    kpmc)
      timeout -s KILL 300 rocprofv3 -i "$R/tools/pmc_bench.txt" -d "$R/gpurun_out/${T}_kpmc_$c" -o pmc --output-format csv \
          -- python3 "$R/tools/kbench.py" --op "$a" --only "$b" --iters 5 > "gpurun_out/${T}_kpmc_$c.log" 2>&1 || exit $?
      python3 tools/pmc_summary.py "gpurun_out/${T}_kpmc_$c" "$c" --out "gpurun_out/${T}_kpmc_$c.json" \
          > "gpurun_out/${T}_kpmc_${c}_summary.txt" || exit 1
      cat "gpurun_out/${T}_kpmc_${c}_summary.txt" | cut -c1-200 ;;
    lib)
      export VACV_LIB_DIR="$R/arm-neon-opencv_amd/$a" ;;
    clocks)
      # kbench OP:ONLY twice with rocm-smi's sclk / power sampled beside it
      ( while true; do date +%T.%N; rocm-smi --showclocks --showpower 2>/dev/null | grep -E "sclk|mclk|Power"; sleep 0.2; done ) \
          > "gpurun_out/${T}_clocks_$b.txt" 2>&1 &
      SMI=$!
      for i in 1 2; do
        timeout -k 10 300 python3 tools/kbench.py --op "$a" --only "$b" --iters "${c:-30}" >> "gpurun_out/${T}_clocks_$b.jsonl" 2>> "gpurun_out/${T}_kbench.err" \
            || { kill $SMI; exit 1; }
        sleep 1
      done
      kill $SMI; wait $SMI 2>/dev/null
      cat "gpurun_out/${T}_clocks_$b.jsonl" | cut -c1-200 ;;
    *) echo "unknown step $S"; exit 2 ;;
  esac
done
say done
