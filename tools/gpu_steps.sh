#!/bin/bash
# Run GPU steps in order, each under its own time limit.  A step that ends in
# a fault / abort / segfault / timeout (124, 134, 137, 139, or a signal) stops
# the script; an ordinary failure (e.g. a failing test, rc 1) is recorded and
# the next step runs.
#   usage: tools/gpu_steps.sh "<seconds>|<name>|<command>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
status=0
for spec in "$@"; do
  secs="${spec%%|*}"; rest="${spec#*|}"; name="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] $(date +%T) timeout ${secs}s: $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc $(date +%T)"
  tail -n 25 "gpurun_out/$name.log"
  case $rc in
    0) ;;
    124|134|137|139) echo "=== [$name] fatal rc=$rc: stopping"; exit $rc ;;
    *) if [ $rc -gt 128 ]; then echo "=== [$name] signal rc=$rc: stopping"; exit $rc; fi; status=1 ;;
  esac
done
exit $status
