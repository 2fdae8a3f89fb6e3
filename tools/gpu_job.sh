#!/bin/bash
# Round-trip job for one gpurun call.  Each GPU step has its own time limit;
# after a crash-class exit (timeout 124/137, abort 134, segfault 139, ...)
# nothing further touches the GPU.  A plain pytest failure (rc 1) continues.
set -u
mkdir -p gpurun_out
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  local t0=$(date +%s)
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc $(( $(date +%s) - t0 ))s" | tee -a gpurun_out/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after $name (rc=$rc)" | tee -a gpurun_out/steps.log
    exit $rc
  fi
  return 0
}
i=0
for step in "$@"; do
  i=$((i+1))
  case $step in
    smoke) run smoke 240 python __graft_entry__.py smoke ;;
    pytest) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    pytestall) run pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ;;
    bench) run bench 420 python bench.py ;;
    *) echo "step$i: $step" >> gpurun_out/steps.log; run "step$i" 600 bash -c "$step" ;;
  esac
done
