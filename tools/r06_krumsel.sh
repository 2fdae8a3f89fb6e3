#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 600 python -u -m pytest tests/test_gpu_krumsel.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06/krumsel_tests.log 2>&1" \
  "timeout -k 10 300 python tools/time_krum_phases.py > gpurun_out/r06/krum_phases_warm4.txt 2>&1" \
  "FRESH=1 timeout -k 10 300 python tools/time_krum_phases.py > gpurun_out/r06/krum_phases_fresh4.txt 2>&1" \
  "timeout -k 10 400 python tools/bench_robust.py dropin dropin_fresh > gpurun_out/r06/dropin_krumsel2.jsonl 2> gpurun_out/r06/dropin_krumsel2.log"
