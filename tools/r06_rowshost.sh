#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 600 python -u -m pytest tests/test_gpu_rows.py tests/test_gpu_golden.py tests/test_gpu_fullsize.py tests/test_gpu_pairsel.py tests/test_gpu_world2.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06/rowshost_tests.log 2>&1" \
  "timeout -k 10 300 python tools/time_krum_phases.py > gpurun_out/r06/krum_phases_warm2.txt 2>&1" \
  "FRESH=1 timeout -k 10 300 python tools/time_krum_phases.py > gpurun_out/r06/krum_phases_fresh2.txt 2>&1" \
  "timeout -k 10 400 python tools/bench_robust.py dropin dropin_fresh > gpurun_out/r06/dropin_rowshost.jsonl 2> gpurun_out/r06/dropin_rowshost.log"
