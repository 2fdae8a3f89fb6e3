#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 600 python -u -m pytest tests/test_gpu_pairgram.py tests/test_gpu_golden.py tests/test_gpu_fullsize.py tests/test_gpu_pairsel.py tests/test_krum_certify.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06/graph_tests.log 2>&1" \
  "timeout -k 10 500 python -u tools/bench_robust.py dropin dropin_fresh > gpurun_out/r06/dropin3.jsonl" \
  "timeout -k 10 300 python tools/time_krum_phases.py > gpurun_out/r06/krum_phases3.txt 2>&1" \
  "FRESH=1 timeout -k 10 300 python tools/time_krum_phases.py > gpurun_out/r06/krum_phases3_fresh.txt 2>&1" \
  "timeout -k 10 300 python tools/probe_upload_cost.py > gpurun_out/r06/upload_cost3.json"
