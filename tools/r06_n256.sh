#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 600 python -u -m pytest tests/test_gpu_pairgram.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06/pairgram_tests_n256.log 2>&1" \
  "timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/prof_krum_large -o run --output-format csv -- python tools/bench_robust.py krum_large > gpurun_out/r06/krum_large.jsonl" \
  "timeout -k 10 300 python tools/time_krum_phases.py > gpurun_out/r06/krum_phases.txt 2>&1" \
  "FRESH=1 timeout -k 10 300 python tools/time_krum_phases.py > gpurun_out/r06/krum_phases_fresh.txt 2>&1"
