#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 600 python -u -m pytest tests/test_gpu_pairgram.py -k 'fused or compact' -x -q --timeout 120 --timeout-method thread > gpurun_out/r06/fused_tests2.log 2>&1" \
  "KNOB=fused timeout -k 10 300 python tools/ab_gram_stages.py 50 100 200 > gpurun_out/r06/gram_fused_ab2.jsonl" \
  "timeout -k 10 300 python tools/time_krum_devsel.py > gpurun_out/r06/krum_devsel_warm2.txt 2>&1" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/prof_fused2 -o run --output-format csv -- python tools/time_krum_devsel.py > gpurun_out/r06/krum_devsel_traced2.txt 2>&1"
