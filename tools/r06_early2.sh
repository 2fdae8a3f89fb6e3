#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
bash tools/gpu_job.sh \
  "timeout -k 10 600 python -u -m pytest tests/test_gpu_pairgram.py -k 'compact' -x -q --timeout 120 --timeout-method thread > gpurun_out/r06/early2_tests.log 2>&1" \
  "MODES=2,1 timeout -k 10 300 python tools/ab_gram_stages.py 66 80 100 112 > gpurun_out/r06/gram_early_nt7_ab.jsonl"
