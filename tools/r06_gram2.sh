#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_pairgram.py -x -q --timeout 120 --timeout-method thread -k 'compact or settings or flags' > gpurun_out/r06/pairgram_tests2.log 2>&1" \
  "timeout -k 10 300 python tools/ab_gram_stages.py 50 52 64 33 > gpurun_out/r06/gram_stages_ab2.jsonl"
