#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 600 python -u -m pytest tests/test_gpu_pairgram.py -k 'compact or fused' -x -q --timeout 120 --timeout-method thread > gpurun_out/r06/early_tests.log 2>&1" \
  "MODES=4,1 timeout -k 10 300 python tools/ab_gram_stages.py 33 50 50 64 > gpurun_out/r06/gram_wave_ab.jsonl"
