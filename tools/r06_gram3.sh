#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_pairgram.py -x -q --timeout 120 --timeout-method thread -k 'compact or settings' > gpurun_out/r06/pairgram_tests3.log 2>&1" \
  "timeout -k 10 300 python tools/ab_gram_stages.py 50 52 33 > gpurun_out/r06/gram_stages_ab3.jsonl" \
  "CHUNKS=1024,512,768,384 timeout -k 10 300 python tools/ab_gram_chunks.py 50 > gpurun_out/r06/gram_chunks_ab.jsonl"
