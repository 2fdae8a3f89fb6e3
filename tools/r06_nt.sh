#!/bin/bash
# A/B: the Gram main pass's compact stages with non-temporal LDS loads
# (stages 4) against the default (1); the stages test over modes 0-4 first
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_pairgram.py -k compact_stages -x -q --timeout 120 --timeout-method thread" \
  "KNOB=stages MODES=4,1 timeout -k 10 300 python tools/ab_gram_stages.py 40 50 64 > gpurun_out/gram_nt_ab.jsonl" \
  "KNOB=stages MODES=1,4 timeout -k 10 300 python tools/ab_gram_stages.py 50 33 > gpurun_out/gram_nt_ab2.jsonl"
