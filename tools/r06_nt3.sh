#!/bin/bash
# non-temporal stage loads as the default (stages 1) against plain loads
# (stages 4): the Gram tests, then interleaved A/Bs for the compact (n <= 64)
# and full-tile (65-112) forms
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 600 python -u -m pytest tests/test_gpu_pairgram.py tests/test_gpu_krumsel.py -x -q --timeout 120 --timeout-method thread" \
  "KNOB=stages MODES=1,4 ROUNDS=8 timeout -k 10 500 python tools/ab_gram_stages.py 50 40 64 66 100 112 > gpurun_out/gram_nt_ab4.jsonl"
