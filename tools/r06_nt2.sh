#!/bin/bash
# longer interleaved A/B of the non-temporal stage loads (stages 4 vs 1)
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "KNOB=stages MODES=4,1 ROUNDS=12 timeout -k 10 400 python tools/ab_gram_stages.py 50 40 64 50 > gpurun_out/gram_nt_ab3.jsonl"
