#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
bash tools/gpu_job.sh \
  "MODES=3,1 timeout -k 10 300 python tools/ab_gram_stages.py 50 50 50 40 > gpurun_out/r06/gram_prio_ab2.jsonl"
