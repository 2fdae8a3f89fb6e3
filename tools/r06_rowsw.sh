#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
bash tools/gpu_job.sh \
  "timeout -k 10 400 python tools/ab_rows_width.py > gpurun_out/r06/rows_width_ab.jsonl"
