#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
bash tools/gpu_job.sh \
  "timeout -k 10 300 python tools/time_stage.py > gpurun_out/r06/time_stage.txt 2>&1"
