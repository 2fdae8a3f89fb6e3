#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
bash tools/gpu_job.sh \
  "timeout -k 10 300 python tools/prof_median_host.py > gpurun_out/r06/median_host_marks.txt 2>&1"
