#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
bash tools/gpu_job.sh \
  "timeout -k 10 300 python tools/time_krum_devsel.py > gpurun_out/r06/krum_devsel_warm5.txt 2>&1"
