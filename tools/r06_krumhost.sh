#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 300 python tools/time_krum_phases.py > gpurun_out/r06/krum_phases.txt 2>&1" \
  "FRESH=1 timeout -k 10 300 python tools/time_krum_phases.py > gpurun_out/r06/krum_phases_fresh.txt 2>&1"
