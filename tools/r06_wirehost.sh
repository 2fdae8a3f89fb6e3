#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
bash tools/gpu_job.sh \
  "timeout -k 10 400 python tools/prof_wire_host.py > gpurun_out/r06/prof_wire_host.txt 2>&1"
