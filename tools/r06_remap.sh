#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
bash tools/gpu_job.sh \
  "timeout -k 10 400 python tools/ab_os_remap.py > gpurun_out/r06/os_remap_ab.jsonl"
