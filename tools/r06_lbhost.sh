#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
bash tools/gpu_job.sh \
  "timeout -k 10 300 python tools/probe_layout_b_host.py > gpurun_out/r06/layout_b_host.jsonl 2> gpurun_out/r06/layout_b_host_prof.txt"
