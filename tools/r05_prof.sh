#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 200 python -u tools/profile_rule.py krum > gpurun_out/prof_krum.txt" \
  "timeout -k 10 200 python -u tools/profile_rule.py layout_b > gpurun_out/prof_layout_b.txt" \
  "timeout -k 10 200 python -u tools/profile_rule.py fedavg > gpurun_out/prof_fedavg.txt" \
  "timeout -k 10 200 python -u tools/time_share_host.py --views 1 > gpurun_out/share_host_views.txt"
