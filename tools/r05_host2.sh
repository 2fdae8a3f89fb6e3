#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_job.sh pytestall \
  "timeout -k 10 180 ./tools/probe/bin/valu_probe3 > gpurun_out/valu3.txt" \
  "timeout -k 10 300 python -u tools/bench_share.py --aggregate --world 8 > gpurun_out/share_agg.jsonl" \
  "timeout -k 10 200 python -u tools/time_share_host.py --views 1 > gpurun_out/share_host_views.txt"
bash tools/gpu_job.sh "timeout -k 10 300 python -u tools/bench_robust.py dropin > gpurun_out/dropin.jsonl"
