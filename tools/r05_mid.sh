#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_job.sh pytestall smoke \
  "timeout -k 10 400 python -u bench.py --e2e > gpurun_out/bench.jsonl" \
  "timeout -k 10 300 python -u tools/bench_share.py --aggregate --world 8 > gpurun_out/share_agg.jsonl" \
  "timeout -k 10 300 python -u tools/bench_robust.py dropin > gpurun_out/dropin.jsonl" \
  "timeout -k 10 200 python -u tools/profile_rule.py layout_b > gpurun_out/prof_layout_b.txt"
