#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
P=/tmp/r06sq
bash tools/gpu_job.sh \
  "timeout -k 10 600 python -u -m pytest tests/ -m gpu -k 'norm' -x -q --timeout 120 --timeout-method thread > gpurun_out/r06/sqnorm_tests.log 2>&1" \
  "timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P -o run --output-format csv -- python tools/bench_robust.py dropin > gpurun_out/r06/dropin_sqnorm.jsonl"
find $P -name '*kernel_stats.csv' -exec cp {} gpurun_out/r06/dropin_sqnorm_kernel_stats.csv \;
