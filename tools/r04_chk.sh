#!/bin/bash
# Drop-in rules and C5 order statistics (regression check), layout B with
# the 1-MiB pinned ring.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_rows.py tests/test_gpu_golden.py -q -x --timeout 200 --timeout-method thread > gpurun_out/rows.log 2>&1" \
  "timeout -k 10 300 python -u tools/bench_robust.py dropin orderstat > gpurun_out/robust_a.jsonl" \
  "timeout -k 10 200 python -u tools/probe_layout_b.py > gpurun_out/layout_b.jsonl" \
  "cd tools/probe/r3/tree && timeout -k 10 300 python -u tools/bench_robust.py dropin > ../../../../gpurun_out/robust_r3.jsonl" \
  "timeout -k 10 300 python -u tools/bench_robust.py dropin > gpurun_out/robust_b.jsonl" \
  "timeout -k 10 200 python -u tools/probe_layout_b.py >> gpurun_out/layout_b.jsonl" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dropin -o run --output-format csv -- python tools/bench_robust.py dropin"
