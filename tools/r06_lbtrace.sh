#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/prof_lb -o run --output-format csv -- python tools/probe_layout_b.py --only agg_views,rows_views > gpurun_out/r06/layout_b_trace.jsonl"
