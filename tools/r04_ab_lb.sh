#!/bin/bash
# Host-table uploads on a side stream: every GPU test, the layout-B probe,
# its kernel trace, and the bench line (plugin surfaces).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_job.sh pytestall \
  "timeout -k 10 200 python -u tools/probe_layout_b.py > gpurun_out/layout_b.jsonl" \
  "timeout -k 10 200 python -u tools/probe_layout_b.py >> gpurun_out/layout_b.jsonl" \
  "timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lb -o run --output-format csv -- python tools/probe_layout_b.py --rounds 2" \
  bench
