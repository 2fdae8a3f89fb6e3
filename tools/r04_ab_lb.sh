#!/bin/bash
# Row-set weighted sum with two clients' loads in flight: row-set and
# golden parity, the layout-B probe, the bench line.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_rows.py tests/test_gpu_golden.py tests/test_gpu_server.py tests/test_gpu_world2.py -q --timeout 200 --timeout-method thread > gpurun_out/rows.log 2>&1" \
  "timeout -k 10 200 python -u tools/probe_layout_b.py > gpurun_out/layout_b.jsonl" \
  "timeout -k 10 200 python -u tools/probe_layout_b.py >> gpurun_out/layout_b.jsonl" \
  bench
