#!/bin/bash
# secret-sharing recovery with eight share rows in flight and NT loads
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 400 python -u -m pytest tests/test_gpu_wire.py -x -q --timeout 120 --timeout-method thread" \
  "timeout -k 10 300 python tools/bench_wire.py ss > gpurun_out/ss8.jsonl"
