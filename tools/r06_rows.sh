#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 500 python -u -m pytest tests/test_gpu_rows.py tests/test_gpu_golden.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06/rows_tests.log 2>&1" \
  "timeout -k 10 400 python tools/probe_layout_b.py > gpurun_out/r06/layout_b_batched.jsonl"
