#!/bin/bash
# Row-set tests incl. back-to-back aggregate() calls without host sync.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_rows.py -q --timeout 200 --timeout-method thread > gpurun_out/rows.log 2>&1"
