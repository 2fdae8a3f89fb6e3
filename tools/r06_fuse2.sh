#!/bin/bash
# the metric tests after the fused-pass test fix
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 400 python -u -m pytest tests/test_gpu_wire.py -x -q --timeout 120 --timeout-method thread"
