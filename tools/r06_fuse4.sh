#!/bin/bash
# the fused B-local pass's tests over the pipeline's row counts
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 400 python -u -m pytest tests/test_gpu_wire.py -x -q -k 'fused or dissim' --timeout 120 --timeout-method thread"
