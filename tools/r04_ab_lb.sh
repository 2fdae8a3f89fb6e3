#!/bin/bash
# Gram parity at every tile count.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_pairgram.py -q --timeout 200 --timeout-method thread > gpurun_out/pairgram.log 2>&1"
