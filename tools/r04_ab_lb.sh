#!/bin/bash
# Gram plans from one wave per pass: parity (pairgram, C4, sharded Krum)
# and the chain's kernel trace.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_pairgram.py tests/test_gpu_fullsize.py -k 'pairgram or krum or c4' -q --timeout 250 --timeout-method thread > gpurun_out/pairgram.log 2>&1" \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_world2.py -q -k 'sharded or peer_assembly_aggregate' --timeout 250 --timeout-method thread > gpurun_out/world2.log 2>&1" \
  "timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gram -o run --output-format csv -- python tools/probe_gram_data.py"
