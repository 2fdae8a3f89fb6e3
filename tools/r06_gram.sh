#!/bin/bash
# Gram stages A/B + the pairgram tests + the Krum chain under a kernel trace.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_pairgram.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06/pairgram_tests.log 2>&1" \
  "timeout -k 10 300 python tools/ab_gram_stages.py 50 52 64 100 > gpurun_out/r06/gram_stages_ab.jsonl" \
  "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/prof_krum2 -o run --output-format csv -- python tools/bench_robust.py krum > gpurun_out/r06/krum_traced.jsonl"
