#!/bin/bash
# Gram path: parity (stress families logged), C4 in both placements, the
# Gram timing, its kernel trace and the C4 robust-bench Krum line.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "FSAGG_TEST_LOG=gpurun_out/stress.jsonl timeout -k 10 300 python -u -m pytest tests/test_gpu_pairgram.py -q --timeout 200 --timeout-method thread > gpurun_out/pairgram.log 2>&1" \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 250 --timeout-method thread -k c4 > gpurun_out/c4.log 2>&1" \
  "timeout -k 10 200 python -u tools/probe_gram_data.py > gpurun_out/gram_ab_staged.jsonl" \
  "timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gram -o run --output-format csv -- python tools/probe_gram_data.py" \
  "timeout -k 10 300 python -u tools/bench_robust.py krum > gpurun_out/robust_krum.jsonl"
