#!/bin/bash
# Gram path: parity (stress families logged, n up to 208), C4 in both
# placements, the Gram timing and kernel trace, and the robust-bench Krum
# lines at n = 50 (C4), 100 and 200.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "FSAGG_TEST_LOG=gpurun_out/stress.jsonl timeout -k 10 400 python -u -m pytest tests/test_gpu_pairgram.py -q --timeout 200 --timeout-method thread > gpurun_out/pairgram.log 2>&1" \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 250 --timeout-method thread -k c4 > gpurun_out/c4.log 2>&1" \
  "timeout -k 10 200 python -u tools/probe_gram_data.py > gpurun_out/gram_ab_staged.jsonl" \
  "timeout -k 10 400 python -u tools/bench_robust.py krum krum_large > gpurun_out/robust_krum.jsonl" \
  "timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_krum -o run --output-format csv -- python tools/bench_robust.py krum krum_large"
