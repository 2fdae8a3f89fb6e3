#!/bin/bash
# Two-wave order statistics: parity tests, then the interleaved A/B sweep.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_orderstat_pair.py tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k 'pair or median_trimmed or refinement or nonfinite'" \
  "timeout -k 10 300 python -u tools/bench_pair.py > gpurun_out/pair_ab.jsonl"
