#!/bin/bash
# Round-4 full GPU pass: the MFMA rounding probe (raw products, k-step
# error per data family, the alignment window), pytest -m gpu, smoke, bench.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "timeout -k 10 200 python -u tools/probe/mfma_numerics.py raw kstep > gpurun_out/mfma_numerics.jsonl" \
  "timeout -k 10 200 python -u tools/probe/mfma_numerics.py window > gpurun_out/mfma_window.jsonl" \
  pytestall smoke bench
