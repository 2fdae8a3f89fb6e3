#!/bin/bash
# fp32 k-step sums in the compact Gram pass: tests + A/B; weighted-sum V sweep
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
: > gpurun_out/r06/tune_wsum_sizes.txt
steps=(
  "timeout -k 10 400 python -u -m pytest tests/test_gpu_pairgram.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06/pairgram_tests_sum32.log 2>&1"
  "KNOB=sum32 CHUNKS=1,2,4 timeout -k 10 300 python tools/ab_gram_chunks.py 50 33 64 > gpurun_out/r06/gram_sum32_ab.jsonl"
)
for P in 8000000 12000000 15000000 18000000 20000000 23520848 25000000 28000000 32000000; do
  steps+=("echo P=$P >> gpurun_out/r06/tune_wsum_sizes.txt && P=$P VARS=3,9,5,11 GRIDS=0 PVARS= NOREAD=1 ROUNDS=9 timeout -k 10 200 python tools/tune_wsum.py >> gpurun_out/r06/tune_wsum_sizes.txt")
done
bash tools/gpu_job.sh "${steps[@]}"
