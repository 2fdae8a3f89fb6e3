#!/bin/bash
# Certified Krum selection on the Gram path: pairgram parity (stress
# families logged), the C4 full-size test in both row placements, the peer
# assembly through aggregate(), and the Gram timing + kernel trace.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "FSAGG_TEST_LOG=gpurun_out/stress.jsonl timeout -k 10 300 python -u -m pytest tests/test_gpu_pairgram.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pairgram.log 2>&1" \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 250 --timeout-method thread -k c4 > gpurun_out/c4.log 2>&1" \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_world2.py -x -q --timeout 200 --timeout-method thread -k 'peer_assembly_aggregate or lost_rank' > gpurun_out/world2.log 2>&1" \
  "timeout -k 10 200 python -u tools/probe_gram_data.py > gpurun_out/gram_ab_staged.jsonl" \
  "timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gram -o run -- python tools/probe_gram_data.py"
